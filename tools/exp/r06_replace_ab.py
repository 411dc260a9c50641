#!/usr/bin/env python3
"""REPLACE A/B: bench.py's api.replace leg alone (the
REPLACE harness at 1080p/5000, 59 frames, parity against
tests/golden/long_config3r.json), in one process, under whatever sort-pool
environment the caller set (KLT_SORT_SPIN_US, KLT_SORT_NO_CLAMP).  Prints one
JSON line: us_per_replace_median, the selection's host-sort time, parity.
usage: python tools/exp/r06_replace_ab.py OUTDIR [label]"""
import json
import os
import sys
import types
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import kltamd  # noqa: E402

label = sys.argv[2] if len(sys.argv) > 2 else "run"
W, H, NF, n = 1920, 1080, 5000, 59
lib = kltamd.load()
lib.KLTSetVerbosity(0)
host = []
for t in range(n + 1):
    f = np.empty((H, W), np.uint8)
    lib.klt_synth_frame(1080, t, W, H, f.ctypes.data)
    host.append(f)
args = types.SimpleNamespace(replace_frames=n, seed=1080)
r = bench.replace_leg(lib, host, W, H, NF, args)
sm = r["select_median"] or {}
print(json.dumps({"label": label, "env": {k: os.environ.get(k) for k in ("KLT_SORT_SPIN_US", "KLT_SORT_NO_CLAMP")},
                  "us_per_replace_median": r["us_per_replace_median"],
                  "us_downloads_and_host_sort": sm.get("us_downloads_and_host_sort"),
                  "us_device_splits": sm.get("us_device_splits"),
                  "parity_mismatched": (r.get("parity") or {}).get("columns_mismatched"),
                  "usable_cpus_hint": len(os.sched_getaffinity(0))}), flush=True)
