#!/usr/bin/env python3
"""The REPLACE harness (example3.c with REPLACE) at 1080p/5000 for a few
frames, to read the selection engine's timeline (KLT_SEL_TRACE=1) and the
per-replace wall clock.  usage: KLT_SEL_TRACE=1 python tools/exp/replace_probe.py [frames]"""
import ctypes as C
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import kltamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
W, H, NF = 1920, 1080, 5000
lib = kltamd.load()
lib.KLTSetVerbosity(0)
host = []
for t in range(n + 1):
    f = np.empty((H, W), np.uint8)
    lib.klt_synth_frame(1080, t, W, H, f.ctypes.data)
    host.append(f)
u8 = lambda a: a.ctypes.data_as(C.POINTER(C.c_ubyte))  # noqa: E731
tc = lib.KLTCreateTrackingContext()
tc.contents.sequentialMode = 1
fl = lib.KLTCreateFeatureList(NF)
lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
rep = []
for t in range(1, n + 1):
    lib.KLTTrackFeatures(tc, u8(host[t - 1]), u8(host[t]), W, H, fl)
    print(f"frame {t}", file=sys.stderr, flush=True)
    a = time.perf_counter()
    lib.KLTReplaceLostFeatures(tc, u8(host[t]), W, H, fl)
    rep.append(1e6 * (time.perf_counter() - a))
print("replace us per call:", [round(r) for r in rep], "median", round(statistics.median(rep[1:])))
