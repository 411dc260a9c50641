#!/usr/bin/env python3
"""One bench.pass_4k() measurement (the roofline_4k line: 4K pyramid pass in
BASELINE config 4's shape, and back to back) in a process of its own, so that
libraries can be A/B'd by KLT_AMD_LIB in alternating processes."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402

import bench  # noqa: E402
import kltamd  # noqa: E402

lib = kltamd.load()
lib.KLTSetVerbosity(0)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
r = bench.pass_4k(lib, dev)
print(json.dumps({"l0": r["kernels_us_per_frame"]["k_pyr_l0"], "l1": r["kernels_us_per_frame"]["k_pyr_l1"],
                  "track": r["kernels_us_per_frame"]["k_track"], "frac": r["frac"],
                  "po_l0": r["pyramids_only"]["kernels_us_per_frame"]["k_pyr_l0"],
                  "po_l1": r["pyramids_only"]["kernels_us_per_frame"]["k_pyr_l1"],
                  "po_frac": r["pyramids_only"]["frac"]}))
