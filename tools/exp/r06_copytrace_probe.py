#!/usr/bin/env python3
"""rocprofv3 --memory-copy-trace reported, after
tools/seq_variance.py, "timed out after 30 seconds waiting for 573 completion
callbacks from HSA for async memory copy tracing".  Which program shapes
leave async-copy completions undelivered at exit?  Run each mode under
`rocprofv3 --kernel-trace --memory-copy-trace` and look for the timeout line.

modes:
  torch        600 pinned host->device copies by torch (no KLT library at all)
  hip          the library loaded, 600 pinned H2D copies through its own
               klt_hip_* upload path (KLTTrackFeatures per call, registered buffers)
  seq_live     3 KLTTrackSequence calls, exit with the tracking context live
  seq_freed    the same, contexts freed and the parked device contexts released
  torch_d2h    one pageable device->host copy by torch (tensor.cpu(), 400 MB)
  torch_d2h_seq  that copy, then seq_live (tools/seq_variance.py's shape)
  torch_init_seq the device initialised by torch (one tensor, no copy), then seq_live
usage: python tools/exp/r06_copytrace_probe.py MODE"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

mode = sys.argv[1]
t0 = time.perf_counter()
if mode == "torch_init_seq":
    import torch
    z = torch.zeros(16, device="cuda")
    torch.cuda.synchronize()
    mode = "seq_live"
if mode.startswith("torch_d2h"):
    import torch
    fr = torch.zeros((201, 1080, 1920), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    h = fr.cpu().numpy()
    del fr
    mode = "seq_live" if mode == "torch_d2h_seq" else "done"
if mode == "done":
    pass
elif mode == "torch":
    import torch
    src = torch.empty(2 << 20, dtype=torch.uint8).pin_memory()
    dst = torch.empty(2 << 20, dtype=torch.uint8, device="cuda")
    for _ in range(600):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
else:
    import kltamd
    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    W, H, NF, n = 1920, 1080, 1000, 41
    U8P = C.POINTER(C.c_ubyte)
    host = []
    for t in range(n):
        f = np.empty((H, W), np.uint8)
        lib.klt_synth_frame(1080, t, W, H, f.ctypes.data)
        host.append(f)
    if mode == "hip":
        tc = lib.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        fl = lib.KLTCreateFeatureList(NF)
        lib.KLTSelectGoodFeatures(tc, host[0].ctypes.data_as(U8P), W, H, fl)
        for t in range(1, n):
            lib.KLTTrackFeatures(tc, host[t - 1].ctypes.data_as(U8P), host[t].ctypes.data_as(U8P), W, H, fl)
    else:
        arr = (U8P * n)(*[h.ctypes.data_as(U8P) for h in host])
        ft = lib.KLTCreateFeatureTable(n - 1, NF)
        for k in range(3):
            tc = lib.KLTCreateTrackingContext()
            tc.contents.sequentialMode = 1
            fl = lib.KLTCreateFeatureList(NF)
            lib.KLTSelectGoodFeatures(tc, host[0].ctypes.data_as(U8P), W, H, fl)
            lib.KLTTrackSequence(tc, arr, n, W, H, fl, ft, 0)
            if mode == "seq_freed" or k < 2:
                lib.KLTFreeFeatureList(fl)
                lib.KLTFreeTrackingContext(tc)
        if mode == "seq_freed":
            lib.klt_amd_release_cached_devices()
print(f"{mode}: done in {time.perf_counter() - t0:.2f} s, exiting", flush=True)
