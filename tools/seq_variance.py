#!/usr/bin/env python3
"""KLTTrackSequence call-to-call variance (calls 2-3x slower now
and then).  One process makes --calls calls over the same 1080p/5000 host
frames and feature table (each with a fresh tracking context and selection,
as bench.py's api.sequence leg does), with KLT_SEQ_TRACE=1 so the library
prints, per call, the host time spent waiting for a staging slot's DMA,
copying frames into pinned staging, waiting for and handing out table rows.
Between calls it measures the host's memcpy bandwidth (pageable -> pageable,
400 MB) and the H2D DMA bandwidth (pinned, 256 MB), to tell a slow host or
bus from a slow library.  usage: tools/seq_variance.py OUTDIR [--calls 12]"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--calls", type=int, default=12)
    ap.add_argument("--frames", type=int, default=201)
    a = ap.parse_args()
    os.environ["KLT_SEQ_TRACE"] = "1"
    # no torch in this process: after a device->host copy in a process whose
    # device torch initialised, rocprofv3 --memory-copy-trace never receives
    # another device->host completion (tools/exp/r06_copytrace_probe.py,
    # DESIGN.md section 5), and this tool is meant to run under that trace
    import kltamd
    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    W, H, NF, n = 1920, 1080, 5000, a.frames
    U8P = C.POINTER(C.c_ubyte)
    # the frames synthesised on the host (include/klt_synth.h, the bytes k_synth writes)
    host = np.empty((n, H, W), np.uint8)
    for t in range(n):
        lib.klt_synth_frame(1080, t, W, H, host[t].ctypes.data)
    arr = (U8P * n)(*[host[t].ctypes.data_as(U8P) for t in range(n)])
    ft = lib.KLTCreateFeatureTable(n - 1, NF)
    src = np.ones(400 << 20, np.uint8)
    dst = np.empty_like(src)
    # the bus probe: a 256 MiB page-locked host buffer -> device copy through
    # the library's own context (klt_hip_register_host + klt_hip_memcpy)
    ptc = lib.KLTCreateTrackingContext()
    pctx = lib.klt_amd_device_context(ptc)
    pin = np.ones(256 << 20, np.uint8)
    assert lib.klt_hip_register_host(pctx, pin.ctypes.data, pin.nbytes) == 0
    gdst = lib.klt_hip_malloc(pctx, pin.nbytes)
    rows = []
    for k in range(a.calls):
        t0 = time.perf_counter()
        np.copyto(dst, src)
        memcpy_gbs = src.nbytes / (time.perf_counter() - t0) / 1e9
        t0 = time.perf_counter()
        assert lib.klt_hip_memcpy(pctx, gdst, pin.ctypes.data, pin.nbytes, 1) == 0
        h2d_gbs = pin.nbytes / (time.perf_counter() - t0) / 1e9
        tc = lib.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        fl = lib.KLTCreateFeatureList(NF)
        lib.KLTSelectGoodFeatures(tc, host[0].ctypes.data_as(U8P), W, H, fl)
        sys.stderr.flush()
        t0 = time.perf_counter()
        lib.KLTTrackSequence(tc, arr, n, W, H, fl, ft, 0)
        dt = time.perf_counter() - t0
        lib.KLTFreeFeatureList(fl)
        lib.KLTFreeTrackingContext(tc)
        row = {"call": k, "fps": (n - 1) / dt, "ms": 1e3 * dt, "host_memcpy_gbs_before": memcpy_gbs,
               "h2d_pinned_gbs_before": h2d_gbs}
        rows.append(row)
        print(json.dumps(row), flush=True)
    lib.KLTFreeFeatureTable(ft)
    lib.klt_hip_free(pctx, gdst)
    lib.KLTFreeTrackingContext(ptc)
    Path(a.out, "seq_variance.json").write_text(json.dumps(rows, indent=1) + "\n")


if __name__ == "__main__":
    main()
