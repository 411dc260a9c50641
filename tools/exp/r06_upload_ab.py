#!/usr/bin/env python3
"""Per-call KLTTrackFeatures at 1080p/5000, torch-free:
host frames in pageable numpy (distinct per frame, as bench api.per_call), the
example3.c harness loop (two fixed buffers), and the same loop with the
buffers registered.  Prints one JSON line of medians (us per call) under
whatever upload environment the caller set (KLT_AMD_UPLOAD_GROUPS,
KLT_AMD_HOST_THREADS, KLT_AMD_COPY_PIECE), and whether every list equals the
first configuration's (the caller compares digests across runs).
usage: python tools/exp/r06_upload_ab.py [label] [frames]"""
import ctypes as C
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import kltamd  # noqa: E402
from kltabi import fl_to_arrays  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "run"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
W, H, NF = 1920, 1080, 5000
lib = kltamd.load()
lib.KLTSetVerbosity(0)
U8P = C.POINTER(C.c_ubyte)
u8 = lambda a: a.ctypes.data_as(U8P)  # noqa: E731
host = []
for t in range(n + 1):
    f = np.empty((H, W), np.uint8)
    lib.klt_synth_frame(1080, t, W, H, f.ctypes.data)
    host.append(f)


def digest(fl):
    h = hashlib.sha256()
    for a, dt in zip(fl_to_arrays(fl), ("<f4", "<f4", "<i4")):
        h.update(np.ascontiguousarray(a, dt).tobytes())
    return h.hexdigest()[:16]


def per_call():
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
    ts = []
    for t in range(1, n + 1):
        a = time.perf_counter()
        lib.KLTTrackFeatures(tc, u8(host[t - 1]), u8(host[t]), W, H, fl)
        ts.append(time.perf_counter() - a)
    d = digest(fl)
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)
    return ts[1:], d


def harness(register):
    img1 = np.empty((H, W), np.uint8)
    img2 = np.empty((H, W), np.uint8)
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    if register:
        for b in (img1, img2):
            assert lib.klt_amd_register_buffer(tc, b.ctypes.data_as(C.c_void_p), b.nbytes) == 0
    fl = lib.KLTCreateFeatureList(NF)
    img1[:] = host[0]
    lib.KLTSelectGoodFeatures(tc, u8(img1), W, H, fl)
    ts = []
    for t in range(1, n + 1):
        img2[:] = host[t]
        a = time.perf_counter()
        lib.KLTTrackFeatures(tc, u8(img1), u8(img2), W, H, fl)
        ts.append(time.perf_counter() - a)
        img1[:] = img2
    d = digest(fl)
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)
    return ts[1:], d


per_call()  # device context, pools, kernels warm
pc, d0 = per_call()
hv, d1 = harness(False)
rg, d2 = harness(True)
med = lambda ts: round(1e6 * float(np.median(ts)), 1)  # noqa: E731
print(json.dumps({"label": label,
                  "env": {k: os.environ.get(k) for k in ("KLT_AMD_UPLOAD_GROUPS", "KLT_AMD_HOST_THREADS",
                                                         "KLT_AMD_COPY_PIECE", "KLT_AMD_UPLOAD_PIPE", "KLT_AMD_SYNC_SPIN_US", "KLT_AMD_UPLOAD_FIRST")},
                  "us_per_call_pageable": med(pc), "us_per_call_harness": med(hv), "us_per_call_registered": med(rg),
                  "digest": d0, "lists_equal": d0 == d1 == d2}), flush=True)
