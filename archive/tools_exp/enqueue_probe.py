#!/usr/bin/env python3
"""Host cost of one batched klt_hip_track_frames call (the driver-shaped
timed region: 20 frames of 1080p/5000, one chunk) in this process, by how the
caller synchronizes before it and which stream the context uses.  Prints the
median enqueue time (the call's return) and the median time to drain.

usage: python archive/tools_exp/enqueue_probe.py [frames] [reps]
"""
import ctypes as C
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import kltamd  # noqa: E402
from kltamd.device import PyrDesc, TrackDesc, check, use_torch_stream  # noqa: E402


def main():
    nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    W, H, NF = 1920, 1080, 5000
    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    dev = torch.device("cuda", 0)
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    ctx = lib.klt_amd_device_context(tc)
    check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 1), "overlap")
    stream = use_torch_stream(lib, ctx, dev)
    frames = torch.empty((nfr + 2, H, W), dtype=torch.uint8, device=dev)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, 1080, 0, nfr + 2, W, H, C.c_void_p(frames.data_ptr()), W, W * H),
          "synth")
    torch.cuda.synchronize()
    f0 = frames[0].cpu().numpy()
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, f0.ctypes.data_as(C.POINTER(C.c_ubyte)), W, H, fl)
    sel = np.array([[fl.contents.feature[k].contents.x, fl.contents.feature[k].contents.y,
                     fl.contents.feature[k].contents.val] for k in range(NF)])
    lib.KLTFreeFeatureList(fl)
    x0 = torch.tensor(sel[:, 0], dtype=torch.float32, device=dev)
    y0 = torch.tensor(sel[:, 1], dtype=torch.float32, device=dev)
    v0 = torch.tensor(sel[:, 2], dtype=torch.int32, device=dev)
    x, y, v = x0.clone(), y0.clone(), v0.clone()
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, 2, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    fptr = frames.data_ptr()
    fa = (ctx, C.byref(pd), C.byref(td), C.c_void_p(fptr + W * H), W, W * H, nfr, 64, C.c_void_p(x.data_ptr()),
          C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), NF, None, None, None, 0)

    def case(name, sync):
        enq, tot = [], []
        for _ in range(reps):
            x.copy_(x0), y.copy_(y0), v.copy_(v0)
            check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fptr), W), "begin")
            sync()
            t0 = time.perf_counter()
            rc = lib.klt_hip_track_frames(*fa)
            t1 = time.perf_counter()
            sync()
            t2 = time.perf_counter()
            check(lib, ctx, rc, name)
            enq.append(1e6 * (t1 - t0))
            tot.append(1e6 * (t2 - t0))
        print(f"{name:40s} enqueue {statistics.median(enq):7.1f} us  total {statistics.median(tot):7.1f} us")

    def spin():
        while not stream.query():
            pass
        torch.cuda.synchronize()

    def idle_then_sync():
        torch.cuda.synchronize()
        time.sleep(0.002)

    def heavy_then_sync():
        # 1 ms of GPU work before the sync: the host thread sleeps in the wait
        check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fptr), W), "begin")
        for _ in range(40):
            check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fptr), W), "begin")
        torch.cuda.synchronize()

    def heavy_then_spin():
        for _ in range(41):
            check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fptr), W), "begin")
        spin()

    def sync_then_cpu_busy():
        torch.cuda.synchronize()
        t = time.perf_counter()
        while time.perf_counter() - t < 300e-6:
            pass

    def heavy_sync_then_cpu_busy():
        for _ in range(41):
            check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fptr), W), "begin")
        sync_then_cpu_busy()

    case("sync, then 300 us of host busy loop", sync_then_cpu_busy)
    case("1 ms of GPU work, sync, 300 us busy loop", heavy_sync_then_cpu_busy)
    case("1 ms of GPU work, then spin-poll + sync", heavy_then_spin)
    case("torch.cuda.synchronize", torch.cuda.synchronize)
    case("spin-poll, then torch.cuda.synchronize", spin)
    case("sync + 2 ms host sleep", idle_then_sync)
    case("1 ms of GPU work, then sync", heavy_then_sync)
    case("stream.synchronize (torch stream)", stream.synchronize)
    case("klt_hip_sync (context stream)", lambda: lib.klt_hip_sync(ctx))
    check(lib, ctx, lib.klt_hip_set_stream(ctx, None), "own stream")
    case("own stream, klt_hip_sync", lambda: lib.klt_hip_sync(ctx))
    case("own stream, torch.cuda.synchronize", torch.cuda.synchronize)
    lib.KLTFreeTrackingContext(tc)


if __name__ == "__main__":
    main()
