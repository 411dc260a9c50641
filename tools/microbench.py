#!/usr/bin/env python3
"""Kernel microbenchmarks (one kernel class at a time, nothing overlapping).

  python tools/microbench.py pyr   --width 3840 --height 2160 --reps 200
  python tools/microbench.py track --width 1920 --height 1080 --features 5000 --reps 200

pyr:   builds pyramids of resident frames back to back on one stream.
track: tracks the same feature set between the same two resident pyramids,
       restoring the feature arrays before each launch.
Prints one JSON line with per-launch averages from HIP events, and is meant to
run under `rocprofv3 --kernel-trace --stats` or `--pmc` as well.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["pyr", "track", "frames", "api", "apiseq"])
    ap.add_argument("--prof", action="store_true",
                    help="per-wave phase cycles (needs KLT_AMD_LIB=.../lib/prof/libklt_amd.so)")
    ap.add_argument("--overlap", action="store_true", help="frames: pyramids of chunk c+1 on a second stream")
    ap.add_argument("--no-patch", action="store_true", help="tracker: per-pixel gathers only")
    ap.add_argument("--input-order", action="store_true", help="tracker: no band ordering")
    ap.add_argument("--no-merge", action="store_true", help="tracker: residue passes of their own")
    ap.add_argument("--table", action="store_true", help="frames: write the feature table (as bench.py does)")
    ap.add_argument("--chunk", type=int, default=16, help="frames: frames per batch")
    ap.add_argument("--pyr-only", action="store_true", help="frames: build the batched pyramids, track nothing")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--features", type=int, default=5000)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--reduction", choices=["exact", "fast"], default="exact")
    ap.add_argument("--no-table", action="store_true", help="apiseq: no feature table")
    ap.add_argument("--count", action="store_true", help="frames: count Newton iterations / passes of the timed rep")
    ap.add_argument("--host-threads", type=int, default=-1, help="apiseq: host pool workers (-1: default)")
    ap.add_argument("--generic", action="store_true")
    ap.add_argument("--max-it", type=int, default=0, help="tracker: override max_iterations")
    ap.add_argument("--lost", action="store_true", help="tracker: mark every feature lost (launch floor)")
    ap.add_argument("--window", type=int, default=0, help="tracker: override window width/height")
    ap.add_argument("--impl", type=int, default=0, help="tracker kernel for the default configuration: "
                                                        "0 track7.hip, 1 generic k_track_frames_g")
    a = ap.parse_args()

    import kltamd
    from kltamd.device import D2D, H2D, PyrDesc, Timing, TrackDesc, check

    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    W, H = a.width, a.height
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    lib.klt_amd_set_reduction(tc, 0 if a.reduction == "exact" else 1)
    ctx = lib.klt_amd_device_context(tc)
    lib.klt_hip_set_path(ctx, 1 if a.generic else 0)
    check(lib, ctx, lib.klt_hip_set_track_order(ctx, 1 if a.input_order else 0), "order")
    check(lib, ctx, lib.klt_hip_set_track_merge(ctx, 0 if a.no_merge else 1), "merge")
    check(lib, ctx, lib.klt_hip_set_track_patch(ctx, 0 if a.no_patch else 1), "patch")
    check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 1 if a.overlap else 0), "overlap")
    check(lib, ctx, lib.klt_hip_set_track_impl(ctx, a.impl), "impl")
    if a.host_threads >= 0:
        check(lib, ctx, lib.klt_hip_set_host_threads(ctx, a.host_threads), "host_threads")
    nf = max(a.frames, 2)
    frames = lib.klt_hip_malloc(ctx, nf * W * H)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, 1080, 0, nf, W, H, frames, W, W * H), "synth")
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    if a.max_it:
        tc.contents.max_iterations = a.max_it
    if a.window:
        tc.contents.window_width = tc.contents.window_height = a.window
    lib.klt_amd_track_desc(tc, C.byref(td))
    out = {"mode": a.mode, "resolution": f"{W}x{H}", "reps": a.reps}

    def build(slot, t):
        check(lib, ctx, lib.klt_hip_build_pyramid(ctx, slot, C.byref(pd), C.c_void_p(frames + (t % nf) * W * H),
                                                  W, 0), "build")

    if a.mode == "pyr":
        for t in range(10):
            build(t % 2, t)
        lib.klt_hip_sync(ctx)
        lib.klt_hip_set_timing(ctx, 1)
        t0 = time.perf_counter()
        for t in range(a.reps):
            build(t % 2, t)
        lib.klt_hip_sync(ctx)
        wall = time.perf_counter() - t0
        tm = Timing()
        check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
        l0 = 1e3 * tm.ms_pyr_l0 / max(tm.n_pyr_l0, 1)
        l1 = 1e3 * tm.ms_pyr_l1 / max(tm.n_pyr_l1, 1)
        gen = 1e3 * tm.ms_generic / max(tm.n_generic, 1)
        px = W * H
        byts = px * 13 + (W // 4) * (H // 4) * 12
        pass_us = gen if a.generic else l0 + l1
        out.update({"k_pyr_l0_us": l0, "k_pyr_l1_us": l1, "generic_us": gen, "wall_us_per_frame": 1e6 * wall / a.reps,
                    "pass_GBps": byts / (pass_us * 1e-6) / 1e9, "frac_8TBs": byts / (pass_us * 1e-6) / 8e12,
                    "gpix_s": px / (pass_us * 1e-6) / 1e9})
    elif a.mode == "api":
        # the public klt.h path: host u8 frames, KLTTrackFeatures per frame (PCIe inclusive)
        nh = max(a.frames, 3)
        host = []
        for t in range(nh):
            h = np.empty((H, W), np.uint8)
            lib.klt_synth_frame(1080, t, W, H, h.ctypes.data)
            host.append(h)
        u8 = lambda z: z.ctypes.data_as(kltamd.abi.U8P)  # noqa: E731
        fl = lib.KLTCreateFeatureList(a.features)
        lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
        lib.KLTTrackFeatures(tc, u8(host[0]), u8(host[1]), W, H, fl)  # first call builds both pyramids
        times = []
        for t in range(2, nh):
            t0 = time.perf_counter()
            lib.KLTTrackFeatures(tc, u8(host[t - 1]), u8(host[t]), W, H, fl)
            times.append(time.perf_counter() - t0)
        live = sum(1 for k in range(a.features) if fl.contents.feature[k].contents.val >= 0)
        lib.KLTFreeFeatureList(fl)
        out.update({"features": a.features, "calls": len(times), "fps": len(times) / sum(times),
                    "us_per_call_median": 1e6 * float(np.median(times)), "live_at_end": live})
    elif a.mode == "apiseq":
        # KLTTrackSequence: host u8 frames, uploads overlapped with the batched device path
        nh = max(a.frames, 3)
        host = []
        for t in range(nh):
            h = np.empty((H, W), np.uint8)
            lib.klt_synth_frame(1080, t, W, H, h.ctypes.data)
            host.append(h)
        u8 = lambda z: z.ctypes.data_as(kltamd.abi.U8P)  # noqa: E731
        arr = (kltamd.abi.U8P * nh)(*[u8(z) for z in host])
        fl = lib.KLTCreateFeatureList(a.features)
        lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
        ft = lib.KLTCreateFeatureTable(nh - 1, a.features)
        for rep in range(a.reps if a.reps < 50 else 3):  # apiseq: --reps below 50 sets the call count
            fl = lib.KLTCreateFeatureList(a.features)
            lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
            t0 = time.perf_counter()
            lib.KLTTrackSequence(tc, arr, nh, W, H, fl, ft if not a.no_table else None, 0)
            dt = time.perf_counter() - t0
            print(f"apiseq rep {rep}: {(nh - 1) / dt:.0f} fps", file=sys.stderr, flush=True)
            live = sum(1 for k in range(a.features) if fl.contents.feature[k].contents.val >= 0)
            lib.KLTFreeFeatureList(fl)
        lib.KLTFreeFeatureTable(ft)
        out.update({"features": a.features, "frames_tracked": nh - 1, "fps": (nh - 1) / dt,
                    "us_per_frame": 1e6 * dt / (nh - 1), "live_at_end": live,
                    "note": "host frames, PCIe upload and feature-table download included"})
    elif a.mode == "frames":
        # batched sequence: select on frame 0, track frames 1..nf-1 in chunks
        h0 = np.empty((H, W), np.uint8)
        lib.klt_synth_frame(1080, 0, W, H, h0.ctypes.data)
        fl = lib.KLTCreateFeatureList(a.features)
        lib.KLTSelectGoodFeatures(tc, h0.ctypes.data_as(kltamd.abi.U8P), W, H, fl)
        n = a.features
        xs = np.array([fl.contents.feature[k].contents.x for k in range(n)], np.float32)
        ys = np.array([fl.contents.feature[k].contents.y for k in range(n)], np.float32)
        vs = np.array([fl.contents.feature[k].contents.val for k in range(n)], np.int32)
        lib.KLTFreeFeatureList(fl)
        d = [lib.klt_hip_malloc(ctx, 4 * n) for _ in range(3)]
        d0 = [lib.klt_hip_malloc(ctx, 4 * n) for _ in range(3)]
        for dd, arr in zip(d0, (xs, ys, vs)):
            check(lib, ctx, lib.klt_hip_memcpy(ctx, dd, arr.ctypes.data, arr.nbytes, H2D), "h2d")
        for dd, ss in zip(d, d0):
            check(lib, ctx, lib.klt_hip_memcpy(ctx, dd, ss, 4 * n, D2D), "d2d")
        check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(frames), W), "begin")
        T = nf - 1
        warm = min(T, 2 * a.chunk)
        check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(frames + W * H), W,
                                                 W * H, warm, a.chunk, d[0], d[1], d[2], n, None, None, None,
                                                 0), "warm")
        if a.pyr_only:
            n = 0

        tab = [lib.klt_hip_malloc(ctx, 4 * max(n, 1) * T) for _ in range(3)] if a.table else [None] * 3

        def rep():
            # restart from the seed frame and the selected features
            for dd, ss in zip(d, d0):
                check(lib, ctx, lib.klt_hip_memcpy(ctx, dd, ss, 4 * n, D2D), "d2d")
            check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(frames), W), "begin")
            check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(frames + W * H),
                                                     W, W * H, T, a.chunk, d[0], d[1], d[2], n, tab[0], tab[1],
                                                     tab[2], n if a.table else 0), "frames")

        lib.klt_hip_sync(ctx)
        t0 = time.perf_counter()
        for r in range(a.reps):
            rep()
        lib.klt_hip_sync(ctx)
        wall = time.perf_counter() - t0
        done = a.reps * T
        lib.klt_hip_set_timing(ctx, 1)  # one more pass with per-launch events
        pbuf = None
        if a.prof:
            nslot = (n + 64) * 12
            pbuf = lib.klt_hip_malloc(ctx, 8 * nslot)
            check(lib, ctx, lib.klt_hip_memcpy(ctx, pbuf, np.zeros(nslot, np.uint64).ctypes.data, 8 * nslot, H2D),
                  "zero")
            lib.klt_hip_set_prof(ctx, pbuf)
        if a.count:
            check(lib, ctx, lib.klt_hip_set_track_count(ctx, 1), "count")
        rep()
        if a.count:
            solves, passes = C.c_ulonglong(0), C.c_ulonglong(0)
            check(lib, ctx, lib.klt_hip_get_track_count(ctx, C.byref(solves), C.byref(passes), 0), "count")
            out["newton_iterations"], out["gather_passes"] = solves.value, passes.value
        if a.prof:
            lib.klt_hip_sync(ctx)
            pr = np.empty(nslot, np.uint64)
            check(lib, ctx, lib.klt_hip_memcpy(ctx, pr.ctypes.data, pbuf, 8 * nslot, 2), "prof")
            pr = pr.reshape(-1, 12).astype(np.float64)
            pr = pr[pr[:, 4] > 0]  # waves that ran frames
            names = ["gather_interp", "sums", "solve", "residue", "frame", "iterations", "passes", "wall_ticks",
                     "-", "-", "levels", "pass_top"]
            # accumulated over the timed rep's launches (last launch overwrites per slot): per wave per frame
            fr = a.chunk
            out["prof_cycles_per_wave_frame"] = {nm: float(pr[:, k].mean() / fr) for k, nm in enumerate(names)
                                                 if nm != "-"}
            out["prof_cycles_per_wave_frame"].pop("wall_ticks")
            out["prof_waves"] = int(pr.shape[0])
            rate = C.c_int(0)
            # wall_clock64 runs at hipDeviceAttributeWallClockRate kHz (100 MHz on MI300-class parts)
            out["prof_clock64_ghz"] = float(pr[:, 4].sum() / (pr[:, 7].sum() / 100e6) / 1e9)
            out["prof_wave_life_us"] = float(pr[:, 7].mean() / 100.0)
            st = (pr[:, 8] - pr[:, 8].min()) / 100.0
            en = (pr[:, 9] - pr[:, 8].min()) / 100.0
            out["prof_start_us_pct"] = [float(np.percentile(st, q)) for q in (0, 25, 50, 75, 90, 100)]
            out["prof_end_us_pct"] = [float(np.percentile(en, q)) for q in (0, 25, 50, 75, 90, 100)]
        tm = Timing()
        check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
        vv = np.empty(n, np.int32)
        check(lib, ctx, lib.klt_hip_memcpy(ctx, vv.ctypes.data, d[2], 4 * n, 2), "d2h")
        out.update({"features": n, "chunk": a.chunk, "frames": done, "fps_wall": done / wall,
                    "us_per_frame_wall": 1e6 * wall / done,
                    "l0_us_per_frame": 1e3 * tm.ms_pyr_l0 / max(tm.frames_pyr_l0, 1),
                    "l1_us_per_frame": 1e3 * tm.ms_pyr_l1 / max(tm.frames_pyr_l1, 1),
                    "track_us_per_frame": 1e3 * tm.ms_track / max(tm.frames_track, 1),
                    "status_hist": {int(k): int(c) for k, c in zip(*np.unique(vv, return_counts=True))}})
    else:
        h0 = np.empty((H, W), np.uint8)
        lib.klt_synth_frame(1080, 0, W, H, h0.ctypes.data)
        fl = lib.KLTCreateFeatureList(a.features)
        lib.KLTSelectGoodFeatures(tc, h0.ctypes.data_as(kltamd.abi.U8P), W, H, fl)
        n = a.features
        xs = np.array([fl.contents.feature[k].contents.x for k in range(n)], np.float32)
        ys = np.array([fl.contents.feature[k].contents.y for k in range(n)], np.float32)
        vs = np.array([fl.contents.feature[k].contents.val for k in range(n)], np.int32)
        lib.KLTFreeFeatureList(fl)
        if a.lost:
            vs[:] = -1
        build(0, 0)
        build(1, 1)
        st = [lib.klt_hip_malloc(ctx, 4 * n) for _ in range(3)]
        wk = [lib.klt_hip_malloc(ctx, 4 * n) for _ in range(3)]
        for d, arr in zip(st, (xs, ys, vs)):
            check(lib, ctx, lib.klt_hip_memcpy(ctx, d, arr.ctypes.data, arr.nbytes, H2D), "h2d")

        def once():
            for d, s in zip(wk, st):
                check(lib, ctx, lib.klt_hip_memcpy(ctx, d, s, 4 * n, D2D), "d2d")
            check(lib, ctx, lib.klt_hip_track(ctx, 0, 1, C.byref(td), wk[0], wk[1], wk[2], n, 1), "track")

        for _ in range(5):
            once()
        lib.klt_hip_sync(ctx)
        lib.klt_hip_set_timing(ctx, 1)
        for _ in range(a.reps):
            once()
        tm = Timing()
        check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
        vv = np.empty(n, np.int32)
        check(lib, ctx, lib.klt_hip_memcpy(ctx, vv.ctypes.data, wk[2], 4 * n, 2), "d2h")
        out.update({"features": n, "k_track_us": 1e3 * tm.ms_track / max(tm.n_track, 1),
                    "status_hist": {int(k): int(c) for k, c in zip(*np.unique(vv, return_counts=True))}})
    print(json.dumps(out), flush=True)
    lib.KLTFreeTrackingContext(tc)


if __name__ == "__main__":
    main()
