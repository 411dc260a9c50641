#!/usr/bin/env python3
"""Per-call timeline of KLTTrackFeatures (example3.c's loop, 1080p/5000).

  run:     python tools/api_timeline.py run [--register] [--frames N]
           (under rocprofv3 --kernel-trace --memory-copy-trace --output-format csv)
  summary: python tools/api_timeline.py summary <dir with *_kernel_trace.csv, *_memory_copy_trace.csv>

The summary splits each steady-state call into device spans: the frame's H2D
copy (first DMA start to last DMA end), the copy-to-kernel hand-off, k_pyr_l0,
k_pyr_l1, level 1's end to the tracker's start (the feature list's copy kernel
between them), the tracker, the two copy kernels' own durations, and the gap
from the tracker's end to the next
call's copy (host side: synchronize, feature list unpack, the caller's own
work, the next call's feature pack and frame staging)."""
from __future__ import annotations

import argparse
import csv
import glob
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def run(a):
    import ctypes as C
    import kltamd
    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    W, H, NF = 1920, 1080, 5000
    host = []
    for t in range(a.frames + 1):
        f = np.empty((H, W), np.uint8)
        lib.klt_synth_frame(1080, t, W, H, f.ctypes.data)
        host.append(f)
    img1, img2 = np.empty((H, W), np.uint8), np.empty((H, W), np.uint8)
    u8 = lambda z: z.ctypes.data_as(C.POINTER(C.c_ubyte))  # noqa: E731
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    if a.register:
        for b in (img1, img2):
            assert lib.klt_amd_register_buffer(tc, b.ctypes.data_as(C.c_void_p), b.nbytes) == 0
    fl = lib.KLTCreateFeatureList(NF)
    img1[:] = host[0]
    lib.KLTSelectGoodFeatures(tc, u8(img1), W, H, fl)
    ts = []
    for t in range(1, a.frames + 1):
        img2[:] = host[t]
        t0 = time.perf_counter()
        lib.KLTTrackFeatures(tc, u8(img1), u8(img2), W, H, fl)
        ts.append(time.perf_counter() - t0)
        img1[:] = img2
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)
    print(f"median {1e6 * np.median(ts[1:]):.1f} us per call, {len(ts) / sum(ts):.0f} frames/s")


def summary(a):
    kt = [r for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
    mc = [r for f in glob.glob(f"{a.dir}/**/*memory_copy_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
    ev = []
    for r in kt:
        name = r["Kernel_Name"]
        short = next((k for k in ("k_pyr_l0", "k_pyr_l1", "k_track", "k_band_order", "k_min_eigen", "k_sel",
                                  "k_copy_words") if k in name), "other")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
    for r in mc:
        if r["Direction"].endswith("HOST_TO_DEVICE"):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "h2d"))
    ev.sort()
    # a call: the H2D copies of its frame (one DMA registered, several staged
    # groups otherwise), then its kernels
    calls, cur = [], None
    for e in ev:
        if e[2] == "h2d":
            if cur is None or "k_pyr_l0" in cur:
                cur = {"h2d": [e[0], e[1]]}
                calls.append(cur)
            else:
                cur["h2d"][1] = max(cur["h2d"][1], e[1])
        elif cur is not None:
            if e[2] == "k_copy_words":  # the feature list in (before the tracker) and out (after it)
                cur.setdefault("copies", []).append(e)
            cur.setdefault(e[2], e)
    spans = {k: [] for k in ("h2d", "handoff", "k_pyr_l0", "k_pyr_l1", "l1_to_track", "k_track", "copy_in", "copy_out",
                             "track_end_to_next_h2d", "call")}
    for i, c in enumerate(calls[2:-1], start=2):
        if not all(k in c for k in ("k_pyr_l0", "k_pyr_l1", "k_track")):
            continue
        nxt = calls[i + 1]["h2d"][0]
        spans["h2d"].append(c["h2d"][1] - c["h2d"][0])
        spans["handoff"].append(c["k_pyr_l0"][0] - c["h2d"][1])
        for k in ("k_pyr_l0", "k_pyr_l1", "k_track"):
            spans[k].append(c[k][1] - c[k][0])
        spans["l1_to_track"].append(c["k_track"][0] - c["k_pyr_l1"][1])
        cp = c.get("copies", [])
        if len(cp) >= 2:
            spans["copy_in"].append(cp[0][1] - cp[0][0])
            spans["copy_out"].append(cp[-1][1] - cp[-1][0])
        spans["track_end_to_next_h2d"].append(nxt - c["k_track"][1])
        spans["call"].append(nxt - c["h2d"][0])
    print({k: round(float(np.median(v)) / 1000, 1) for k, v in spans.items() if v}, "us (median),", len(spans["call"]), "calls")


ap = argparse.ArgumentParser()
sub = ap.add_subparsers(dest="cmd", required=True)
r = sub.add_parser("run")
r.add_argument("--register", action="store_true")
r.add_argument("--frames", type=int, default=60)
s = sub.add_parser("summary")
s.add_argument("dir")
a = ap.parse_args()
run(a) if a.cmd == "run" else summary(a)
