#!/usr/bin/env python3
"""KLT hot-path benchmark (BASELINE.json: frames/sec + pyramid Gpix/s @1080p 5000 feats).

One step = one frame of sequential tracking, entirely on the device:
  build the new frame's pyramid (fused gfx950 kernels) + track every live
  feature from the previous frame's pyramid (wave64-per-feature LK),
the work KLTTrackFeatures does per call in sequential mode
(trackFeatures.c:1285-1511).  Frames are synthetic (include/klt_synth.h),
generated straight into HBM before timing; features are selected on frame 0
with KLTSelectGoodFeatures and stay device-resident.

N GPUs: one process per GPU (torchrun), each tracks its own sequence
(BASELINE config 5: "8 independent 1080p/5000-feat sequences", seed 1080+rank);
no data-path collective; value = total frames / max-over-ranks time.

Extra keys: pyramid_gpix_s, roofline (pyramid pass, HIP events on the launch
stream; measured_peak: this box's copy/fill GB/s beside the 8 TB/s spec),
roofline_4k (the same pass at 3840x2160 with 20 000 features tracked between
the launches, BASELINE config 4 on one GPU; pyramids_only: the same frames built
back to back), kernels (avg us per launch), tracker
(Newton iterations counted on the device in a separate replay,
feature-iterations/s over the tracker's own event time), cpu_baseline (the reference compiled
from its own sources, oracle/_ref, timed on this host), parity (GPU vs that
reference on the CPU sample, cell by cell), sharded_4k (every rank, at every
N: BASELINE config 4 -- 4K, 20 000 features, 1 000 frames -- with the features
sharded by row band over the N GPUs and one all-gather per 64-frame chunk;
strong scaling; the all-gather timed by HIP events in a replay; the list
checked against the reference's column digests).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

METRIC = "frames/sec + pyramid Gpix/s @1080p 5000 feats, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
REPLAY_WARMUP_S = 0.030  # untimed replays before the event-timed one (same clock state in every run shape)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--mode", choices=["sequences", "sharded"], default="sequences",
                   help="sequences: one independent sequence per GPU (configs 3/5, weak scaling); "
                        "sharded: one 4K sequence, features sharded by row band over the GPUs (config 4, "
                        "strong scaling)")
    p.add_argument("--steps", type=int, default=None, help="timed frames (default 489; sharded 490)")
    p.add_argument("--warmup", type=int, default=None, help="untimed frames (default 10; sharded 64)")
    p.add_argument("--width", type=int, default=None, help="default 1920 (sharded 3840)")
    p.add_argument("--height", type=int, default=None, help="default 1080 (sharded 2160)")
    p.add_argument("--features", type=int, default=None, help="default 5000 (sharded 20000)")
    p.add_argument("--seed", type=int, default=None, help="default 1080 (sharded 2160)")
    p.add_argument("--margin", type=int, default=64, help="sharded: level-0 rows built beyond a band")
    p.add_argument("--cpu-frames", type=int, default=160,
                   help="frames of the bounded CPU-baseline sample (rank 0, N=1)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-4k", action="store_true", help="skip the 4K legs (pass roofline, frames_4k; rank 0, N=1)")
    p.add_argument("--no-frames-4k", action="store_true",
                   help="skip the frames_4k leg (config 4 on one GPU: 1000 4K frames, device and KLTTrackSequence)")
    p.add_argument("--no-sharded-4k", action="store_true",
                   help="skip the sharded_4k leg (BASELINE config 4 sharded over the N ranks: 4K, 20 000 features, "
                        "1 000 frames, one all-gather per chunk; every rank)")
    p.add_argument("--reduction", choices=["exact", "fast"], default="exact")
    p.add_argument("--chunk", type=int, default=None,
                   help="frames per batched pyramid/track launch (klt_hip_track_frames; default 64; sharded: frames "
                        "per exchange, 64; "
                        "capped at ceil(steps / --min-chunks)); 0 = the per-frame pipelined path "
                        "(klt_hip_track_sequence)")
    p.add_argument("--replay-frames", type=int, default=489,
                   help="frames of the per-kernel event replay and the tracker-count replay (at least --steps); "
                        "they run at the production chunk (--chunk, default 64) whatever --steps caps the timed "
                        "region's chunk at")
    p.add_argument("--api-frames", type=int, default=200,
                   help="host frames for the klt.h API legs (KLTTrackFeatures per call, KLTTrackSequence); "
                        "rank 0, N=1; 0 = skip")
    p.add_argument("--no-fast", action="store_true", help="skip the fast (wave-shuffle) reduction replay")
    p.add_argument("--replace-frames", type=int, default=59,
                   help="frames of the api.replace leg (REPLACE harness, rank 0, N=1); 0 = skip")
    p.add_argument("--serial", action="store_true",
                   help="build and track on one stream; default: chunk c+1's pyramids are built on a second "
                        "stream while chunk c is tracked (they fill the CUs the tracker's last waves leave idle)")
    p.add_argument("--min-chunks", type=int, default=1,
                   help="the timed region holds at least this many chunks (the chunk is capped at "
                        "ceil(steps / min-chunks)); default 1: a region of at most --chunk frames is one launch "
                        "pair on one stream (nothing to overlap), a longer one overlaps chunk c+1's pyramids with "
                        "chunk c's tracking")
    p.add_argument("--no-device-warmup", dest="device_warmup", action="store_false",
                   help="skip the untimed, discarded >= 30 ms run of the timed schedule before the W warm-up frames "
                        "(sequences mode; the timed region then starts at the clock left by the host-side selection)")
    p.add_argument("--keep-order-cache", action="store_true", help=argparse.SUPPRESS)  # A/B hook
    p.add_argument("--event-timing", choices=["timed", "replay"], default="replay",
                   help="record per-kernel HIP events inside the timed region or in a replay")
    a = p.parse_args()
    sharded = a.mode == "sharded"
    for k, dflt, shd in (("steps", 489, 490), ("warmup", 10, 64), ("width", 1920, 3840), ("height", 1080, 2160),
                         ("features", 5000, 20000), ("seed", 1080, 2160), ("chunk", 64, 64)):
        if getattr(a, k) is None:
            setattr(a, k, shd if sharded else dflt)
    a.chunk_requested = a.chunk
    if a.chunk > 0 and a.steps > 0:
        a.chunk = min(a.chunk, max(1, -(-a.steps // max(1, a.min_chunks))))  # >= min_chunks in the timed region
    return a


def main() -> None:
    args = parse()
    # the library's per-call KLTTrackSequence stage line (stderr): the API leg
    # captures it for each timed call (api.sequence.calls_trace); read once,
    # at the process's first KLTTrackSequence
    os.environ.setdefault("KLT_SEQ_TRACE", "1")
    import torch
    import torch.distributed as dist

    import kltamd
    from kltamd.device import EXACT, FAST, PyrDesc, Timing, TrackDesc, check, use_torch_stream

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    # rehearsal only (KLT_BENCH_SHARE_GPU=1): every rank on GPU 0, gloo instead of RCCL
    share = os.environ.get("KLT_BENCH_SHARE_GPU") == "1"
    gpu_index = 0 if share else local
    torch.cuda.set_device(gpu_index)
    dev = torch.device("cuda", gpu_index)
    # a process group whenever torch.distributed.run launched us (RANK set),
    # also at N = 1: `torchrun --nproc-per-node 1 bench.py` then runs the
    # sharded_4k leg's all-gather through RCCL on one GPU
    if world > 1 or "RANK" in os.environ:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    if args.mode == "sharded":
        return run_sharded(args, world, rank, dev)

    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    W, H, NF = args.width, args.height, args.features
    # the timed region covers `steps` frames; the event and count replays cover
    # `replay` frames at the production chunk, so that the roofline and tracker
    # lines measure 64-frame launches even when --steps caps the timed chunk
    replay = max(args.steps, args.replay_frames)
    rchunk = args.chunk_requested
    nframes = 1 + args.warmup + replay
    seed = args.seed + rank

    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    lib.klt_amd_set_reduction(tc, EXACT if args.reduction == "exact" else FAST)
    ctx = lib.klt_amd_device_context(tc)
    check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 0 if args.serial else 1), "overlap")
    use_torch_stream(lib, ctx, dev)  # library kernels and torch ops ordered on one stream

    # frames straight into HBM (torch owns the memory; the library only sees pointers)
    frames = torch.empty((nframes, H, W), dtype=torch.uint8, device=dev)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, seed, 0, nframes, W, H, C.c_void_p(frames.data_ptr()),
                                             W, W * H), "synth")
    torch.cuda.synchronize()

    # selection on frame 0 through the public API
    f0 = frames[0].cpu().numpy()
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, f0.ctypes.data_as(C.POINTER(C.c_ubyte)), W, H, fl)
    sel = np.array([[fl.contents.feature[k].contents.x, fl.contents.feature[k].contents.y]
                    for k in range(NF)], np.float32)
    selv = np.array([fl.contents.feature[k].contents.val for k in range(NF)], np.int32)
    lib.KLTFreeFeatureList(fl)
    x0 = torch.from_numpy(sel[:, 0].copy()).to(dev)
    y0 = torch.from_numpy(sel[:, 1].copy()).to(dev)
    v0 = torch.from_numpy(selv.copy()).to(dev)
    x, y, v = x0.clone(), y0.clone(), v0.clone()

    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    fptr = frames.data_ptr()
    slot = C.c_int(0)
    # the harness's feature table (KLTStoreFeatureList after every frame), in HBM
    tab = [torch.empty((nframes, NF), dtype=dt, device=dev) for dt in (torch.float32, torch.float32, torch.int32)]

    def build0(t):
        if args.chunk > 0:
            check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fptr + t * W * H), W), "begin")
            return
        check(lib, ctx, lib.klt_hip_build_pyramid(ctx, 0, C.byref(pd), C.c_void_p(fptr + t * W * H), W, 0),
              "build")
        slot.value = 0

    def frames_args(t0, n, chunk):
        """klt_hip_track_frames' arguments for frames t0 .. t0+n-1 (built
        outside the timed region: the marshalling is the harness's, not the
        library's)"""
        tp = [C.c_void_p(a.data_ptr() + a.element_size() * t0 * NF) for a in tab]
        return (ctx, C.byref(pd), C.byref(td), C.c_void_p(fptr + t0 * W * H), W, W * H, n, chunk,
                C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), NF, tp[0], tp[1],
                tp[2], NF)

    def run(t0, n, chunk=None):
        chunk = args.chunk if chunk is None else chunk
        if chunk > 0:
            check(lib, ctx, lib.klt_hip_track_frames(*frames_args(t0, n, chunk)), "track_frames")
            return
        check(lib, ctx, lib.klt_hip_track_sequence(ctx, C.byref(pd), C.byref(td), C.c_void_p(fptr), W, W * H,
                                                   t0, n, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                                                   C.c_void_p(v.data_ptr()), NF, C.byref(slot)), "track_sequence")

    build0(0)
    t_start = 1 + args.warmup
    timed_events = args.event_timing == "timed"
    if args.chunk > 0:
        fa = frames_args(t_start, args.steps, args.chunk)
        timed = lambda: lib.klt_hip_track_frames(*fa)  # noqa: E731
    else:
        timed = lambda: run(t_start, args.steps) or 0  # noqa: E731
    fused = bool(lib.klt_hip_pyramid_path(ctx, slot.value) == 1) if args.chunk == 0 else bool(lib.klt_hip_fused_path(ctx, C.byref(pd)) == 1)
    # device warm-up: the timed schedule over the timed frames, from a copy of
    # the selection state, untimed and discarded, for at least
    # REPLAY_WARMUP_S, so that the timed region starts at the sustained shader
    # clock rather than the one the chip holds after the host-side selection
    # (round 5: the first ~30 ms of load run 10-17 % slower,
    # profiles/r05_timed_region_warmup.txt).  Nothing carries over: the
    # features are restored and frame 0's pyramid rebuilt, and the 1 GB of
    # frames read since leaves no timed frame in the 256 MB MALL by the time
    # the timed region reaches it.  The W warm-up frames then run as before.
    d0, dev_warm_runs = time.perf_counter(), 0
    while args.device_warmup and args.steps > 0:
        x.copy_(x0); y.copy_(y0); v.copy_(v0)
        build0(0)
        run(1, args.warmup + args.steps)
        torch.cuda.synchronize()
        dev_warm_runs += 1
        if time.perf_counter() - d0 >= REPLAY_WARMUP_S:
            break
    dev_warm_ms = 1e3 * (time.perf_counter() - d0)
    x.copy_(x0); y.copy_(y0); v.copy_(v0)
    build0(0)
    # ... and the library's cached processing order (reused by short calls
    # while it covers <= 32 tracked frames) is dropped, so that the W warm-up
    # frames and the timed region find the order state they would find with
    # no device warm-up: the warm-up leaves no state behind but the clock
    if args.device_warmup and not args.keep_order_cache:
        check(lib, ctx, lib.klt_hip_set_track_order(ctx, 0), "track order")
    # the W warm-up steps right before the timed K: the harness's own
    # bookkeeping (argument marshalling, the replay's start-state snapshot,
    # the live count) is done around them, not between them and the timed
    # region, where it left the host's launch path cold (round 4: enqueue
    # 49-53 against 14-18 us, tools/exp/r04aa.sh)
    run(1, args.warmup)
    xs, ys, vs = x.clone(), y.clone(), v.clone()
    lib.klt_hip_set_timing(ctx, 1 if timed_events else 0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    m0 = time.monotonic_ns()
    t0 = time.perf_counter()
    rc = timed()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m1 = time.monotonic_ns()
    check(lib, ctx, rc, "track_frames (timed region)")
    live_before = int((vs >= 0).sum().item())
    if world > 1:
        dist.barrier()
    live_after = int((v >= 0).sum().item())

    tm = Timing()
    exact_tab = [t[t_start - 1:t_start - 1 + args.steps].clone() for t in tab]
    if not timed_events:
        # replay from the same state with events on, on one stream, at the
        # production chunk over `replay` frames: each kernel's duration is then
        # its own (the roofline), not time shared with a kernel overlapping it
        # on the other stream, and the launches are 64-frame launches
        check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 0), "overlap")
        # a fixed warm-up first: the same replay, untimed, repeated for at least
        # REPLAY_WARMUP_S of device time, so that the timed replay follows the
        # same sustained load whatever the timed region's length (the kernels'
        # durations follow the shader clock, which the chip lowers and then
        # partly restores over the first milliseconds of pyramid load:
        # tools/clock_of.py)
        w0, warm_runs = time.perf_counter(), 0
        while True:
            x.copy_(xs); y.copy_(ys); v.copy_(vs)
            build0(t_start - 1)
            run(t_start, replay, rchunk)
            torch.cuda.synchronize()
            warm_runs += 1
            if time.perf_counter() - w0 >= REPLAY_WARMUP_S:
                break
        warm_ms = 1e3 * (time.perf_counter() - w0)
        x.copy_(xs); y.copy_(ys); v.copy_(vs)
        build0(t_start - 1)
        lib.klt_hip_set_timing(ctx, 1)
        run(t_start, replay, rchunk)
    check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
    lib.klt_hip_set_timing(ctx, 0)
    tracker = None
    if args.chunk > 0:
        # tracker work counters (Newton iterations, gather passes) in a replay
        # of their own over the same frames and chunk as the event replay, so
        # that no timed run carries the counting atomics
        x.copy_(xs); y.copy_(ys); v.copy_(vs)
        build0(t_start - 1)
        check(lib, ctx, lib.klt_hip_set_track_count(ctx, 1), "track_count")
        nrep = args.steps if timed_events else replay
        run(t_start, nrep, args.chunk if timed_events else rchunk)
        solves, passes = C.c_ulonglong(0), C.c_ulonglong(0)
        check(lib, ctx, lib.klt_hip_get_track_count(ctx, C.byref(solves), C.byref(passes), 0), "track_count")
        lib.klt_hip_set_track_count(ctx, 0)
        # feature-frames: features live when frame j starts (table row j-1 holds the list after j-1)
        ff = int((tab[2][t_start - 1:t_start - 1 + nrep] >= 0).sum().item())
        # the instance the runtime actually launched (rocprofv3's name for it), so
        # that the PMC summary below is matched to the same kernel
        tracker = tracker_line(solves.value, passes.value, ff, tm, lib.klt_hip_track_kernel(ctx).decode())
        pmc = ROOT / "profiles" / "pmc_tracker.json"
        if pmc.exists():
            try:
                d = json.loads(pmc.read_text())
                if (d.get("workload", "").startswith(f"{W}x{H}, {NF} features")
                        and tracker["kernel"] in d.get("kernel", "")):
                    # the tracker's bound is instruction issue, not HBM; its VALU
                    # instructions per iteration (PMC) set an issue ceiling beside the measured rate
                    tracker["pmc"] = {k: d[k] for k in ("per_iteration", "valu_issue_busy", "wave_time_split",
                                                        "issue_ceiling_iterations_per_s", "clock_hz_assumed")}
                    tracker["pmc"]["source"] = str(pmc.relative_to(ROOT))
                    if tracker.get("feature_iterations_per_s"):
                        tracker["frac_of_issue_ceiling"] = (tracker["feature_iterations_per_s"]
                                                            / d["issue_ceiling_iterations_per_s"])
            except Exception:
                pass

    fast = None
    if args.chunk > 0 and args.reduction == "exact" and not args.no_fast and rank == 0:
        # the same timed region with the wave-shuffle reduction (KLT_HIP_FAST):
        # its own wall clock, then a one-stream replay for the tracker's events
        fast = fast_leg(lib, ctx, td, tab, exact_tab, xs, ys, vs, x, y, v, build0, run, t_start, args)
        check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 0 if args.serial else 1), "overlap")

    dt_max = dt
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_max = float(t.item())

    us = lambda ms, n: (1000.0 * ms / n) if n else None  # noqa: E731
    # per launch (a launch covers `chunk` frames on the batched path) and per frame
    l0 = us(tm.ms_pyr_l0, tm.n_pyr_l0)
    l1 = us(tm.ms_pyr_l1, tm.n_pyr_l1)
    trk = us(tm.ms_track, tm.n_track)
    gen = us(tm.ms_generic, tm.n_generic)
    l0f = us(tm.ms_pyr_l0, tm.frames_pyr_l0)
    l1f = us(tm.ms_pyr_l1, tm.frames_pyr_l1)
    trkf = us(tm.ms_track, tm.frames_track)
    fpl = (tm.frames_pyr_l0 / tm.n_pyr_l0) if tm.n_pyr_l0 else 1.0  # frames per pyramid launch
    pass_us = (l0f or 0) + (l1f or 0) if fused else gen
    px = W * H
    W1, H1 = W // 4, H // 4
    pass_bytes = px * 13 + W1 * H1 * 12  # u8 in; img/gx/gy out at L0 and L1
    l0_bytes = px * 13 + W1 * H * 4      # k_pyr_l0: u8 in, img/gx/gy + sampled row pass out (per frame)

    result = {
        "metric": METRIC,
        "value": world * args.steps / dt_max,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * dt_max / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: include/klt_synth.h value-noise frames, (0.7,0.3) px/frame, seed {args.seed}+rank",
        "config": {"workload": f"{W}x{H}, {NF} features, sequential KLTTrackFeatures pass + KLTStoreFeatureList "
                               f"per frame, {nframes} frames per GPU (BASELINE config 3; config 5 at N>1); "
                               "device-resident: frames in HBM before timing, features and table stay on "
                               "the device (the API-inclusive figure is the `api` key)",
                   "chunk": args.chunk, "chunk_requested": args.chunk_requested,
                   "launches_timed": (-(-args.steps // args.chunk)) if args.chunk > 0 else args.steps,
                   "schedule": schedule_name(args),
                   "resolution": f"{W}x{H}", "features": NF, "frames": nframes,
                   "parallelism": "independent sequence per GPU" if world > 1 else "single GPU",
                   "reduction": args.reduction, "pyramid_path": "fused" if fused else "generic"},
        "pyramid_gpix_s": (px / (pass_us * 1e-6) / 1e9) if pass_us else None,
        "kernels_us_per_launch": {"k_pyr_l0": l0, "k_pyr_l1": l1, "k_track": trk, "generic_pass": gen},
        "kernels_us_per_frame": {"k_pyr_l0": l0f, "k_pyr_l1": l1f, "k_track": trkf},
        "replay": {"frames": replay if not timed_events else args.steps,
                   "chunk": rchunk if not timed_events else args.chunk,
                   "warmup": ({"runs": warm_runs, "ms": warm_ms,
                               "what": f"the same {replay}-frame replay, untimed, repeated for >= "
                                       f"{1e3 * REPLAY_WARMUP_S:.0f} ms right before the timed one"}
                              if not timed_events else None),
                   "what": "per-kernel HIP events and tracker counters come from replays of this length and chunk"},
        "frames_per_launch": fpl,
        "device_warmup": {"runs": dev_warm_runs, "ms": dev_warm_ms,
                          "what": f"frames 1..{args.warmup + args.steps} from the selection state on the timed "
                                  f"schedule, untimed and discarded, repeated for >= {1e3 * REPLAY_WARMUP_S:.0f} ms "
                                  "before the W warm-up frames (--no-device-warmup skips it)"},
        "live_features": {"after_warmup": live_before, "at_end": live_after},
        # host side of the timed region: the time the call took to queue its
        # launches, and CLOCK_MONOTONIC marks around the region (rocprofv3
        # kernel traces use the same clock, so launch latency can be read off)
        "timed_region_host": {"enqueue_us": 1e6 * t_enq, "monotonic_ns": [m0, m1]},
    }
    result["value_kind"] = "device_only"
    if tracker:
        result["tracker"] = tracker
    if fast:
        result["fast"] = fast
    if pass_us:
        ach = pass_bytes / (pass_us * 1e-6) / 1e9
        result["roofline"] = {
            "kernel": "pyramid pass (k_pyr_l0 + k_pyr_l1)", "bound": "hbm", "achieved": ach,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": None, "algorithmic_bytes_per_frame": pass_bytes,
            "algorithmic_bytes_per_launch": pass_bytes * fpl, "frames_per_launch": fpl,
            "us_per_frame": pass_us,
            "k_pyr_l0": {"achieved": (l0_bytes / (l0f * 1e-6) / 1e9) if l0f else None,
                         "algorithmic_bytes_per_frame": l0_bytes},
            "event_timing": "timed region" if timed_events else
                            f"replay on one stream from the timed region's start state: {replay} frames at chunk "
                            f"{rchunk} (each kernel's own duration, production launch length)",
        }
        attach_traffic(result["roofline"], ROOT / "profiles" / "pmc_latest.json", f"{W}x{H}", fpl)

    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"], result["parity"] = cpu_leg(lib, frames, W, H, NF, args, tc, ctx, dev)

    if rank == 0 and world == 1 and args.api_frames > 0:
        result["api"] = api_leg(lib, frames, W, H, NF, args)

    lib.KLTFreeTrackingContext(tc)
    del frames, tab
    if rank == 0 and world == 1 and not args.no_4k:
        result["roofline_4k"] = pass_4k(lib, dev)
        attach_traffic(result["roofline_4k"], ROOT / "profiles" / "pmc_4k_latest.json", "3840x2160",
                       result["roofline_4k"]["frames_per_launch"])
    if rank == 0 and world == 1 and not args.no_4k and not args.no_frames_4k:
        result["frames_4k"] = frames_4k_leg(lib, dev)
    if rank == 0 and world == 1:
        # the fraction also against a measured copy peak
        mp = measured_peaks(dev)
        for key in ("roofline", "roofline_4k"):
            if key in result:
                result[key]["measured_peak"] = dict(mp, frac_vs_copy=result[key]["achieved"] / mp["copy_gbs"],
                                                    frac_vs_fill=result[key]["achieved"] / mp["fill_gbs"])
    if not args.no_sharded_4k:
        # every rank: the config-4 strong-scaling leg (4K/20k, row bands, one
        # all-gather per chunk), so that the driver's --gpus N runs measure it
        sh = sharded_4k_leg(world, rank, dev, args)
        if rank == 0:
            result["sharded_4k"] = sh
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def gather_floats(vals, world, dev):
    """Every rank's list of floats (the same length on every rank), in rank order."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return [list(vals)]
    t = torch.tensor(vals, dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.to(dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def state_digest(x, y, v) -> str:
    """The column digest of tests/golden/long_config*.json: sha256(x f32 LE || y f32 LE || val i32 LE)."""
    import hashlib
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(x.cpu().numpy(), "<f4").tobytes())
    h.update(np.ascontiguousarray(y.cpu().numpy(), "<f4").tobytes())
    h.update(np.ascontiguousarray(v.cpu().numpy(), "<i4").tobytes())
    return h.hexdigest()


def sharded_core(world, rank, dev, W, H, NF, seed, warmup, steps, chunk, margin, reduction="exact", replay=True):
    """BASELINE config 4's sharded loop (trackFeatures.c:1343-1501 inside
    example3.c:54-76, features sharded over the ranks): every rank holds only
    the rows of each frame its band build reads (its band, margin and tile
    halo: kltamd.shard.BandFrames, synthesized in place of its ingest), builds
    pyramids for its row band (+margin) and tracks the features it owns; one
    all-gather of the owners' (x, y, val) slots per chunk (kltamd.shard).

    Frames 1 .. warmup are tracked untimed, frames warmup+1 .. warmup+steps
    are the timed region (barrier + synchronize on both sides, max over
    ranks).  replay: the timed frames again from the same state with HIP
    events on the tracking stream around every all-gather (the RCCL
    collective as the chunk's stream sees it) and after every exchange (chunk
    times), so the timed region itself carries no timing events.  Parity: the
    list after the warm-up, after the timed region and after the replay,
    against the reference's column digests (tests/golden/long_config4.json)
    when the workload is that sequence."""
    import torch
    import torch.distributed as dist

    import kltamd
    from kltabi import GOLDEN
    from kltamd.device import EXACT, FAST, PyrDesc, TrackDesc, check, use_torch_stream
    from kltamd.shard import BandFrames, ShardedSequence, band_of, row_edges

    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    nframes = 1 + warmup + steps
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    lib.klt_amd_set_reduction(tc, EXACT if reduction == "exact" else FAST)
    ctx = lib.klt_amd_device_context(tc)
    use_torch_stream(lib, ctx, dev)  # library kernels and torch ops ordered on one stream

    def load(t0, n, row0, nrows, dst, stride):  # this rank's ingest of rows row0 .. row0+nrows-1
        check(lib, ctx, lib.klt_hip_synth_rows(ctx, seed, t0, n, W, row0, nrows, C.c_void_p(dst), W, stride),
              "synth")

    t_setup = time.perf_counter()
    edges = row_edges(H, world, margin)  # equal level-0 rows built per rank (klt_shard_create's bands)
    frames = BandFrames(nframes, H, W, band_of(H, world, rank, margin, edges), load, dev)
    torch.cuda.synchronize()
    f0 = np.empty((H, W), np.uint8)  # frame 0 whole, for the selection every rank makes
    lib.klt_synth_frame(seed, 0, W, H, f0.ctypes.data)
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, f0.ctypes.data_as(C.POINTER(C.c_ubyte)), W, H, fl)
    sel = np.array([[fl.contents.feature[k].contents.x, fl.contents.feature[k].contents.y,
                     fl.contents.feature[k].contents.val] for k in range(NF)], np.float64)
    lib.KLTFreeFeatureList(fl)
    x = torch.from_numpy(sel[:, 0].astype(np.float32)).to(dev)
    y = torch.from_numpy(sel[:, 1].astype(np.float32)).to(dev)
    v = torch.from_numpy(sel[:, 2].astype(np.int32)).to(dev)
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))

    gather_events = []  # (start, end) HIP event pairs around each all-gather, when timing

    def all_gather(out, inp):  # the per-chunk exchange: every rank's slot, in rank order
        ev = None
        if timing[0]:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if not dist.is_initialized():
            out.copy_(inp)
        elif dist.get_backend() == "gloo":  # the shared-GPU rehearsal (KLT_BENCH_SHARE_GPU=1)
            parts = [torch.empty_like(inp) for _ in range(world)]
            dist.all_gather(parts, inp)
            out.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(out, inp)
        if ev is not None:
            ev[1].record()
            gather_events.append(ev)

    timing = [False]
    seq = ShardedSequence(lib, ctx, pd, td, frames, x, y, v, rank, world, all_gather, chunk=chunk,
                          margin=margin, edges=edges)
    seq.begin(0)
    seq.run(1, warmup)
    torch.cuda.synchronize()
    d_warm = state_digest(x, y, v)
    xs, ys, vs = x.clone(), y.clone(), v.clone()
    live_before = int((vs >= 0).sum().item())
    setup_s = time.perf_counter() - t_setup
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seq.run(1 + warmup, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    redone_timed = seq.redone
    d_end = state_digest(x, y, v)
    live_end = int((v >= 0).sum().item())
    per_rank_s = [r[0] for r in gather_floats([dt], world, dev)]
    dt_max = max(per_rank_s)

    rep = None
    if replay and steps > 0:
        # the same frames from the same state, with events: the all-gather's
        # time per chunk and each chunk's time on this rank
        x.copy_(xs); y.copy_(ys); v.copy_(vs)
        seq.begin(warmup)
        torch.cuda.synchronize()
        timing[0] = True
        seq.xch.timing, seq.xch.timing_events = True, []
        if world > 1:
            dist.barrier()
        e_start = torch.cuda.Event(enable_timing=True)
        e_start.record()
        seq.run(1 + warmup, steps)
        torch.cuda.synchronize()
        timing[0] = False
        seq.xch.timing = False
        ag = [a.elapsed_time(b) * 1e3 for a, b in gather_events]
        ends = [e_start] + seq.xch.timing_events
        chunk_us = [a.elapsed_time(b) * 1e3 for a, b in zip(ends, ends[1:])]
        d_rep = state_digest(x, y, v)
        stats = [float(np.median(ag)) if ag else 0.0, max(ag) if ag else 0.0, float(sum(ag)),
                 float(np.median(chunk_us)) if chunk_us else 0.0, float(sum(chunk_us))]
        all_stats = gather_floats(stats, world, dev)
        rep = {"allgather_us_per_chunk_median": max(s[0] for s in all_stats),
               "allgather_us_per_chunk_max": max(s[1] for s in all_stats),
               "allgather_us_per_chunk_median_by_rank": [s[0] for s in all_stats],
               "allgather_us_per_frame": max(s[2] for s in all_stats) / steps,
               "allgather_calls_per_rank": len(ag),
               "chunk_us_median_by_rank": [s[3] for s in all_stats],
               "replay_us_per_frame_by_rank": [s[4] / steps for s in all_stats],
               "allgather_op": ("copy (world 1, no process group)" if not dist.is_initialized() else
                                "torch.distributed.all_gather_into_tensor (" + dist.get_backend() + ")"),
               "what": "a replay of the timed frames from the same state with HIP events on the tracking stream "
                       "around each all-gather (the collective as the chunk's stream sees it, wait included) and "
                       "after each exchange; the timed region carries no events",
               "state_equals_timed_region": d_rep == d_end}
    # parity: the reference's column digests of this sequence (column j = the list after frame j+1)
    fix = GOLDEN / "long_config4.json"
    parity = None
    if fix.exists():
        cfg = json.loads(fix.read_text())
        if (cfg["w"], cfg["h"], cfg["features"], cfg["seed"]) == (W, H, NF, seed) and nframes <= cfg["frames"]:
            cols = cfg["columns"]
            got = [(warmup, d_warm), (warmup + steps, d_end)]
            if rep is not None:
                got.append((warmup + steps, d_rep))
            mism = sum(1 for f, d in got if f >= 1 and d != cols[f - 1])
            parity = {"against": "tests/golden/long_config4.json (reference src/V3 compiled from its own sources, "
                                 "oracle/_ref)",
                      "columns_compared": [f for f, _ in got],
                      "columns_mismatched": mism,
                      "digest": "sha256(x f32 LE || y f32 LE || val i32 LE) of the whole list, rank 0"}
    agree = gather_floats([float(int(d_end[:12], 16))], world, dev)
    out = {
        "value": steps / dt_max,
        "unit": "frames/s",
        "us_per_frame": 1e6 * dt_max / steps,
        "n_gpus": world,
        "scaling": "strong",
        "frames_timed": steps,
        "ms": 1e3 * dt_max,
        "rank_us_per_frame": [1e6 * s / steps for s in per_rank_s],
        "workload": f"{W}x{H}, {NF} features selected on frame 0, one sequence of {nframes} frames (seed {seed}), "
                    f"features sharded by row band over {world} GPU(s) (BASELINE config 4); frames 1..{warmup} "
                    f"untimed, {warmup + 1}..{warmup + steps} timed",
        "chunk": chunk, "margin_rows": margin, "bands_edges": list(edges),
        "rank_frame_rows": [frames.ra, frames.rb],
        "live_features": {"after_warmup": live_before, "at_end": live_end},
        "chunks_redone_full_frame": redone_timed,
        "state_digest": d_end,
        "ranks_agree_on_state": len({a[0] for a in agree}) == 1,
        "setup_s": setup_s,
    }
    if rep is not None:
        out["exchange"] = rep
    if parity is not None:
        out["parity"] = parity
    lib.KLTFreeTrackingContext(tc)
    del frames, x, y, v, xs, ys, vs
    lib.klt_amd_release_cached_devices()
    torch.cuda.empty_cache()
    return out


def sharded_4k_leg(world, rank, dev, args):
    """The north-star's strong-scaling workload in every run, at N = 1 and
    N > 1 (every rank takes part): BASELINE config 4, 3840x2160, 20 000
    features, the 1 000-frame sequence tests/golden/long_config4.json pins,
    64-frame chunks, 64-row margins; 64 frames warm up, 935 are timed."""
    cfg = json.loads((ROOT / "tests" / "golden" / "long_config4.json").read_text())
    wu = 64
    return sharded_core(world, rank, dev, cfg["w"], cfg["h"], cfg["features"], cfg["seed"], wu,
                        cfg["frames"] - 1 - wu, 64, 64)


def run_sharded(args, world, rank, dev) -> None:
    """--mode sharded: config 4 as the whole bench line (sharded_core)."""
    import torch.distributed as dist
    r = sharded_core(world, rank, dev, args.width, args.height, args.features, args.seed, args.warmup, args.steps,
                     args.chunk, args.margin, args.reduction)
    W, H, NF = args.width, args.height, args.features
    result = {
        "metric": METRIC,
        "value": r["value"],
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["us_per_frame"] / 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: include/klt_synth.h value-noise frames, (0.7,0.3) px/frame, seed {args.seed}",
        "config": {"workload": f"{W}x{H}, {NF} features, one sequence, features sharded by row band over "
                               f"{world} GPU(s) (BASELINE config 4)",
                   "resolution": f"{W}x{H}", "features": NF, "frames": 1 + args.warmup + args.steps,
                   "chunk": args.chunk, "margin_rows": args.margin, "parallelism": f"row-band feature sharding x{world}",
                   "rank_frame_rows": r["rank_frame_rows"]},
        "live_features": r["live_features"],
        "chunks_redone_full_frame": r["chunks_redone_full_frame"],
        "state_digest": r["state_digest"],
        "sharded": r,
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def pass_4k(lib, dev, chunk=64, reps=2, nf=20000):
    """The north-star figure (BASELINE.json): the convolve+pyramid pass at
    3840x2160 against the HBM roofline, in BASELINE config 4's shape on one
    GPU: resident synthetic 4K frames, `nf` features selected on frame 0 and
    tracked (klt_hip_track_frames, one stream, 64-frame launches), so every
    pyramid launch follows a tracker launch as in production.  `reps` chunks
    are timed with HIP events on the launch stream after one warm-up chunk;
    each kernel's event time is its own duration (one stream: nothing runs
    beside it).  The same frames built back to back with no tracking
    (`pyramids_only`) run the pyramid kernels at the lower clock the chip holds
    under sustained pyramid load; both are reported.
    Algorithmic bytes as for the 1080p line: 13.75 B/px (u8 in, img/gx/gy out
    at both levels)."""
    import torch
    from kltamd.device import PyrDesc, TrackDesc, Timing, check, use_torch_stream
    W, H = 3840, 2160
    # the earlier legs' parked device contexts and torch's cached blocks go
    # back to the driver first, so the 4K banks are not laid out in their holes
    lib.klt_amd_release_cached_devices()
    torch.cuda.empty_cache()
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    ctx = lib.klt_amd_device_context(tc)
    use_torch_stream(lib, ctx, dev)
    n = 1 + chunk * (1 + reps)
    fr = torch.empty((n, H, W), dtype=torch.uint8, device=dev)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, 2160, 0, n, W, H, C.c_void_p(fr.data_ptr()), W, W * H), "synth")
    f0 = fr[0].cpu().numpy()
    fl = lib.KLTCreateFeatureList(nf)
    lib.KLTSelectGoodFeatures(tc, f0.ctypes.data_as(C.POINTER(C.c_ubyte)), W, H, fl)
    sel = np.array([[fl.contents.feature[k].contents.x, fl.contents.feature[k].contents.y,
                     fl.contents.feature[k].contents.val] for k in range(nf)], np.float64)
    lib.KLTFreeFeatureList(fl)
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    base = fr.data_ptr()

    def leg(features):
        x = torch.from_numpy(sel[:, 0].astype(np.float32)).to(dev)
        y = torch.from_numpy(sel[:, 1].astype(np.float32)).to(dev)
        v = torch.from_numpy(sel[:, 2].astype(np.int32)).to(dev)
        k = nf if features else 0

        def run(t0, m):
            check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(base + t0 * W * H),
                                                     W, W * H, m, chunk, C.c_void_p(x.data_ptr()),
                                                     C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), k, None,
                                                     None, None, 0), "4k")

        check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(base), W), "4k begin")
        run(1, chunk)
        torch.cuda.synchronize()
        lib.klt_hip_set_timing(ctx, 1)
        run(1 + chunk, chunk * reps)
        tm = Timing()
        check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "4k timing")
        lib.klt_hip_set_timing(ctx, 0)
        l0 = 1000.0 * tm.ms_pyr_l0 / tm.frames_pyr_l0
        l1 = 1000.0 * tm.ms_pyr_l1 / tm.frames_pyr_l1
        trk = 1000.0 * tm.ms_track / tm.frames_track if tm.frames_track else None
        return l0, l1, trk, tm, int((v >= 0).sum().item())

    # every bank of the arena is written once before anything is timed (the
    # legs' timed chunks land in banks their warm-up chunk did not touch)
    check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(base), W), "4k begin")
    check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(base + W * H), W, W * H,
                                             n - 1, chunk, None, None, None, 0, None, None, None, 0), "4k touch")
    torch.cuda.synchronize()
    p0, p1, _, ptm, _ = leg(False)
    l0, l1, trk, tm, live = leg(True)
    lib.KLTFreeTrackingContext(tc)
    del fr
    torch.cuda.empty_cache()
    by = W * H * 13 + (W // 4) * (H // 4) * 12
    ach = by / ((l0 + l1) * 1e-6) / 1e9
    pach = by / ((p0 + p1) * 1e-6) / 1e9
    return {"workload": f"{W}x{H} pyramid pass, batched {chunk} frames per launch, {nf} features tracked between "
                        "the pyramid launches (BASELINE config 4 on one GPU)",
            "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": None, "frames_per_launch": tm.frames_pyr_l0 / tm.n_pyr_l0,
            "algorithmic_bytes_per_frame": by, "us_per_frame": l0 + l1,
            "kernels_us_per_frame": {"k_pyr_l0": l0, "k_pyr_l1": l1, "k_track": trk}, "frames_timed": int(tm.frames_pyr_l0),
            "live_features_at_end": live,
            "pyramid_gpix_s": W * H / ((l0 + l1) * 1e-6) / 1e9,
            "event_timing": "HIP events on the launch stream, one stream",
            "pyramids_only": {"what": "the same frames built back to back with no features tracked",
                              "achieved": pach, "frac": pach / HBM_PEAK_GBS, "us_per_frame": p0 + p1,
                              "kernels_us_per_frame": {"k_pyr_l0": p0, "k_pyr_l1": p1},
                              "frames_timed": int(ptm.frames_pyr_l0)}}


def frames_4k_leg(lib, dev, chunk=64):
    """North_star's frames/s at 4K: BASELINE config 4 on one GPU -- 3840x2160,
    20 000 features selected on frame 0, all 1000 tracked frames (seed 2160,
    the sequence tests/golden/long_config4.json pins), KLTStoreFeatureList per
    frame.  Two regions, each timed by the wall clock after an untimed warm-up
    run of its own:
      device: frames synthesised into HBM, klt_hip_track_frames with the
              feature table on the device (the 1080p headline's path, 64-frame
              chunks, the next chunk's pyramids on a second stream);
      sequence: KLTTrackSequence over host frames (pageable numpy) writing a
              host KLT_FeatureTable -- frame uploads over PCIe, pyramids,
              tracking and the table rows coming back, all inside the region.
    Parity: every column of both tables against the reference's per-frame
    digests (long_config4.json, made by the reference compiled from its own
    sources), bit for bit."""
    import hashlib
    import torch
    from kltabi import GOLDEN, fl_to_arrays
    from kltamd.device import PyrDesc, TrackDesc, check, use_torch_stream
    cfg = json.loads((GOLDEN / "long_config4.json").read_text())
    W, H, NF, NFR, seed = cfg["w"], cfg["h"], cfg["features"], cfg["frames"], cfg["seed"]
    T = NFR - 1
    U8P = C.POINTER(C.c_ubyte)
    lib.klt_amd_release_cached_devices()
    torch.cuda.empty_cache()

    def digest_cols(X, Y, V):
        out = []
        for j in range(X.shape[0]):
            h = hashlib.sha256()
            h.update(np.ascontiguousarray(X[j], "<f4").tobytes())
            h.update(np.ascontiguousarray(Y[j], "<f4").tobytes())
            h.update(np.ascontiguousarray(V[j], "<i4").tobytes())
            out.append(h.hexdigest())
        return out

    def mismatched(cols):
        return sum(1 for a, b in zip(cols, cfg["columns"]) if a != b) + abs(len(cols) - len(cfg["columns"]))

    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    ctx = lib.klt_amd_device_context(tc)
    check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 1), "overlap")
    use_torch_stream(lib, ctx, dev)
    fr = torch.empty((NFR, H, W), dtype=torch.uint8, device=dev)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, seed, 0, NFR, W, H, C.c_void_p(fr.data_ptr()), W, W * H), "synth")
    host = fr.cpu().numpy()  # the sequence leg's pageable host frames (the same bytes)
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, host[0].ctypes.data_as(U8P), W, H, fl)
    sel = fl_to_arrays(fl)
    lib.KLTFreeFeatureList(fl)
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    tab = [torch.empty((T, NF), dtype=dt, device=dev) for dt in (torch.float32, torch.float32, torch.int32)]
    xyz = [torch.from_numpy(np.asarray(a).copy()).to(dev) for a in sel]

    def device_run():
        for t, a in zip(xyz, sel):
            t.copy_(torch.from_numpy(np.asarray(a)))
        check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fr.data_ptr()), W), "4k begin")
        torch.cuda.synchronize()
        a = time.perf_counter()
        check(lib, ctx, lib.klt_hip_track_frames(
            ctx, C.byref(pd), C.byref(td), C.c_void_p(fr.data_ptr() + W * H), W, W * H, T, chunk,
            *[C.c_void_p(t.data_ptr()) for t in xyz], NF, *[C.c_void_p(t.data_ptr()) for t in tab], NF), "4k frames")
        torch.cuda.synchronize()
        return time.perf_counter() - a

    device_run()  # warm-up: allocations, banks written once
    dt_dev = device_run()
    dev_cols = digest_cols(*(t.cpu().numpy() for t in tab))
    live_dev = int((xyz[2] >= 0).sum().item())
    lib.KLTFreeTrackingContext(tc)
    del fr, tab, xyz
    torch.cuda.empty_cache()

    arr = (U8P * NFR)(*[host[t].ctypes.data_as(U8P) for t in range(NFR)])
    ft = lib.KLTCreateFeatureTable(T, NF)

    def sequence():
        tc = lib.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        fl = lib.KLTCreateFeatureList(NF)
        lib.KLTSelectGoodFeatures(tc, host[0].ctypes.data_as(U8P), W, H, fl)
        a = time.perf_counter()
        lib.KLTTrackSequence(tc, arr, NFR, W, H, fl, ft, 0)
        d = time.perf_counter() - a
        lib.KLTFreeFeatureList(fl)
        lib.KLTFreeTrackingContext(tc)
        return d

    sequence()  # warm-up call: the device context, staging and host threads; the table's first touch
    dt_seq = sequence()
    nfr = ft.contents.nFrames
    base = C.addressof(ft.contents.feature[0][0].contents)
    raw = np.ctypeslib.as_array((C.c_uint8 * (64 * NF * nfr)).from_address(base)).view(np.int32)
    raw = raw.reshape(NF, nfr, 16)[:, :T]
    seq_cols = digest_cols(raw[:, :, 0].view(np.float32).T, raw[:, :, 1].view(np.float32).T, raw[:, :, 2].T)
    lib.KLTFreeFeatureTable(ft)
    del host
    lib.klt_amd_release_cached_devices()
    return {"workload": f"{W}x{H}, {NF} features selected on frame 0, {T} tracked frames (BASELINE config 4 on one "
                        f"GPU, seed {seed}), KLTStoreFeatureList per frame",
            "device": {"value": T / dt_dev, "unit": "frames/s", "frames": T, "ms": 1e3 * dt_dev,
                       "region": "klt_hip_track_frames over frames resident in HBM, feature table on the device, "
                                 f"{chunk}-frame chunks, next chunk's pyramids on a second stream",
                       "live_features_at_end": live_dev, "columns_mismatched": mismatched(dev_cols)},
            "sequence": {"value": T / dt_seq, "unit": "frames/s", "frames": T, "ms": 1e3 * dt_seq,
                         "region": "one KLTTrackSequence call over pageable host frames writing a host "
                                   "KLT_FeatureTable (PCIe uploads and table rows inside the region)",
                         "columns_mismatched": mismatched(seq_cols)},
            "parity": f"every column of both tables against tests/golden/long_config4.json ({len(cfg['columns'])} "
                      "reference digests)"}


def attach_traffic(line, pmc, resolution, fpl) -> None:
    """roofline.traffic: HBM bytes per launch from the committed PMC summary of
    the same kernels (tools/pmc_traffic.sh + tools/pmc_traffic_json.py), when
    it was taken at this resolution.  Static: rocprofv3 counters cannot be
    read from inside this process."""
    if not pmc.exists():
        return
    try:
        d = json.loads(pmc.read_text())
    except ValueError:
        return
    if d.get("resolution") != resolution:
        return
    line["traffic"] = d["pass_hbm_bytes_per_frame"] * fpl  # per launch, like `achieved`
    line["traffic_per_frame"] = d["pass_hbm_bytes_per_frame"]
    line["traffic_over_algorithmic"] = d["pass_hbm_bytes_per_frame"] / d["pass_algorithmic_bytes_per_frame"]
    line["traffic_source"] = str(pmc.relative_to(ROOT))
    line["traffic_kind"] = ("static: FETCH_SIZE (x2, gfx950) + WRITE_SIZE from separate rocprofv3 --pmc passes over "
                            f"the same kernels at {resolution}, {d.get('frames_per_launch', '?')} frames per launch "
                            "(tools/pmc_traffic.sh); counters cannot be read inside this process")


def schedule_name(args) -> str:
    """What the timed region actually launched."""
    if args.chunk == 0:
        return "per-frame pipeline: frame t+1's pyramid on a second stream while frame t is tracked"
    n = -(-args.steps // args.chunk)
    if args.serial or n < 2:
        return f"{n} chunk(s) of <= {args.chunk} frames, pyramids and tracker on one stream"
    return (f"{n} chunks of <= {args.chunk} frames; pyramids of chunk c+1 on a second stream while chunk c is "
            "tracked (the first chunk's pyramids are not overlapped)")


def fast_leg(lib, ctx, td, tab, exact_tab, xs, ys, vs, x, y, v, build0, run, t_start, args):
    """The timed region again with KLT_HIP_FAST: the tracker's five window
    sums by a wave butterfly instead of the reference's sequential 49-term
    sums (trackFeatures.c:241-248, :271-278).  Not bit-exact: reported with its
    distance from the exact run over the same frames (val mismatches, max
    |dx|,|dy| over cells tracked by both); the tolerance it is held to is
    tests/test_gpu_long.py::test_fast_reduction_tolerance."""
    import torch
    from kltamd.device import FAST, Timing, check
    saved = td.reduction
    td.reduction = FAST
    try:
        x.copy_(xs); y.copy_(ys); v.copy_(vs)
        build0(t_start - 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(t_start, args.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ft = [t[t_start - 1:t_start - 1 + args.steps].clone() for t in tab]
        # per-kernel events in a one-stream replay, as for the exact line
        x.copy_(xs); y.copy_(ys); v.copy_(vs)
        check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 0), "overlap")
        build0(t_start - 1)
        lib.klt_hip_set_timing(ctx, 1)
        run(t_start, max(args.steps, args.replay_frames), args.chunk_requested)  # as the exact line's replay
        tm = Timing()
        check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
        lib.klt_hip_set_timing(ctx, 0)
    finally:
        td.reduction = saved
    ev, fv = exact_tab[2], ft[2]
    both = (ev == 0) & (fv == 0)
    dx = (exact_tab[0][both].double() - ft[0][both].double()).abs()
    dy = (exact_tab[1][both].double() - ft[1][both].double()).abs()
    return {"value": args.steps / dt, "unit": "frames/s", "ms_per_step": 1000.0 * dt / args.steps,
            "k_track_us_per_frame": 1000.0 * tm.ms_track / tm.frames_track if tm.frames_track else None,
            "vs_exact": {"cells": int(ev.numel()), "val_mismatches": int((ev != fv).sum().item()),
                         "max_dx": float(dx.max().item()) if dx.numel() else 0.0,
                         "max_dy": float(dy.max().item()) if dy.numel() else 0.0,
                         "tracked_in_both": int(both.sum().item())},
            "note": "wave-shuffle window sums (KLT_HIP_FAST); not bit-exact, see vs_exact"}


def api_leg(lib, frames, W, H, NF, args):
    """SURVEY 8(d)'s frames/sec through the klt.h API, host frames in pageable
    memory, PCIe and the feature-list round trip inside the timed region:
      per_call: one KLTTrackFeatures call per frame, wall clock around each
                call as example3.c:61-63 times it; the first call (two pyramids)
                is excluded, as the reference's steady state;
      sequence: KLTTrackSequence over the same frames with a feature table
                (the example3.c loop + KLTStoreFeatureList in one call;
                klt_amd.h), after a warm-up call of its own for allocations.
    Both select on frame 0 of the same sequence the device line tracks."""
    import torch
    from kltabi import fl_to_arrays
    U8P = C.POINTER(C.c_ubyte)
    n = min(args.api_frames, frames.shape[0] - 1)
    host = [np.ascontiguousarray(frames[t].cpu().numpy()) for t in range(n + 1)]
    torch.cuda.synchronize()
    u8 = lambda a: a.ctypes.data_as(U8P)  # noqa: E731

    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
    lib.KLTTrackFeatures(tc, u8(host[0]), u8(host[1]), W, H, fl)  # builds both pyramids: not steady state
    times = []
    for t in range(2, n + 1):
        a = time.perf_counter()
        lib.KLTTrackFeatures(tc, u8(host[t - 1]), u8(host[t]), W, H, fl)
        times.append(time.perf_counter() - a)
    pc = fl_to_arrays(fl)
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)

    def harness_loop(register):
        """example3.c:44-76 as written: two fixed buffers, img2 refilled per
        frame (pgmReadFile) and copied into img1 after the call; only the
        KLTTrackFeatures call is timed.  register: the klt_amd.h opt-in that
        page-locks both buffers once."""
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
        out = fl_to_arrays(fl)
        lib.KLTFreeFeatureList(fl)
        lib.KLTFreeTrackingContext(tc)
        return ts[1:], out  # the first call builds two pyramids

    h_times, h_out = harness_loop(False)
    r_times, r_out = harness_loop(True)
    same_reg = all(np.array_equal(np.asarray(p).view(np.int32), np.asarray(q).view(np.int32))
                   for p, q in zip(pc, r_out)) and all(
        np.array_equal(np.asarray(p).view(np.int32), np.asarray(q).view(np.int32)) for p, q in zip(pc, h_out))

    replace = replace_leg(lib, host, W, H, NF, args)

    arr = (U8P * (n + 1))(*[u8(a) for a in host])
    ft = lib.KLTCreateFeatureTable(n, NF)

    import resource
    import tempfile

    def sequence(trace=None):
        """one KLTTrackSequence call; trace (a dict): the library's KLT_SEQ_TRACE line
        of the call (stderr, captured) and the process's involuntary context switches
        and page faults over it"""
        tc = lib.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        fl = lib.KLTCreateFeatureList(NF)
        lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
        if trace is not None:
            sys.stderr.flush()
            tmp, saved = tempfile.TemporaryFile(mode="w+"), os.dup(2)
            os.dup2(tmp.fileno(), 2)
            r0 = resource.getrusage(resource.RUSAGE_SELF)
        a = time.perf_counter()
        lib.KLTTrackSequence(tc, arr, n + 1, W, H, fl, ft, 0)
        dt = time.perf_counter() - a
        if trace is not None:
            r1 = resource.getrusage(resource.RUSAGE_SELF)
            os.dup2(saved, 2)
            os.close(saved)
            tmp.seek(0)
            line = [t for t in tmp.read().splitlines() if t.startswith("seqtrace")]
            tmp.close()
            kv = dict(t.split("=") for t in line[-1].split()[1:]) if line else {}
            trace["stages_us"] = {k: float(v) for k, v in kv.items() if k.endswith("_us")} if line else None
            # minor page faults per stage: the process's (_pf) and the calling thread's (_tf)
            trace["stage_faults"] = {k: int(v) for k, v in kv.items() if k.endswith(("_pf", "_tf"))} if line else None
            trace["involuntary_context_switches"] = r1.ru_nivcsw - r0.ru_nivcsw
            trace["minor_page_faults"] = r1.ru_minflt - r0.ru_minflt
            trace["process_cpu_s"] = (r1.ru_utime + r1.ru_stime) - (r0.ru_utime + r0.ru_stime)
        out = fl_to_arrays(fl)
        lib.KLTFreeFeatureList(fl)
        lib.KLTFreeTrackingContext(tc)
        return dt, out

    def h2d_gbs():
        """the bus right now: one 256 MiB pinned -> device copy"""
        torch.cuda.synchronize()
        a = time.perf_counter()
        bus_dst.copy_(bus_src, non_blocking=True)
        torch.cuda.synchronize()
        return bus_src.numel() / (time.perf_counter() - a) / 1e9

    # two calls warm the device context that the timed call's tracking context
    # then takes over (klt_api.c keeps the device contexts of freed tracking
    # contexts: banks, staging, host threads); the table's pages are touched
    dt_cold, _ = sequence()
    sequence()
    # five timed calls, min / median / max reported with the pinned H2D rate
    # measured right before each: the call moves 2 MB per frame over PCIe
    # (KLT_SEQ_TRACE: the host-side staging copy and the DMA are its time), so a
    # slower call goes with a slower bus (tools/seq_variance.py)
    bus_src = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
    bus_dst = torch.empty(256 << 20, dtype=torch.uint8, device=frames.device)
    runs, bus, traces = [], [], []
    for _ in range(5):
        bus.append(h2d_gbs())
        traces.append({})
        runs.append(sequence(traces[-1]))
    del bus_src, bus_dst
    dts = [r[0] for r in runs]
    dt, sq = sorted(dts)[len(dts) // 2], runs[-1][1]
    lib.KLTFreeFeatureTable(ft)
    same = all(np.array_equal(np.asarray(p).view(np.int32), np.asarray(q).view(np.int32)) for p, q in zip(pc, sq))
    return {
        "per_call": {"value": len(times) / sum(times), "unit": "frames/s", "calls": len(times),
                     "us_per_call_median": 1e6 * float(np.median(times)),
                     "region": "wall clock around each KLTTrackFeatures call (example3.c:61-63): host u8 frame "
                               "H2D, both device kernels, feature list in/out"},
        "sequence": {"value": n / dt, "unit": "frames/s", "frames": n,
                     "region": "one KLTTrackSequence call over host frames 0..n writing every column of a "
                               "KLT_FeatureTable (frame uploads, pyramids of frames 0..n, tracking, table rows "
                               "down and stored); the median of calls 3-7 in the process on the same table, each "
                               "with a fresh tracking context and selection",
                     "calls_fps": [n / d for d in dts],
                     "calls_fps_min_median_max": [n / max(dts), n / dt, n / min(dts)],
                     "h2d_pinned_gbs_before_each_call": bus,
                     "fraction_of_bus_each_call": [(n / d) * W * H / (b * 1e9) for d, b in zip(dts, bus)],
                     "first_call_value": n / dt_cold,
                     "calls_trace": traces,
                     "first_call": "the process's first KLTTrackSequence: device allocations, pinned staging, "
                                   "host threads, the table's first touch"},
        "per_call_harness": {"value": len(h_times) / sum(h_times), "unit": "frames/s", "calls": len(h_times),
                             "us_per_call_median": 1e6 * float(np.median(h_times)),
                             "region": "example3.c's loop as written: two fixed host buffers (img2 refilled, copied "
                                       "into img1), wall clock around each KLTTrackFeatures"},
        "per_call_registered": {"value": len(r_times) / sum(r_times), "unit": "frames/s", "calls": len(r_times),
                                "us_per_call_median": 1e6 * float(np.median(r_times)),
                                "region": "the same loop after klt_amd_register_buffer on img1 and img2 (klt_amd.h "
                                          "opt-in: one DMA from the caller's pages, no staging copy)",
                                "equals_per_call": bool(same_reg)},
        "replace": replace,
        "frames": f"{W}x{H} u8 host frames (pageable numpy), {NF} features, seed {args.seed}",
        "per_call_equals_sequence": bool(same),
    }


def replace_leg(lib, host, W, H, NF, args):
    """The REPLACE harness (example3.c:62-71 with REPLACE): KLTTrackFeatures
    then KLTReplaceLostFeatures on the new frame, per host frame; wall clock
    around each call.  Parity: the list after each frame against the
    reference's digests of the same sequence (tests/golden/long_config3r.json,
    the reference compiled from its own sources) where the workload matches."""
    import hashlib
    from kltabi import fl_to_arrays
    U8P = C.POINTER(C.c_ubyte)
    u8 = lambda a: a.ctypes.data_as(U8P)  # noqa: E731
    n = min(args.replace_frames, len(host) - 1)
    if n < 2:
        return None
    fix = ROOT / "tests" / "golden" / "long_config3r.json"
    want = None
    if fix.exists():
        d = json.loads(fix.read_text())
        if (d["w"], d["h"], d["features"], d["seed"]) == (W, H, NF, args.seed):
            want = d["columns"]
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, u8(host[0]), W, H, fl)
    trk, rep, cols, replaced = [], [], [], 0
    sel_stats = []
    ctx = lib.klt_amd_device_context(tc)
    for t in range(1, n + 1):
        a = time.perf_counter()
        lib.KLTTrackFeatures(tc, u8(host[t - 1]), u8(host[t]), W, H, fl)
        b = time.perf_counter()
        lost = NF - lib.KLTCountRemainingFeatures(fl)
        c = time.perf_counter()
        lib.KLTReplaceLostFeatures(tc, u8(host[t]), W, H, fl)
        e = time.perf_counter()
        trk.append(b - a)
        rep.append(e - c)
        if lost > 0:
            st = [C.c_long() for _ in range(3)]
            us = (C.c_double * 4)()
            lib.klt_hip_select_stats(ctx, *[C.byref(q) for q in st], us)
            sel_stats.append([q.value for q in st] + list(us))
        x, y, v = fl_to_arrays(fl)
        replaced += lost - (NF - int((v >= 0).sum()))
        h = hashlib.sha256()
        for arr, dt in ((x, "<f4"), (y, "<f4"), (v, "<i4")):
            h.update(np.ascontiguousarray(arr, dt).tobytes())
        cols.append(h.hexdigest())
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)
    steady = slice(1, None)  # the first track call builds two pyramids
    per_frame = [p + q for p, q in zip(trk, rep)][steady]
    out = {"value": len(per_frame) / sum(per_frame), "unit": "frames/s", "frames": n,
           "us_per_replace_median": 1e6 * float(np.median(rep[steady])),
           "us_per_track_median": 1e6 * float(np.median(trk[steady])),
           "features_replaced": replaced,
           "select_median": dict(zip(("map_points_downloaded", "device_partition_steps", "sorted_positions_visited",
                                      "us_map_init", "us_device_splits", "us_downloads_and_host_sort", "us_select_total"),
                                     (float(np.median([q[k] for q in sel_stats])) for k in range(7))))
           if sel_stats else None,
           "region": "wall clock around KLTTrackFeatures + KLTReplaceLostFeatures per frame (example3.c:61-69 "
                     "with REPLACE), host u8 frames; first frame excluded"}
    if want is not None:
        m = min(len(want), len(cols))
        bad = [j for j in range(m) if cols[j] != want[j]]
        out["parity"] = {"against": "tests/golden/long_config3r.json (reference, oracle/_ref)",
                         "columns_compared": m, "columns_mismatched": len(bad),
                         "first_mismatch": bad[0] + 1 if bad else None}
    return out


def tracker_line(solves, passes, feature_frames, tm, kernel):
    """the LK tracker is gather/latency and VALU bound, not an HBM
    roofline kernel; report its work rate as feature-iterations per second.
    An iteration is one 2x2 system formed (a body of the reference's Newton
    loop, trackFeatures.c:418-455, both levels summed); counted on the device
    (klt_hip_set_track_count) over the same frames the kernel events time."""
    s = tm.ms_track * 1e-3
    return {
        "kernel": kernel, "bound": "VALU / gather latency (no HBM roofline, SURVEY 8d)",
        "newton_iterations": solves, "gather_passes": passes, "feature_frames": feature_frames,
        "iterations_per_feature_frame": solves / feature_frames if feature_frames else None,
        "passes_per_feature_frame": passes / feature_frames if feature_frames else None,
        "feature_iterations_per_s": solves / s if s > 0 else None,
        "feature_frames_per_s": feature_frames / s if s > 0 else None,
        "ns_per_iteration": s * 1e9 / solves if solves else None,
    }


def measured_peaks(dev, nbytes=2 << 30, reps=5):
    """Measured HBM peaks on this box, for context next to the 8 TB/s spec:
    a device-to-device copy of 2 GiB (read + write bytes) and a 2 GiB fill
    (write bytes; the pyramid pass writes 13 of its 13.75 B/px), torch's own
    kernels, HIP events on the current stream, best of `reps`."""
    import torch
    a = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)

    def best(fn, moved):
        fn()
        out = 0.0
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            out = max(out, moved / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        return out

    copy = best(lambda: b.copy_(a), 2.0 * nbytes)
    fill = best(lambda: b.fill_(2.0), 1.0 * nbytes)
    del a, b
    torch.cuda.empty_cache()
    return {"copy_gbs": copy, "fill_gbs": fill, "source": "torch copy_/fill_ of 2 GiB, HIP events, best of 5"}


def cpu_leg(lib, frames, W, H, NF, args, tc, ctx, dev):
    """Bounded sample of the same workload on the host: the reference CPU path
    (oracle/_ref, built from /root/reference) or, if absent, the oracle port.
    Then the GPU runs the same frames and every cell is compared."""
    import torch
    from kltabi import REF_LIB, KLTRunner, OracleTracker, bind_klt, load_oracle

    S = min(args.cpu_frames, frames.shape[0])
    host = [frames[t].cpu().numpy() for t in range(S)]
    kind = "reference" if REF_LIB.exists() else "port"
    rl = bind_klt(REF_LIB) if kind == "reference" else None
    cols = []  # the list after every frame (example3.c's KLTStoreFeatureList columns)
    sel_t = time.perf_counter()
    if rl is not None:
        rl.KLTSetVerbosity(0)
        rtc = rl.KLTCreateTrackingContext()
        rtc.contents.sequentialMode = 1
        fl = rl.KLTCreateFeatureList(NF)
        u8 = lambda a: a.ctypes.data_as(C.POINTER(C.c_ubyte))  # noqa: E731
        rl.KLTSelectGoodFeatures(rtc, u8(host[0]), W, H, fl)
        sel_s = time.perf_counter() - sel_t
        times, ctimes = [], []
        lx, ly, lv = list_view(fl)
        for t in range(1, S):
            a, ca = time.perf_counter(), time.process_time()
            rl.KLTTrackFeatures(rtc, u8(host[t - 1]), u8(host[t]), W, H, fl)
            times.append(time.perf_counter() - a)
            ctimes.append(time.process_time() - ca)
            cols.append((lx.copy(), ly.copy(), lv.copy()))  # KLTStoreFeatureList, outside the timed call
        cx, cy, cv = cols[-1]
        rl.KLTFreeFeatureList(fl)
        rl.KLTFreeTrackingContext(rtc)
    else:
        ot = OracleTracker(load_oracle())
        ot.params.sequentialMode = 1
        ot.lib.orc_set_params(ot.h, C.byref(ot.params))
        cx, cy, cv = ot.select(host[0], NF)
        sel_s = time.perf_counter() - sel_t
        times, ctimes = [], []
        for t in range(1, S):
            a, ca = time.perf_counter(), time.process_time()
            ot.track(host[t - 1], host[t], cx, cy, cv)
            times.append(time.perf_counter() - a)
            ctimes.append(time.process_time() - ca)
            cols.append((cx.copy(), cy.copy(), cv.copy()))
    steady = times[1:] if len(times) > 1 else times  # first call builds two pyramids
    csteady = ctimes[1:] if len(ctimes) > 1 else ctimes
    cpu_fps = len(steady) / sum(steady)
    # the reference harness's own metric is clock() (example3.c:61-63): process CPU time
    clock_fps = len(csteady) / sum(csteady) if sum(csteady) > 0 else None

    # the timed GPU path on the same frames (same reduction): cell-by-cell parity
    # over every column of the feature table
    TX, TY, TV = gpu_sequence(lib, host, NF, args.chunk, not args.serial, args.reduction)
    mism = 0
    for j, (cx_, cy_, cv_) in enumerate(cols):
        mism += int((TX[j].view(np.int32) != cx_.view(np.int32)).sum() +
                    (TY[j].view(np.int32) != cy_.view(np.int32)).sum() + (TV[j] != cv_).sum())
    cpu = {"value": cpu_fps, "unit": "frames/s", "cores": 1, "kind": kind, "value_clock": clock_fps,
           "sample": f"first {S} frames of the same {W}x{H} sequence, {NF} features, sequential mode; "
                     f"{len(steady)} steady-state KLTTrackFeatures calls timed (wall clock), "
                     f"selection {sel_s:.2f}s not included",
           "cpu_model": cpu_model(), "nproc": os.cpu_count()}
    par = {"frames": S, "features": NF, "cells": 3 * NF * len(cols), "mismatched_values": mism,
           "compared": "x, y (bit patterns) and val of every (feature, frame) cell of the feature table",
           "reduction": args.reduction, "live_at_end": int((cv >= 0).sum()), "against": kind}
    return cpu, par


def list_view(fl):
    """(x, y, val) views of a klt.h feature list whose 64-byte records are one
    block (KLTCreateFeatureList, klt.c:143-170)."""
    n = fl.contents.nFeatures
    base = C.addressof(fl.contents.feature[0].contents)
    assert C.addressof(fl.contents.feature[n - 1].contents) == base + 64 * (n - 1)
    raw = np.ctypeslib.as_array((C.c_uint8 * (64 * n)).from_address(base)).view(np.int32).reshape(n, 16)
    return raw[:, 0].view(np.float32), raw[:, 1].view(np.float32), raw[:, 2]


def gpu_sequence(lib, host, NF, chunk, overlap, reduction="exact"):
    """The timed path (klt_hip_track_frames -- or klt_hip_track_sequence for
    chunk 0 -- frames + features in HBM) on the CPU sample's frames: select on
    frame 0, then track frames 1..S-1.  Returns the feature table [S-1, NF]
    (row j = the list after frame j+1; for chunk 0 only the last row is real)."""
    from kltamd.device import EXACT, FAST
    import torch
    from kltamd.device import PyrDesc, TrackDesc, check, use_torch_stream
    H, W = host[0].shape
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    lib.klt_amd_set_reduction(tc, EXACT if reduction == "exact" else FAST)
    ctx = lib.klt_amd_device_context(tc)
    dev = torch.device("cuda", torch.cuda.current_device())
    use_torch_stream(lib, ctx, dev)
    check(lib, ctx, lib.klt_hip_set_frames_overlap(ctx, 1 if overlap else 0), "overlap")  # the timed schedule
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, host[0].ctypes.data_as(C.POINTER(C.c_ubyte)), W, H, fl)
    x = torch.tensor([fl.contents.feature[k].contents.x for k in range(NF)], dtype=torch.float32, device=dev)
    y = torch.tensor([fl.contents.feature[k].contents.y for k in range(NF)], dtype=torch.float32, device=dev)
    v = torch.tensor([fl.contents.feature[k].contents.val for k in range(NF)], dtype=torch.int32, device=dev)
    lib.KLTFreeFeatureList(fl)
    fr = torch.from_numpy(np.stack(host)).to(dev)
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    T = len(host) - 1
    tab = [torch.zeros((T, NF), dtype=dt, device=dev) for dt in (torch.float32, torch.float32, torch.int32)]
    if chunk > 0:
        tp = [C.c_void_p(a.data_ptr()) for a in tab]
        check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fr.data_ptr()), W), "begin")
        check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(fr.data_ptr() + W * H), W,
                                                 W * H, T, chunk, C.c_void_p(x.data_ptr()),
                                                 C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), NF, tp[0],
                                                 tp[1], tp[2], NF), "frames")
    else:
        check(lib, ctx, lib.klt_hip_build_pyramid(ctx, 0, C.byref(pd), C.c_void_p(fr.data_ptr()), W, 0), "build")
        slot = C.c_int(0)
        check(lib, ctx, lib.klt_hip_track_sequence(ctx, C.byref(pd), C.byref(td), C.c_void_p(fr.data_ptr()), W,
                                                   W * H, 1, len(host) - 1, C.c_void_p(x.data_ptr()),
                                                   C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), NF,
                                                   C.byref(slot)), "sequence")
    torch.cuda.synchronize()
    if chunk == 0:  # the pipelined path keeps no table: its final list is the last row
        tab[0][-1].copy_(x), tab[1][-1].copy_(y), tab[2][-1].copy_(v)
    out = tuple(a.cpu().numpy() for a in tab)
    lib.KLTFreeTrackingContext(tc)
    return out


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
