#!/usr/bin/env python3
"""Config 4 (feature-sharded 4K sequence) on ONE GPU.  Pass 1: every rank of
an N-rank row-band decomposition runs in turn per chunk (its own device
context, band pyramids and features, klt_hip_track_frames_band with the next
chunk built ahead), and the ranks' results are merged exactly as
kltamd.shard.merge_chunk merges them over RCCL; every N must end in the same
feature state bit for bit (the state digest).  Pass 2: each rank alone replays
its whole schedule from the merged chunk-start states -- band call with the
next chunk built ahead on its pyramid stream, then the host read of the escape
flag, as ShardedSequence does -- timed by the host clock, in a process of its
own (one device context, as on an N-GPU node: the ranks' streams must not
share hardware queues).  That is what one rank does, and gives the projected
N-GPU rate
    frame time(N) = max over ranks (rank time per frame) + exchange(N)
with the exchange (one all-reduce of 3n+1 int32 per chunk) from
--exchange-us, since one GPU cannot measure RCCL over xGMI.
usage: python tools/shard_sim.py [--worlds 1 2 4 8] [--margins 64] [--frames 129] [--chunk 32]
"""
from __future__ import annotations

import argparse
import os
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--features", type=int, default=20000)
    ap.add_argument("--frames", type=int, default=129, help="frames incl. the selection frame")
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--margins", type=int, nargs="+", default=[64])
    ap.add_argument("--seed", type=int, default=2160)
    ap.add_argument("--balanced", action="store_true", help="bands of equal feature counts (balanced_edges)")
    ap.add_argument("--no-ahead", action="store_true", help="pass 2 without building the next chunk ahead")
    ap.add_argument("--own-streams", action="store_true",
                    help="pass 2: the library on its own streams (not a torch pool stream), synchronized by host")
    ap.add_argument("--lazy-flag", action="store_true",
                    help="pass 2: read chunk c's escape flag after chunk c+1 is queued (a speculative driver "
                         "redoes c and drops c+1 when it is set), so the host never drains the stream per chunk")
    ap.add_argument("--keep-states", default=None,
                    help="save pass 1's chunk-start states as DIR/states_w<N>.npz (for a profiled --replay)")
    ap.add_argument("--pass1-shared", action="store_true",
                    help="pass 1 (the merged states) through one device context for every rank, each chunk "
                         "started from a whole-frame pyramid: one bank arena instead of N (long chunks at 4K)")
    ap.add_argument("--replay", default=None, help=argparse.SUPPRESS)  # internal: pass 2 of one rank (npz of states)
    ap.add_argument("--rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--exchange-us", type=float, default=40.0,
                    help="assumed per-chunk exchange: RCCL all-reduce of 3n+1 int32 + escape-flag read (N > 1)")
    a = ap.parse_args()

    import torch
    import kltamd
    from kltamd.device import PyrDesc, Timing, TrackDesc, check, use_torch_stream
    from kltamd.shard import balanced_edges, band_of, merge_chunk
    from kltabi import fl_to_arrays, u8ptr

    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    W, H, NF = a.width, a.height, a.features
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fr = torch.empty((a.frames, H, W), dtype=torch.uint8, device=dev)
    tc0 = lib.KLTCreateTrackingContext()
    ctx0 = lib.klt_amd_device_context(tc0)
    check(lib, ctx0, lib.klt_hip_synth_frames(ctx0, a.seed, 0, a.frames, W, H, C.c_void_p(fr.data_ptr()), W, W * H),
          "synth")
    torch.cuda.synchronize()
    f0 = np.ascontiguousarray(fr[0].cpu().numpy())
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc0, u8ptr(f0), W, H, fl)
    xs, ys, vs = (torch.from_numpy(np.asarray(t)).to(dev) for t in fl_to_arrays(fl))
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc0)

    class Rank:
        def __init__(self, world, rank, margin, own=False):
            self.tc = lib.KLTCreateTrackingContext()
            self.tc.contents.sequentialMode = 1
            self.ctx = lib.klt_amd_device_context(self.tc)
            if not own:
                use_torch_stream(lib, self.ctx, dev)
            self.pd, self.td = PyrDesc(), TrackDesc()
            lib.klt_amd_pyr_desc(self.tc, W, H, self.tc.contents.nPyramidLevels, 1, C.byref(self.pd))
            lib.klt_amd_track_desc(self.tc, C.byref(self.td))
            self.band = band_of(H, world, rank, margin, balanced_edges(ys, vs, H, world) if a.balanced else None)
            self.rank = rank

        def ptr(self, t):
            return C.c_void_p(fr.data_ptr() + t * H * W)

        def begin(self, t):
            check(lib, self.ctx, lib.klt_hip_frames_begin(self.ctx, C.byref(self.pd), self.ptr(t), W), "begin")

        def chunk(self, t0, n, x, y, v, esc, full=False, next_n=0):
            b = self.band
            check(lib, self.ctx, lib.klt_hip_track_frames_band(
                self.ctx, C.byref(self.pd), C.byref(self.td), self.ptr(t0), W, H * W, n, C.c_void_p(x.data_ptr()),
                C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), NF, b.own_lo, b.own_hi, 0 if full else b.row_lo,
                H if full else b.row_hi, C.c_void_p(esc.data_ptr()), self.ptr(t0 + n) if next_n > 0 else None,
                next_n), "band")

    T = a.frames - 1
    chunks = [(c0, min(a.chunk, 1 + T - c0)) for c0 in range(1, 1 + T, a.chunk)]

    if a.replay:
        # pass 2 for one rank, alone in this process
        world = int(np.load(a.replay)["world"])
        margin = int(np.load(a.replay)["margin"])
        st = np.load(a.replay)
        own = a.own_streams
        rk = Rank(world, a.rank, margin, own)
        xr, yr, vr = xs.clone(), ys.clone(), vs.clone()
        esc = torch.zeros(1, dtype=torch.int32, device=dev)
        escs = torch.zeros(len(chunks), dtype=torch.int32, device=dev)
        esc_host = torch.zeros(len(chunks), dtype=torch.int32, pin_memory=True)
        esc_ev = [torch.cuda.Event() for _ in chunks]
        sx, sy, sv = (torch.from_numpy(st[k]).to(dev) for k in ("x", "y", "v"))
        for rep in range(3):  # the first two warm the device up (allocations, clocks); the last is timed
            rk.begin(0)
            lib.klt_hip_set_timing(rk.ctx, 1 if rep == 2 else 0)  # per-kernel events of the timed run
            torch.cuda.synchronize()
            t_start = time.perf_counter()
            for ci, (c0, n) in enumerate(chunks):
                nn = chunks[ci + 1][1] if ci + 1 < len(chunks) and not a.no_ahead else 0
                xr.copy_(sx[ci]), yr.copy_(sy[ci]), vr.copy_(sv[ci])
                e = escs[ci:ci + 1] if a.lazy_flag else esc
                e.zero_()
                if own:
                    torch.cuda.current_stream().synchronize()
                rk.chunk(c0, n, xr, yr, vr, e, next_n=nn)
                if own:
                    check(lib, rk.ctx, lib.klt_hip_sync(rk.ctx), "sync")
                if not a.lazy_flag:
                    int(esc.item())  # the host's read of the escape flag (merge_chunk)
                else:
                    esc_host[ci:ci + 1].copy_(e, non_blocking=True)
                    esc_ev[ci].record()
                    if ci > 0:  # chunk c-1's flag, read while chunk c runs
                        esc_ev[ci - 1].synchronize()
                        int(esc_host[ci - 1])
            torch.cuda.synchronize()
        frames_timed = sum(n for _, n in chunks)
        wall = 1e6 * (time.perf_counter() - t_start) / frames_timed
        tm = Timing()
        check(lib, rk.ctx, lib.klt_hip_get_timing(rk.ctx, C.byref(tm)), "timing")
        # per-kernel event time per frame of the timed run (overlapping kernels share the GPU: with
        # build-ahead these are contended durations; with --no-ahead each kernel runs alone)
        kern = {"k_pyr_l0": 1e3 * tm.ms_pyr_l0 / frames_timed, "k_pyr_l1": 1e3 * tm.ms_pyr_l1 / frames_timed,
                "k_track": 1e3 * tm.ms_track / frames_timed}
        print(json.dumps({"rank": a.rank, "us_per_frame": wall, "kernels_us_per_frame": kern}))
        return

    out = {"workload": f"{W}x{H}, {NF} features, {a.frames - 1} tracked frames, {a.chunk}-frame chunks"
                       + (", bands of equal feature counts" if a.balanced else ""),
           "exchange_us_assumed": a.exchange_us, "runs": []}
    base_fps = None
    for margin in a.margins:
        for world in a.worlds:
            ranks = [Rank(world, r, margin) for r in range(1 if a.pass1_shared else world)]
            if a.pass1_shared:
                # one context; each rank's chunk starts from frame c0-1's whole-frame pyramid (band-built
                # rows equal whole-frame ones, so the states are the same) without build-ahead
                for r in range(1, world):
                    rk = Rank.__new__(Rank)
                    rk.__dict__.update(ranks[0].__dict__)
                    rk.band = band_of(H, world, r, margin, balanced_edges(ys, vs, H, world) if a.balanced else None)
                    rk.rank = r
                    ranks.append(rk)
            for rk in ranks[:1] if a.pass1_shared else ranks:
                rk.begin(0)
            x, y, v = xs.clone(), ys.clone(), vs.clone()
            starts, redone, per_rank = [], 0, [[0.0, 0.0, 0.0, 0] for _ in ranks]
            for ci, (c0, n) in enumerate(chunks):
                nn = chunks[ci + 1][1] if ci + 1 < len(chunks) else 0
                state = (x.clone(), y.clone(), v.clone())
                starts.append(state)
                outs, esc_any = [], 0
                for i, rk in enumerate(ranks):
                    xr, yr, vr = (t.clone() for t in state)
                    esc = torch.zeros(1, dtype=torch.int32, device=dev)
                    lib.klt_hip_set_timing(rk.ctx, 1)
                    if a.pass1_shared:
                        rk.begin(c0 - 1)
                    rk.chunk(c0, n, xr, yr, vr, esc, next_n=0 if a.pass1_shared else nn)
                    tm = Timing()
                    check(lib, rk.ctx, lib.klt_hip_get_timing(rk.ctx, C.byref(tm)), "timing")
                    lib.klt_hip_set_timing(rk.ctx, 0)
                    pr = per_rank[i]
                    pr[0] += tm.ms_pyr_l0 * 1e3
                    pr[1] += tm.ms_pyr_l1 * 1e3
                    pr[2] += tm.ms_track * 1e3
                    pr[3] += n
                    esc_any += int(esc.item())
                    outs.append((xr, yr, vr))
                if esc_any:
                    redone += 1
                    outs = []
                    for rk in ranks:
                        xr, yr, vr = (t.clone() for t in state)
                        esc = torch.zeros(1, dtype=torch.int32, device=dev)
                        rk.begin(c0 - 1)
                        rk.chunk(c0, n, xr, yr, vr, esc, full=True, next_n=0 if a.pass1_shared else nn)
                        outs.append((xr, yr, vr))
                acc = None
                for rk, (xr, yr, vr) in zip(ranks, outs):
                    parts = []
                    merge_chunk(xr, yr, vr, state[1], state[2], rk.band, rk.rank, lambda t, p=parts: p.append(t.clone()))
                    acc = parts[0] if acc is None else acc + parts[0]
                x.view(torch.int32).copy_(acc[0]), y.view(torch.int32).copy_(acc[1]), v.copy_(acc[2])
            digest = int((x.view(torch.int32).to(torch.int64).sum() * 3 + y.view(torch.int32).to(torch.int64).sum() * 5
                          + v.to(torch.int64).sum() * 7).item())
            # pass 2: each rank alone over the whole schedule, in a process of its own
            # (the third of three runs timed: allocations and clocks settle first)
            import subprocess
            import tempfile
            with tempfile.TemporaryDirectory() as td:
                f = f"{td}/states.npz"
                np.savez(f, world=world, margin=margin,
                         x=np.stack([t[0].cpu().numpy() for t in starts]),
                         y=np.stack([t[1].cpu().numpy() for t in starts]),
                         v=np.stack([t[2].cpu().numpy() for t in starts]))
                if a.keep_states:
                    import shutil
                    os.makedirs(a.keep_states, exist_ok=True)
                    shutil.copy(f, f"{a.keep_states}/states_w{world}.npz")
                rank_us, rank_kern = [], []
                for r in range(world):
                    cmd = [sys.executable, __file__, "--replay", f, "--rank", str(r), "--width", str(W), "--height",
                           str(H), "--features", str(NF), "--frames", str(a.frames), "--chunk", str(a.chunk),
                           "--seed", str(a.seed)] + (["--no-ahead"] if a.no_ahead else []) + \
                          (["--own-streams"] if a.own_streams else []) + (["--balanced"] if a.balanced else []) + \
                          (["--lazy-flag"] if a.lazy_flag else [])
                    res = subprocess.run(cmd, check=True, capture_output=True, text=True)
                    rr = json.loads(res.stdout.strip().splitlines()[-1])
                    rank_us.append(rr["us_per_frame"])
                    rank_kern.append(rr["kernels_us_per_frame"])
            nch = len(chunks)
            frames = sum(n for _, n in chunks)
            exch = a.exchange_us * nch / frames if world > 1 else 0.0
            fps = 1e6 / (max(rank_us) + exch)
            if world == 1:
                base_fps = fps
            run = {"world": world, "margin_rows": margin, "chunks_redone_full_frame": redone,
                   "state_digest": digest, "us_per_frame_max_rank": max(rank_us),
                   "us_per_frame_exchange": exch, "projected_fps": fps,
                   "projected_speedup": fps / base_fps if base_fps else None,
                   "per_rank_us_per_frame": [{"rank": i, "band_rows": [rk.band.row_lo, rk.band.row_hi],
                                              "wall": rank_us[i], "replay_kernels": rank_kern[i],
                                              "k_pyr_l0": p[0] / p[3], "k_pyr_l1": p[1] / p[3], "k_track": p[2] / p[3]}
                                             for i, (rk, p) in enumerate(zip(ranks, per_rank))]}
            out["runs"].append(run)
            print(json.dumps({k: run[k] for k in ("world", "margin_rows", "chunks_redone_full_frame", "state_digest",
                                                  "us_per_frame_max_rank", "projected_fps", "projected_speedup")}),
                  flush=True)
            for rk in ranks[:1] if a.pass1_shared else ranks:
                lib.KLTFreeTrackingContext(rk.tc)
            torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
