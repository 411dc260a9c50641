#!/usr/bin/env python3
"""Config 4 (feature-sharded 4K sequence) on ONE GPU: the projected 1 -> N
GPU curve of kltamd.shard.ShardedSequence, measured per rank.

Pass 1 runs every rank of an N-rank row-band decomposition in turn per chunk
(klt_hip_track_frames_band, the next chunk built ahead) and merges them with
the exchange's own device kernels (klt_hip_gather_order/pack/unpack): every N
must end in the same feature state bit for bit (the state digest), and the
all-gathered slots of every chunk are kept.  Pass 2 runs, for each rank in a
process of its own (one device context, as on an N-GPU node), the production
driver itself -- ShardedSequence.run over the whole sequence, speculative
(chunk c+1 queued before chunk c's verdict is read), band pyramids built
ahead -- with only the RCCL transfer replaced by a copy of pass 1's gathered
slots for that chunk.  It is timed by the host clock, and per chunk by an
event after each exchange.  Since the collective makes every rank wait for
the slowest one every chunk, the projected N-GPU frame time is

    sum over chunks of max over ranks (chunk time) + exchange(N)

(reported beside the looser max over ranks of each rank's own total), with
the exchange (an all-gather of the ranks' slots plus its latency) from
--exchange-us per chunk, since one GPU cannot measure RCCL over xGMI.
usage: python tools/shard_sim.py [--worlds 1 8] [--margins 64] [--frames 1001] [--chunk 64]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
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
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--first-chunk", type=int, default=None, help="first chunk's frames (default: chunk)")
    ap.add_argument("--track-prio", type=int, default=None,
                    help="replays: klt_hip_set_track_prio (default: the library's, raised)")
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--margins", type=int, nargs="+", default=[64])
    ap.add_argument("--seed", type=int, default=2160)
    ap.add_argument("--edges", default=None, help="explicit band edges for the largest world, comma-separated "
                    "(overrides --bands there)")
    ap.add_argument("--bands", choices=["equal", "features", "rows", "cost"], default="rows",
                    help="band edges: equal rows, equal feature counts (balanced_edges), or equal level-0 rows "
                         "built incl. margins (row_edges), or rows built and features owned together (cost_edges)")
    ap.add_argument("--keep-states", default=None, help="save pass 1's record as DIR/states_w<N>.npz")
    ap.add_argument("--pass1-shared", action="store_true",
                    help="pass 1 through one device context for every rank, each chunk started from a "
                         "whole-frame pyramid: one bank arena instead of N (long chunks at 4K)")
    ap.add_argument("--replay", default=None, help=argparse.SUPPRESS)  # internal: pass 2 of one rank
    ap.add_argument("--rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--exchange-us", type=float, default=40.0,
                    help="assumed per-chunk exchange at N > 1: an all-gather of the ranks' slots over xGMI")
    ap.add_argument("--exchange-in-stream-us", type=float, default=0.0,
                    help="model the all-gather's latency in the schedule instead of adding --exchange-us per chunk: "
                         "a device-side stall of this many us (torch.cuda._sleep, calibrated) in the all-gather's "
                         "place on the tracking stream of every replayed rank at N > 1")
    a = ap.parse_args()

    import torch
    import kltamd
    from kltamd.device import PyrDesc, Timing, TrackDesc, check, use_torch_stream
    from kltamd.shard import (FullFrames, ShardedSequence, balanced_edges, band_edges, band_of, chunk_plan,
                              cost_edges, row_edges, slot_words)
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

    T = a.frames - 1
    chunks = chunk_plan(1, T, a.chunk, a.first_chunk)  # the production driver's plan

    def descs(tc):
        pd, td = PyrDesc(), TrackDesc()
        lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
        lib.klt_amd_track_desc(tc, C.byref(td))
        return pd, td

    if a.replay:
        # pass 2 for one rank, alone in this process: the production driver,
        # its all-gather replaced by pass 1's gathered slots of each chunk
        rec = np.load(a.replay)
        world, margin = int(rec["world"]), int(rec["margin"])
        edges = [int(e) for e in rec["row_edges"]] if len(rec["row_edges"]) else None
        flat = torch.from_numpy(rec["slots"]).to(dev)
        offs = rec["slot_offsets"]
        tc = lib.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        ctx = lib.klt_amd_device_context(tc)
        use_torch_stream(lib, ctx, dev)
        if a.track_prio is not None:
            check(lib, ctx, lib.klt_hip_set_track_prio(ctx, a.track_prio), "track_prio")
        pd, td = descs(tc)
        k = [0]
        stall_cycles = 0
        if a.exchange_in_stream_us > 0 and world > 1:
            # calibrate torch.cuda._sleep (shader-clock cycles) to microseconds
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            per_us = []
            for _ in range(5):
                e0.record()
                torch.cuda._sleep(200000)
                e1.record()
                e1.synchronize()
                per_us.append(200000 / (e0.elapsed_time(e1) * 1e3))
            stall_cycles = int(a.exchange_in_stream_us * sorted(per_us)[len(per_us) // 2])

        def replay_gather(out, inp):  # chunk k's slots as RCCL would have delivered them
            s0, s1 = int(offs[k[0]]), int(offs[k[0] + 1])
            torch.add(flat[s0:s1], 0, out=out[:s1 - s0])  # a compute kernel, as RCCL's all-gather is
            if stall_cycles:
                torch.cuda._sleep(stall_cycles)  # the collective's latency, in its place in stream order
            k[0] += 1

        ev_start = torch.cuda.Event(enable_timing=True)
        # runs 0-1 warm the device up (allocations, clocks); run 2 is timed (host
        # clock, an event after every exchange); run 3 records per-kernel events
        # (their own markers cost time on the stream, so not in the timed run)
        for rep in range(4):
            x, y, v = xs.clone(), ys.clone(), vs.clone()
            k[0] = 0
            seq = ShardedSequence(lib, ctx, pd, td, FullFrames(fr), x, y, v, a.rank, world, replay_gather,
                                  chunk=a.chunk, margin=margin, edges=edges, first_chunk=a.first_chunk)
            seq.xch.timing = rep == 2
            seq.begin(0)
            lib.klt_hip_set_timing(ctx, 1 if rep == 3 else 0)
            torch.cuda.synchronize()
            ev_start.record()
            t_start = time.perf_counter()
            seq.run(1, T)
            torch.cuda.synchronize()
            if rep == 2:
                wall = time.perf_counter() - t_start
                evs = [ev_start] + seq.xch.timing_events
                per_chunk = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(len(evs) - 1)]  # us
                redone = seq.redone
        tm = Timing()
        check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
        # per-kernel event time per frame (build-ahead: contended durations)
        kern = {"k_pyr_l0": 1e3 * tm.ms_pyr_l0 / T, "k_pyr_l1": 1e3 * tm.ms_pyr_l1 / T,
                "k_track": 1e3 * tm.ms_track / T}
        print(json.dumps({"rank": a.rank, "us_per_frame": 1e6 * wall / T, "chunk_us": per_chunk,
                          "kernels_us_per_frame": kern, "redone": redone,
                          "digest": int((x.view(torch.int32).to(torch.int64).sum() * 3 +
                                         y.view(torch.int32).to(torch.int64).sum() * 5 +
                                         v.to(torch.int64).sum() * 7).item())}))
        lib.KLTFreeTrackingContext(tc)
        return

    class Rank:
        def __init__(self, world, rank, margin, edges):
            self.tc = lib.KLTCreateTrackingContext()
            self.tc.contents.sequentialMode = 1
            self.ctx = lib.klt_amd_device_context(self.tc)
            use_torch_stream(lib, self.ctx, dev)
            self.pd, self.td = descs(self.tc)
            self.band = band_of(H, world, rank, margin, edges)
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

    out = {"workload": f"{W}x{H}, {NF} features, {T} tracked frames, {a.chunk}-frame chunks"
                       + {"equal": "", "features": ", bands of equal feature counts",
                          "rows": ", bands of equal built rows",
                          "cost": ", bands of equal built rows + features owned"}[a.bands],
           "exchange_us_assumed_per_chunk": a.exchange_us, "runs": []}
    base = None
    for margin in a.margins:
        for world in a.worlds:
            explicit = [int(e) for e in a.edges.split(",")] if a.edges else None
            edges = (explicit if explicit and len(explicit) == world + 1 else
                     balanced_edges(ys, vs, H, world) if a.bands == "features" else
                     row_edges(H, world, margin) if a.bands == "rows" else
                     cost_edges(ys, vs, H, world, margin) if a.bands == "cost" else
                     [r * H // world for r in range(world + 1)])
            gedges = band_edges(H, world, edges)
            ranks = [Rank(world, r, margin, edges) for r in range(1 if a.pass1_shared else world)]
            if a.pass1_shared:
                for r in range(1, world):
                    rk = Rank.__new__(Rank)
                    rk.__dict__.update(ranks[0].__dict__)
                    rk.band = band_of(H, world, r, margin, edges)
                    rk.rank = r
                    ranks.append(rk)
            for rk in ranks[:1] if a.pass1_shared else ranks:
                rk.begin(0)
            ctx = ranks[0].ctx
            x, y, v = xs.clone(), ys.clone(), vs.clone()
            redone, slots_rec, owned_rec = 0, [], []
            work = torch.zeros(lib.klt_hip_gather_work_ints(NF, world), dtype=torch.int32, device=dev)
            E = (C.c_float * (world + 1))(*gedges)
            flags = torch.zeros(2, dtype=torch.int32, device=dev)
            for ci, (c0, n) in enumerate(chunks):
                nn = chunks[ci + 1][1] if ci + 1 < len(chunks) else 0
                state = (x.clone(), y.clone(), v.clone())
                outs, escs = [], []
                for rk in ranks:
                    xr, yr, vr = (t.clone() for t in state)
                    esc = torch.zeros(1, dtype=torch.int32, device=dev)
                    if a.pass1_shared:
                        rk.begin(c0 - 1)
                    rk.chunk(c0, n, xr, yr, vr, esc, next_n=0 if a.pass1_shared else nn)
                    outs.append((xr, yr, vr))
                    escs.append(esc)
                if sum(int(e.item()) for e in escs):
                    redone += 1
                    outs = []
                    for rk, esc in zip(ranks, escs):
                        xr, yr, vr = (t.clone() for t in state)
                        esc.zero_()
                        rk.begin(c0 - 1)
                        rk.chunk(c0, n, xr, yr, vr, esc, full=True, next_n=0 if a.pass1_shared else nn)
                        outs.append((xr, yr, vr))
                # the exchange with its own kernels: order, each rank's slot, unpack
                check(lib, ctx, lib.klt_hip_gather_order(ctx, None, C.c_void_p(state[1].data_ptr()),
                                                         C.c_void_p(state[2].data_ptr()), NF, E, world,
                                                         C.c_void_p(work.data_ptr()), None, None, None), "order")
                owned_rec.append(work[NF:NF + world].cpu().tolist())  # each rank's features at the chunk's start
                S = max(1, int(max(owned_rec[-1])))
                Wd = slot_words(S)
                slots = torch.zeros(world * Wd, dtype=torch.int32, device=dev)
                for r, ((xr, yr, vr), esc) in enumerate(zip(outs, escs)):
                    check(lib, ctx, lib.klt_hip_gather_pack(
                        ctx, C.c_void_p(xr.data_ptr()), C.c_void_p(yr.data_ptr()), C.c_void_p(vr.data_ptr()),
                        C.c_void_p(work.data_ptr()), NF, world, r, C.c_void_p(esc.data_ptr()), 0,
                        C.c_void_p(slots[r * Wd:].data_ptr()), S), "pack")
                check(lib, ctx, lib.klt_hip_gather_unpack(ctx, C.c_void_p(slots.data_ptr()), world, 0,
                                                          C.c_void_p(work.data_ptr()), NF, world, S,
                                                          C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                                                          C.c_void_p(v.data_ptr()), C.c_void_p(flags.data_ptr()),
                                                          None), "unpack")
                assert int(flags[1].item()) == 0
                slots_rec.append(slots.cpu().numpy())
            digest = int((x.view(torch.int32).to(torch.int64).sum() * 3 + y.view(torch.int32).to(torch.int64).sum() * 5
                          + v.to(torch.int64).sum() * 7).item())
            for rk in ranks[:1] if a.pass1_shared else ranks:
                lib.KLTFreeTrackingContext(rk.tc)
            torch.cuda.synchronize()
            # pass 2: each rank alone over the whole schedule, in a process of its own
            reps = []
            with tempfile.TemporaryDirectory() as td:
                f = f"{td}/rec.npz"
                offs = np.cumsum([0] + [len(s) for s in slots_rec])
                np.savez(f, world=world, margin=margin, row_edges=np.asarray(edges if edges else [], np.int64),
                         slots=np.concatenate(slots_rec), slot_offsets=offs)
                if a.keep_states:
                    import shutil
                    os.makedirs(a.keep_states, exist_ok=True)
                    shutil.copy(f, f"{a.keep_states}/states_w{world}.npz")
                for r in range(world):
                    cmd = [sys.executable, __file__, "--replay", f, "--rank", str(r), "--width", str(W), "--height",
                           str(H), "--features", str(NF), "--frames", str(a.frames), "--chunk", str(a.chunk),
                           "--seed", str(a.seed), "--exchange-in-stream-us", str(a.exchange_in_stream_us)] + (
                        [] if a.first_chunk is None else
                                                     ["--first-chunk", str(a.first_chunk)]) + (
                        [] if a.track_prio is None else ["--track-prio", str(a.track_prio)])
                    res = subprocess.run(cmd, check=True, capture_output=True, text=True)
                    reps.append(json.loads(res.stdout.strip().splitlines()[-1]))
            frames = sum(n for _, n in chunks)
            nch = len(chunks)
            assert all(len(rr["chunk_us"]) == nch for rr in reps)
            assert all(rr["digest"] == digest for rr in reps), "a replayed rank ended in another state"
            # the exchange either added per chunk (conservative: as if nothing hid it) or already inside
            # the measured chunk times (--exchange-in-stream-us)
            exch = a.exchange_us * nch / frames if world > 1 and a.exchange_in_stream_us <= 0 else 0.0
            synced = sum(max(rr["chunk_us"][c] for rr in reps) for c in range(nch)) / frames
            loose = max(rr["us_per_frame"] for rr in reps)
            fps = 1e6 / (synced + exch)
            if world == 1:
                base = fps
            run = {"world": world, "margin_rows": margin, "chunks_redone_full_frame": redone,
                   "exchange_model": (f"in stream: a {a.exchange_in_stream_us:g} us device stall in the all-gather's "
                                      "place, inside the measured chunk times" if a.exchange_in_stream_us > 0
                                      else f"added: {a.exchange_us:g} us per chunk on top of the measured chunk times"),
                   "state_digest": digest, "us_per_frame_synced": synced, "us_per_frame_max_rank_total": loose,
                   "us_per_frame_exchange": exch, "projected_fps": fps,
                   "projected_speedup": fps / base if base else None,
                   "per_rank": [{"rank": i, "band_rows": [band_of(H, world, i, margin, edges).row_lo,
                                                          band_of(H, world, i, margin, edges).row_hi],
                                 "wall_us_per_frame": rr["us_per_frame"],
                                 "owned_features_mean": float(np.mean([c[i] for c in owned_rec])),
                                 "chunk_us_mean": float(np.mean(rr["chunk_us"])),
                                 "replay_kernels_us_per_frame": rr["kernels_us_per_frame"], "redone": rr["redone"]}
                                for i, rr in enumerate(reps)],
                   "chunk_us_max_over_ranks": [max(rr["chunk_us"][c] for rr in reps) for c in range(nch)]}
            out["runs"].append(run)
            print(json.dumps({k: run[k] for k in ("world", "margin_rows", "chunks_redone_full_frame", "state_digest",
                                                  "exchange_model",
                                                  "us_per_frame_synced", "us_per_frame_max_rank_total",
                                                  "projected_fps", "projected_speedup")}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
