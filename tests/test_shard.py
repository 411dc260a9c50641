"""Feature-sharded mode (BASELINE config 4): the exchange logic on CPU with a
real world-size-2 gloo process group, band bookkeeping, and (GPU) bit-exact
equality of the sharded sequence with the single-GPU one."""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import synth

import kltamd  # noqa: F401  (package import path)
from kltamd.shard import Band, band_edges, band_of, gather_merge_ref, gather_order_ref, owned_mask, row_edges


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_chunk_plan():
    """chunk_plan: the first chunk's length (default: chunk), then whole
    chunks; contiguous and covering the frames exactly."""
    from kltamd.shard import chunk_plan
    assert chunk_plan(1, 1000, 64, 16)[:3] == [(1, 16), (17, 64), (81, 64)]
    assert chunk_plan(1, 1000, 64)[:2] == [(1, 64), (65, 64)] and chunk_plan(1, 1000, 64)[-1] == (961, 40)
    assert chunk_plan(5, 3, 64) == [(5, 3)] and chunk_plan(5, 0, 64) == [] and chunk_plan(1, 2, 1) == [(1, 1), (2, 1)]
    for t0, n, c, f in [(1, 1000, 64, None), (3, 129, 32, 5), (0, 7, 4, 100), (2, 65, 64, 1)]:
        p = chunk_plan(t0, n, c, f)
        assert p[0][0] == t0 and sum(k for _, k in p) == n and all(k <= c for _, k in p)
        assert all(a0 + k == b0 for (a0, k), (b0, _) in zip(p, p[1:]))


@pytest.mark.parametrize("H", [7, 100, 251, 480, 1080, 2160, 4320])
def test_row_edges_c_equals_python(amd, H):
    """klt_shard_band_edges (the C driver's bands) == kltamd.shard.row_edges
    for every world size and several margins; the bands partition the rows,
    and no rank builds more level-0 rows than with equal bands by more than a
    tile (at 4K / 8 ranks / margin 64: 384 against 448)."""
    from kltamd.shard import built_rows
    for world in range(1, 17):
        for margin in (0, 1, 16, 48, 64, 100):
            e = (C.c_int * (world + 1))()
            assert amd.klt_shard_band_edges(H, world, margin, e) == 0
            py = row_edges(H, world, margin)
            assert list(e) == py, (H, world, margin, list(e), py)
            assert py[0] == 0 and py[-1] == H and all(b > a for a, b in zip(py, py[1:])) or H < world
            eq = [r * H // world for r in range(world + 1)]
            cost = max(built_rows(H, band_of(H, world, r, margin, py)) for r in range(world))
            cost_eq = max(built_rows(H, band_of(H, world, r, margin, eq)) for r in range(world))
            assert cost <= cost_eq + 32, (H, world, margin, cost, cost_eq)
    assert max(built_rows(2160, band_of(2160, 8, r, 64, row_edges(2160, 8, 64))) for r in range(8)) == 384
    e = (C.c_int * 20)()
    assert amd.klt_shard_band_edges(2160, 17, 64, e) == -1 and amd.klt_shard_band_edges(0, 2, 64, e) == -1


@pytest.mark.parametrize("H,world", [(480, 2), (2160, 8), (251, 3), (7, 4)])
def test_bands_partition_rows_and_features(H, world):
    bands = [band_of(H, world, r, margin=16) for r in range(world)]
    assert bands[0].own_lo == float("-inf") and bands[-1].own_hi == float("inf")
    for a, b in zip(bands, bands[1:]):
        assert a.own_hi == b.own_lo
    for b in bands:
        assert 0 <= b.row_lo <= b.row_hi <= H
    rng = np.random.default_rng(world)
    y = torch.from_numpy(np.concatenate([rng.uniform(-5, H + 5, 500), [0.0, H - 1e-3, float(H)]]).astype(np.float32))
    v = torch.from_numpy(rng.integers(-5, 1, y.numel()).astype(np.int32))
    owners = sum(owned_mask(y, v, b).int() for b in bands)
    assert torch.equal(owners, (v >= 0).int())  # every live feature has exactly one owner


def _state(n=64, seed=7):
    g = torch.Generator().manual_seed(seed)
    y0 = torch.rand(n, generator=g) * 100
    v0 = torch.where(torch.rand(n, generator=g) < 0.2, torch.full((n,), -1), torch.zeros(n, dtype=torch.int64))
    v0 = v0.to(torch.int32)
    x0 = torch.rand(n, generator=g) * 100
    return x0, y0, v0


def _tracked(x0, y0, v0, world, rank):
    """each rank "tracks" its own features: a rank-specific result; others stale"""
    owned = owned_mask(y0, v0, band_of(100, world, rank, margin=0))
    x, y, v = x0.clone(), y0.clone(), v0.clone()
    x[owned] = x0[owned] + 1000 * (rank + 1)
    y[owned] = -1.0
    v[owned] = -3 - rank
    return x, y, v


def _merge_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x0, y0, v0 = _state()
        x, y, v = _tracked(x0, y0, v0, world, rank)

        def all_gather(out, inp):
            parts = [torch.empty_like(inp) for _ in range(world)]
            dist.all_gather(parts, inp)
            out.copy_(torch.cat(parts))
        esc = gather_merge_ref(x, y, v, y0.clone(), v0.clone(), band_edges(100, world), rank, all_gather,
                               escape=rank + 1)
        q.put((rank, x.numpy(), y.numpy(), v.numpy(), esc))
    finally:
        dist.destroy_process_group()


def test_gather_order_ref_partitions_live_features():
    """Every live feature has exactly one owner; places are 0 .. count-1 in
    index order within each owner; lost features are nobody's."""
    x0, y0, v0 = _state(300, 3)
    for world in (1, 2, 3, 8):
        edges = band_edges(100, world)
        owner, place, counts = gather_order_ref(y0, v0, edges)
        assert torch.equal(owner >= 0, v0 >= 0)
        for r in range(world):
            m = owner == r
            assert torch.equal(m, owned_mask(y0, v0, band_of(100, world, r, 0)))
            assert place[m].tolist() == list(range(counts[r]))
        assert sum(counts) == int((v0 >= 0).sum())


def test_merge_chunk_gloo_world2():
    """The exchange over a real world-size-2 gloo group (CPU): each rank's
    slot of its owned features, all-gathered, merged identically on both."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_merge_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    # the escape flags ride along in the slots' headers: summed on every rank
    assert [r[4] for r in res] == [3, 3]
    # both ranks hold identical arrays ...
    for a, b in zip(res[0][1:4], res[1][1:4]):
        assert np.array_equal(a.view(np.int32), b.view(np.int32))
    # ... equal to the owners' values (lost features as they were)
    x0, y0, v0 = _state()
    x, y, v = x0.clone(), y0.clone(), v0.clone()
    for r in range(world):
        own = owned_mask(y0, v0, band_of(100, world, r, margin=0))
        xr, yr, vr = _tracked(x0, y0, v0, world, r)
        x[own], y[own], v[own] = xr[own], yr[own], vr[own]
    assert np.array_equal(res[0][1].view(np.int32), x.numpy().view(np.int32))
    assert np.array_equal(res[0][2].view(np.int32), y.numpy().view(np.int32))
    assert np.array_equal(res[0][3], v.numpy())


# ---------------------------------------------------------------------------
# GPU: ranks simulated one after another in one process (one context each)
# ---------------------------------------------------------------------------
def _select(gpu, frame, nfeat):
    from kltabi import fl_to_arrays, u8ptr
    h, w = frame.shape
    tc = gpu.KLTCreateTrackingContext()
    fl = gpu.KLTCreateFeatureList(nfeat)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(frame)), w, h, fl)
    x, y, v = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    gpu.KLTFreeTrackingContext(tc)
    return x, y, v


class _Rank:
    def __init__(self, gpu, dfr, H, W, world, rank, margin, edges=None):
        from kltamd.device import PyrDesc, TrackDesc
        self.gpu, self.dfr, self.H, self.W = gpu, dfr, H, W
        self.tc = gpu.KLTCreateTrackingContext()
        self.tc.contents.sequentialMode = 1
        self.ctx = gpu.klt_amd_device_context(self.tc)
        from kltamd.device import use_torch_stream
        use_torch_stream(gpu, self.ctx)
        self.pd, self.td = PyrDesc(), TrackDesc()
        gpu.klt_amd_pyr_desc(self.tc, W, H, self.tc.contents.nPyramidLevels, 1, C.byref(self.pd))
        gpu.klt_amd_track_desc(self.tc, C.byref(self.td))
        self.band = band_of(H, world, rank, margin, edges)
        self.rank = rank
        self.src = None

    def band_only(self):
        """Hold only the band's rows of every frame (kltamd.shard.BandFrames), copied from the full frames."""
        from kltamd.shard import BandFrames
        dfr, W = self.dfr, self.W

        def load(t0, n, row0, nrows, dst, stride):
            from kltamd.device import D2D, check
            part = dfr[t0:t0 + n, row0:row0 + nrows].contiguous()  # [n, nrows, W]
            for f in range(n):
                check(self.gpu, self.ctx, self.gpu.klt_hip_memcpy(
                    self.ctx, C.c_void_p(dst + f * stride), C.c_void_p(part[f].data_ptr()), nrows * W, D2D), "d2d")
            self.gpu.klt_hip_sync(self.ctx)

        self.src = BandFrames(dfr.shape[0], self.H, W, self.band, load, dfr.device)

    def ptr(self, t):
        if self.src is not None:
            return C.c_void_p(self.src.band(t))
        return C.c_void_p(self.dfr.data_ptr() + t * self.H * self.W)

    def begin(self, t):
        ptr = self.src.full(t, 1)[0] if self.src is not None else self.dfr.data_ptr() + t * self.H * self.W
        assert self.gpu.klt_hip_frames_begin(self.ctx, C.byref(self.pd), C.c_void_p(ptr), self.W) == 0

    def chunk(self, t0, n, x, y, v, esc, full=False, next_n=0):
        """next_n > 0: frames t0+n .. are the next chunk, built ahead (klt_hip_track_frames_band's next_frames)"""
        b = self.band
        if full and self.src is not None:  # a redone chunk: whole frames from the source's scratch
            ptr, stride = self.src.full(t0, n)
            first, nxt, next_n = C.c_void_p(ptr), None, 0
        else:
            stride = self.src.stride if self.src is not None else self.H * self.W
            first, nxt = self.ptr(t0), (self.ptr(t0 + n) if next_n > 0 else None)
        rc = self.gpu.klt_hip_track_frames_band(
            self.ctx, C.byref(self.pd), C.byref(self.td), first, self.W, stride, n,
            C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), x.numel(),
            b.own_lo, b.own_hi, 0 if full else b.row_lo, self.H if full else b.row_hi, C.c_void_p(esc.data_ptr()),
            nxt, next_n)
        assert rc == 0, self.gpu.klt_hip_last_error(self.ctx)


def device_gather_merge(gpu, ctx, state, outs, edges, escapes=None):
    """The exchange of simulated ranks with the device kernels: order the
    chunk-start state, pack each rank's result into its slot, unpack the
    stacked slots into a copy of the start state.  Returns (x, y, v)."""
    from kltamd.device import check
    from kltamd.shard import slot_words
    world = len(outs)
    n = state[0].numel()
    dev = state[0].device
    work = torch.zeros(gpu.klt_hip_gather_work_ints(n, world), dtype=torch.int32, device=dev)
    E = (C.c_float * (world + 1))(*edges)
    check(gpu, ctx, gpu.klt_hip_gather_order(ctx, None, C.c_void_p(state[1].data_ptr()),
                                             C.c_void_p(state[2].data_ptr()), n, E, world,
                                             C.c_void_p(work.data_ptr()), None, None, None), "order")
    S = max(1, int(work[n:n + world].max().item()))
    W = slot_words(S)
    slots = torch.zeros(world * W, dtype=torch.int32, device=dev)
    for r, (xr, yr, vr) in enumerate(outs):
        esc = escapes[r] if escapes is not None else None
        check(gpu, ctx, gpu.klt_hip_gather_pack(ctx, C.c_void_p(xr.data_ptr()), C.c_void_p(yr.data_ptr()),
                                                C.c_void_p(vr.data_ptr()), C.c_void_p(work.data_ptr()), n, world, r,
                                                C.c_void_p(esc.data_ptr()) if esc is not None else None, 0,
                                                C.c_void_p(slots[r * W:].data_ptr()), S), "pack")
    x, y, v = (t.clone() for t in state)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    check(gpu, ctx, gpu.klt_hip_gather_unpack(ctx, C.c_void_p(slots.data_ptr()), world, 0,
                                              C.c_void_p(work.data_ptr()), n, world, S, C.c_void_p(x.data_ptr()),
                                              C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()),
                                              C.c_void_p(flags.data_ptr()), None), "unpack")
    assert int(flags[1].item()) == 0
    device_gather_merge.flags = flags.cpu().tolist()
    return x, y, v


@pytest.mark.gpu
@pytest.mark.parametrize("world,n", [(1, 5003), (2, 5003), (3, 5003), (8, 5003), (8, 45001), (15, 20480)])
def test_gather_kernels_equal_reference(gpu, world, n):
    """klt_hip_gather_order/pack/unpack against the torch restatement
    (gather_merge_ref): random chunk-start states with lost features, y
    exactly on band edges, NaN and out-of-frame y, a rank owning nothing;
    the escape flags summed in the slots' headers."""
    from kltamd.device import check
    H = 480
    rng = np.random.default_rng(world)
    y0 = rng.uniform(-10, H + 10, n).astype(np.float32)
    y0[:world + 1] = [r * H // world for r in range(world + 1)]  # on the edges
    y0[world + 1] = np.nan
    if world > 2:
        y0[(y0 >= H // world) & (y0 < 2 * H // world)] = 1.0  # rank 1 owns nothing
    v0 = np.where(rng.uniform(size=n) < 0.15, -1, 0).astype(np.int32)
    x0 = rng.uniform(0, 640, n).astype(np.float32)
    edges = band_edges(H, world)
    # each rank's "result": its owned features moved by a rank-specific amount
    res = []
    for r in range(world):
        own = owned_mask(torch.from_numpy(y0), torch.from_numpy(v0), band_of(H, world, r, 0))
        x, y, v = torch.from_numpy(x0.copy()), torch.from_numpy(y0.copy()), torch.from_numpy(v0.copy())
        x[own] += 1000.0 * (r + 1)
        y[own] = -2.5 * (r + 1)
        v[own] = -7 - r
        res.append((x, y, v))
    # torch reference: rank r's slot from its own result; all ranks' slots stacked
    slots_ref = []
    ref = None
    for r in range(world):
        st = [t.clone() for t in res[r]]

        def ag(out, inp, r=r):
            slots_ref.append(inp.clone())
            out.zero_()
        gather_merge_ref(*st, torch.from_numpy(y0), torch.from_numpy(v0), edges, r, ag, escape=r)
    stacked = torch.cat(slots_ref)
    x, y, v = torch.from_numpy(x0.copy()), torch.from_numpy(y0.copy()), torch.from_numpy(v0.copy())
    esc_ref = gather_merge_ref(x, y, v, torch.from_numpy(y0), torch.from_numpy(v0), edges, 0,
                               lambda out, inp: out.copy_(stacked), escape=0)
    ref = (x, y, v)
    dev = torch.device("cuda", 0)
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    from kltamd.device import use_torch_stream
    use_torch_stream(gpu, ctx, dev)  # the kernels and torch's allocations and reads on one stream
    state = tuple(torch.from_numpy(a.copy()).to(dev) for a in (x0, y0, v0))
    outs = [tuple(t.to(dev) for t in rr) for rr in res]
    escs = [torch.tensor([r], dtype=torch.int32, device=dev) for r in range(world)]
    got = device_gather_merge(gpu, ctx, state, outs, edges, escs)
    for g, w in zip(got, ref):
        assert np.array_equal(g.cpu().numpy().view(np.int32), w.numpy().view(np.int32))
    assert device_gather_merge.flags == [sum(range(world)), 0] == [esc_ref, 0]
    # the fused step (unpack + the next order, klt_hip_gather_unpack_order) on the same slots: the same
    # merged state, its start state saved, the escape flag zeroed, and the merged state's counts
    from kltamd.shard import slot_words
    E = (C.c_float * (world + 1))(*edges)
    work = torch.zeros(gpu.klt_hip_gather_work_ints(n, world), dtype=torch.int32, device=dev)
    assert gpu.klt_hip_gather_order(ctx, None, C.c_void_p(state[1].data_ptr()), C.c_void_p(state[2].data_ptr()), n,
                                    E, world, C.c_void_p(work.data_ptr()), None, None, None) == 0
    S = max(1, int(work[n:n + world].max().item()))
    Wd = slot_words(S)
    slots = torch.zeros(world * Wd, dtype=torch.int32, device=dev)
    for r, (xr, yr, vr) in enumerate(outs):
        assert gpu.klt_hip_gather_pack(ctx, C.c_void_p(xr.data_ptr()), C.c_void_p(yr.data_ptr()),
                                       C.c_void_p(vr.data_ptr()), C.c_void_p(work.data_ptr()), n, world, r,
                                       C.c_void_p(escs[r].data_ptr()), 0, C.c_void_p(slots[r * Wd:].data_ptr()),
                                       S) == 0
    x, y, v = (t.clone() for t in state)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    save = torch.zeros(3 * n, dtype=torch.int32, device=dev)
    esc = torch.ones(1, dtype=torch.int32, device=dev)
    hc = torch.zeros(world, dtype=torch.int32).pin_memory()
    assert gpu.klt_hip_gather_unpack_order(ctx, C.c_void_p(slots.data_ptr()), world, 0, C.c_void_p(work.data_ptr()), n,
                                           world, S, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                                           C.c_void_p(v.data_ptr()), C.c_void_p(flags.data_ptr()), None, E,
                                           C.c_void_p(save.data_ptr()), C.c_void_p(esc.data_ptr()),
                                           C.c_void_p(hc.data_ptr())) == 0
    torch.cuda.synchronize()
    for g, w in zip((x, y, v), ref):
        assert np.array_equal(g.cpu().numpy().view(np.int32), w.numpy().view(np.int32))
    assert np.array_equal(save.cpu().numpy(), np.concatenate([w.numpy().view(np.int32) for w in ref]))
    assert int(esc.item()) == 0 and flags.cpu().tolist() == [esc_ref, 0]
    _, _, counts = gather_order_ref(ref[1], ref[2], edges)
    assert hc.tolist() == counts == work[n:n + world].cpu().tolist()
    gpu.KLTFreeTrackingContext(tc)


def sharded_sequence(gpu, frames, nfeat, world, chunk, margin, ahead=True, band_only=False):
    """Frames[0] selects; frames[1:] are tracked by `world` simulated ranks
    (ahead: each call builds the next chunk's band pyramids ahead; band_only:
    each rank holds only its band's rows, whole frames only to redo a chunk)."""
    H, W = frames[0].shape
    dev = torch.device("cuda", 0)
    dfr = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    x0, y0, v0 = (torch.from_numpy(a).to(dev) for a in _select(gpu, frames[0], nfeat))
    ranks = [_Rank(gpu, dfr, H, W, world, r, margin) for r in range(world)]
    if band_only:
        for rk in ranks:
            rk.band_only()
    for rk in ranks:
        rk.begin(0)
    x, y, v = x0.clone(), y0.clone(), v0.clone()
    redone = 0
    T = len(frames) - 1
    for c0 in range(1, 1 + T, chunk):
        n = min(chunk, 1 + T - c0)
        nn = min(chunk, 1 + T - c0 - n) if ahead else 0
        state = (x.clone(), y.clone(), v.clone())
        outs, esc_any = [], 0
        for rk in ranks:
            xr, yr, vr = (s.clone() for s in state)
            esc = torch.zeros(1, dtype=torch.int32, device=dev)
            rk.chunk(c0, n, xr, yr, vr, esc, next_n=nn)
            esc_any += int(esc.item())
            outs.append((xr, yr, vr))
        if esc_any:
            redone += 1
            outs = []
            for rk in ranks:
                xr, yr, vr = (s.clone() for s in state)
                esc = torch.zeros(1, dtype=torch.int32, device=dev)
                rk.begin(c0 - 1)
                rk.chunk(c0, n, xr, yr, vr, esc, full=True, next_n=nn)
                assert int(esc.item()) == 0
                outs.append((xr, yr, vr))
        # the all-gather, done by hand: every rank's slot packed on the device
        # (klt_hip_gather_pack), the slots stacked, unpacked into the chunk-start state
        x, y, v = device_gather_merge(gpu, ranks[0].ctx, state, outs, band_edges(H, world))
    for rk in ranks:
        gpu.KLTFreeTrackingContext(rk.tc)
    return x.cpu().numpy(), y.cpu().numpy(), v.cpu().numpy(), redone


@pytest.mark.gpu
@pytest.mark.parametrize("world,chunk,margin,ahead,band_only",
                         [(2, 4, 128, True, False), (3, 5, 64, True, False), (4, 3, 40, True, False),
                          (2, 4, 0, True, False), (3, 4, 64, False, False), (4, 3, 0, False, False),
                          (3, 5, 64, True, True), (4, 3, 0, True, True)])
def test_sharded_equals_single_gpu(gpu, oracle, world, chunk, margin, ahead, band_only):
    from kltabi import OracleTracker
    frames = synth(gpu, 2160 + world, 640, 480, 11)
    x, y, v, redone = sharded_sequence(gpu, frames, 1500, world, chunk, margin, ahead, band_only)
    X, Y, V = OracleTracker(oracle).harness(frames, 1500, 11, first=frames[0])
    k = 11 - 2
    assert np.array_equal(v, V[:, k])
    assert np.array_equal(x.view(np.int32), X[:, k].view(np.int32))
    assert np.array_equal(y.view(np.int32), Y[:, k].view(np.int32))
    if margin == 0:
        assert redone > 0  # no margin: features near band edges must escape and be redone


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_4k_20k_equals_reference(gpu, world):
    """BASELINE config 4 (3840x2160, 20000 features): the feature-sharded
    schedule with 2/4/8 simulated ranks (32-frame chunks, 64-row margin, next chunk built ahead)
    reproduces the reference's list after 64 frames -- the digest of column 63
    of tests/golden/long_config4.json (oracle/_ref on the full sequence)."""
    import hashlib
    import json
    from kltabi import GOLDEN
    cfg = json.loads((GOLDEN / "long_config4.json").read_text())
    T = 64
    frames = synth(gpu, cfg["seed"], cfg["w"], cfg["h"], T + 1)
    x, y, v, redone = sharded_sequence(gpu, frames, cfg["features"], world, 32, 64)
    h = hashlib.sha256()
    for a, dt in ((x, "<f4"), (y, "<f4"), (v, "<i4")):
        h.update(np.ascontiguousarray(a, dt).tobytes())
    assert h.hexdigest() == cfg["columns"][T - 1], f"world {world}: sharded list differs (redone {redone})"


# ---------------------------------------------------------------------------
# GPU: the C-ABI driver (include/klt_shard.h) -- ranks rehearsed in one process
# ---------------------------------------------------------------------------
_FRAMES_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_long))


def c_sharded_sequence(gpu, frames, nfeat, world, chunk, margin, band_only=False, real_comm=False, replace=False):
    """klt_shard_track per chunk for every rank (klt_shard_create_local: the
    rank's band, a communicator of its own), then the all-gather done by hand:
    each feature from its owner's result.  real_comm (world 1): the
    RCCL path proper, klt_shard_unique_id + klt_shard_create.  replace: lost
    features replaced after every chunk -- klt_shard_replace over the real
    communicator, else every rank's klt_shard_eigen rows into one map and
    klt_shard_select over it."""
    from kltamd.device import SelectDesc
    H, W = frames[0].shape
    dev = torch.device("cuda", 0)
    dfr = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    x, y, v = (torch.from_numpy(a).to(dev) for a in _select(gpu, frames[0], nfeat))
    ranks, shards, keep = [], [], []
    E = row_edges(H, world, margin)  # klt_shard_create's bands (klt_shard_band_edges)
    for r in range(world):
        rk = _Rank(gpu, dfr, H, W, world, r, margin, E)
        if real_comm:
            assert world == 1
            uid = (C.c_ubyte * 128)()
            assert gpu.klt_shard_unique_id(uid) == 0
            s = gpu.klt_shard_create(rk.ctx, 0, 1, uid, H, margin)
        else:
            s = gpu.klt_shard_create_local(rk.ctx, r, world, H, margin)
        assert s
        lo, hi = C.c_int(), C.c_int()
        assert gpu.klt_shard_rows(s, C.byref(lo), C.byref(hi)) == 0
        b = band_of(H, world, r, margin, E)
        assert lo.value <= b.row_lo and hi.value >= b.row_hi
        if band_only:  # only rows [lo, hi) of each frame on this rank, addressed as whole frames
            part = dfr[:, lo.value:hi.value].contiguous()
            base, stride = part.data_ptr() - lo.value * W, (hi.value - lo.value) * W
            keep.append(part)
        else:
            base, stride = dfr.data_ptr(), H * W
        rk.base, rk.stride = base, stride
        assert gpu.klt_hip_frames_begin(rk.ctx, C.byref(rk.pd), C.c_void_p(dfr.data_ptr()), W) == 0
        ranks.append(rk)
        shards.append(s)
    redone, cur, rebuilt = [0], [0], [0]
    bands = [band_of(H, world, r, margin, E) for r in range(world)]

    def whole(user, frames_out, stride_out):  # whole frames from frame cur[0] on
        frames_out[0] = dfr.data_ptr() + cur[0] * H * W
        stride_out[0] = H * W
        redone[0] += 1
        return 0
    cb = _FRAMES_FN(whole)
    T = len(frames) - 1
    for c0 in range(1, 1 + T, chunk):
        n = min(chunk, 1 + T - c0)
        nn = min(chunk, 1 + T - c0 - n)
        cur[0] = c0 - 1
        merged = (x.clone(), y.clone(), v.clone())
        for r, (rk, s) in enumerate(zip(ranks, shards)):
            xr, yr, vr = x.clone(), y.clone(), v.clone()
            nxt = C.c_void_p(rk.base + (c0 + n) * rk.stride) if nn else None
            rc = gpu.klt_shard_track(s, C.byref(rk.pd), C.byref(rk.td), C.c_void_p(rk.base + c0 * rk.stride), W,
                                     rk.stride, n, nxt, nn, C.c_void_p(xr.data_ptr()), C.c_void_p(yr.data_ptr()),
                                     C.c_void_p(vr.data_ptr()), x.numel(), cb, None)
            assert rc in (0, 1), gpu.klt_shard_last_error(s)
            # a local shard updates its owned features and leaves the others as they were
            own = owned_mask(y, v, bands[r])
            assert torch.equal(xr.view(torch.int32)[~own], x.view(torch.int32)[~own])
            for m, t in zip(merged, (xr, yr, vr)):
                m[own] = t[own]
        x, y, v = merged
        if replace:
            tc = ranks[0].tc.contents
            sd = SelectDesc(tc.window_width, tc.window_height, max(tc.borderx, tc.window_width // 2),
                            max(tc.bordery, tc.window_height // 2), tc.nSkippedPixels)
            cur[0] = c0 + n - 1  # the last tracked frame, whole, when a band is too narrow
            xyz = (C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), x.numel())
            if real_comm:
                rk, s = ranks[0], shards[0]
                rc = gpu.klt_shard_replace(s, C.byref(rk.pd), C.byref(sd), W, tc.mindist, tc.min_eigenvalue,
                                           *xyz, cb, None)
                assert rc == 0, gpu.klt_shard_last_error(s)
            else:
                nx, ny, j0, j1 = (C.c_int() for _ in range(4))
                assert gpu.klt_hip_min_eigen_rows(ranks[0].ctx, C.byref(sd), 0, 0, None, C.byref(nx), C.byref(ny),
                                                  C.byref(j0), C.byref(j1)) == 0
                emap = torch.full((nx.value * ny.value,), -7, dtype=torch.int32, device=dev)
                for rk, s in zip(ranks, shards):
                    rc = gpu.klt_shard_eigen(s, C.byref(rk.pd), C.byref(sd), W, C.c_void_p(emap.data_ptr()), cb, None)
                    assert rc in (0, 1), gpu.klt_shard_last_error(s)
                    rebuilt[0] += rc
                assert not bool((emap == -7).any())  # the ranks' rows tile the map
                rc = gpu.klt_shard_select(shards[0], C.byref(ranks[0].pd), C.byref(sd), tc.mindist,
                                          tc.min_eigenvalue, C.c_void_p(emap.data_ptr()), *xyz)
                assert rc == 0, gpu.klt_shard_last_error(shards[0])
    for rk, s in zip(ranks, shards):
        gpu.klt_shard_destroy(s)
        gpu.KLTFreeTrackingContext(rk.tc)
    del keep
    if replace:
        c_sharded_sequence.rebuilt = rebuilt[0]
    return x.cpu().numpy(), y.cpu().numpy(), v.cpu().numpy(), redone[0]


@pytest.mark.gpu
@pytest.mark.parametrize("world,chunk,margin,band_only,real_comm",
                         [(1, 4, 64, False, True), (3, 5, 64, False, False), (4, 3, 0, True, False),
                          (2, 4, 64, True, False)])
def test_c_shard_equals_single_gpu(gpu, oracle, world, chunk, margin, band_only, real_comm):
    from kltabi import OracleTracker
    frames = synth(gpu, 2160 + world, 640, 480, 11)
    x, y, v, redone = c_sharded_sequence(gpu, frames, 1500, world, chunk, margin, band_only, real_comm)
    X, Y, V = OracleTracker(oracle).harness(frames, 1500, 11, first=frames[0])
    k = 11 - 2
    assert np.array_equal(v, V[:, k])
    assert np.array_equal(x.view(np.int32), X[:, k].view(np.int32))
    assert np.array_equal(y.view(np.int32), Y[:, k].view(np.int32))
    if margin == 0:
        assert redone > 0  # no margin: band-edge features escape; the callback supplies whole frames


@pytest.mark.gpu
@pytest.mark.parametrize("world,margin,real_comm", [(1, 64, True), (3, 64, False), (4, 0, False), (2, 2, False)])
def test_c_shard_replace_equals_single_gpu(gpu, oracle, world, margin, real_comm):
    """KLTReplaceLostFeatures after every frame (the harness with REPLACE):
    ranks' band trackability rows + the same host selection on every rank
    equal the oracle's sequence bit for bit (margin 0: band pyramids too short
    for the selection window, or chunks redone)."""
    from kltabi import OracleTracker
    frames = synth(gpu, 3160 + world, 640, 480, 9)
    x, y, v, redone = c_sharded_sequence(gpu, frames, 800, world, 1, margin, False, real_comm, replace=True)
    X, Y, V = OracleTracker(oracle).harness(frames, 800, 9, first=frames[0], replace=True)
    k = 9 - 2
    assert (V[:, :k + 1] >= 0).sum() > 0 and (V[:, k] > 0).any()  # replacements happened (val = eigenvalue)
    assert np.array_equal(v, V[:, k])
    assert np.array_equal(x.view(np.int32), X[:, k].view(np.int32))
    assert np.array_equal(y.view(np.int32), Y[:, k].view(np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("world,rank,margin", [(4, 1, 0), (3, 2, 0), (3, 0, 64), (15, 1, 0), (15, 14, 0), (15, 7, 1)])
def test_eigen_rows_of_band_pyramid(gpu, world, rank, margin):
    """klt_hip_min_eigen_rows on a band-built pyramid: the rank's grid rows
    equal the whole frame's map (klt_hip_min_eigen), or it reports 1 (nothing
    written) when the 7x7 window reaches rows the band does not hold;
    klt_shard_eigen then rebuilds the frame whole through the callback
    (15 ranks of 480 rows: 32-row bands on tile edges, no margin)."""
    from kltamd.device import SelectDesc
    frames = synth(gpu, 4242, 640, 480, 2)
    H, W = frames[0].shape
    dev = torch.device("cuda", 0)
    dfr = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    E = row_edges(H, world, margin)  # the bands klt_shard_create_local uses below
    rk = _Rank(gpu, dfr, H, W, world, rank, margin, E)
    tc = rk.tc.contents
    sd = SelectDesc(tc.window_width, tc.window_height, max(tc.borderx, tc.window_width // 2),
                    max(tc.bordery, tc.window_height // 2), tc.nSkippedPixels)
    # whole-frame map of frame 1
    assert gpu.klt_hip_frames_begin(rk.ctx, C.byref(rk.pd), C.c_void_p(dfr.data_ptr() + H * W), W) == 0
    nx, ny, j0, j1 = (C.c_int() for _ in range(4))
    assert gpu.klt_hip_min_eigen_rows(rk.ctx, C.byref(sd), 0, H, None, C.byref(nx), C.byref(ny),
                                      C.byref(j0), C.byref(j1)) == 0
    full_map = torch.zeros(nx.value * ny.value, dtype=torch.int32, device=dev)
    assert gpu.klt_hip_min_eigen_rows(rk.ctx, C.byref(sd), 0, H, C.c_void_p(full_map.data_ptr()), C.byref(nx),
                                      C.byref(ny), C.byref(j0), C.byref(j1)) == 0
    assert (j0.value, j1.value) == (0, ny.value)
    # band pyramid of frame 1 (a band call with no features builds it and makes it the previous pyramid)
    rk.begin(0)
    esc = torch.zeros(1, dtype=torch.int32, device=dev)
    e = torch.zeros(0, device=dev)
    b = rk.band
    assert gpu.klt_hip_track_frames_band(rk.ctx, C.byref(rk.pd), C.byref(rk.td), C.c_void_p(dfr.data_ptr() + H * W),
                                         W, H * W, 1, C.c_void_p(e.data_ptr()), C.c_void_p(e.data_ptr()),
                                         C.c_void_p(e.data_ptr()), 0, b.own_lo, b.own_hi, b.row_lo, b.row_hi,
                                         C.c_void_p(esc.data_ptr()), None, 0) == 0
    lo = 0 if rank == 0 else E[rank]
    hi = H if rank == world - 1 else E[rank + 1]
    got = torch.full_like(full_map, -7)
    rc = gpu.klt_hip_min_eigen_rows(rk.ctx, C.byref(sd), lo, hi, C.c_void_p(got.data_ptr()), C.byref(nx),
                                    C.byref(ny), C.byref(j0), C.byref(j1))
    by, step, hh = sd.bordery, sd.nSkippedPixels + 1, sd.window_height // 2
    rows = slice(j0.value * nx.value, j1.value * nx.value)
    assert j1.value > j0.value and all(lo <= by + j * step < hi for j in (j0.value, j1.value - 1))
    # a band build runs whole 32-row level-0 tiles: those rows are valid
    vlo, vhi = b.row_lo // 32 * 32, (H if b.row_hi >= H else min(H, -(-b.row_hi // 32) * 32))
    needs = (by + j0.value * step - hh < vlo) or (by + (j1.value - 1) * step + hh >= vhi)
    assert rc == (1 if needs else 0)
    if rc == 0:
        assert torch.equal(got[rows], full_map[rows])
        assert bool((got[:rows.start] == -7).all()) and bool((got[rows.stop:] == -7).all())
    else:
        assert bool((got == -7).all())
        # the shard rebuilds the frame whole and then succeeds
        s = gpu.klt_shard_create_local(rk.ctx, rank, world, H, margin)
        calls = []

        def whole(user, frames_out, stride_out):
            calls.append(1)
            frames_out[0] = dfr.data_ptr() + H * W
            stride_out[0] = H * W
            return 0
        cb = _FRAMES_FN(whole)
        assert gpu.klt_shard_eigen(s, C.byref(rk.pd), C.byref(sd), W, C.c_void_p(got.data_ptr()), cb, None) == 1
        assert calls == [1] and torch.equal(got[rows], full_map[rows])
        gpu.klt_shard_destroy(s)
    gpu.KLTFreeTrackingContext(rk.tc)


@pytest.mark.gpu
def test_c_shard_errors(gpu):
    """klt_shard.h error behaviour: bad geometry refused at create, a frame
    height that differs from the shard's, an escaped chunk with no whole-frame
    callback, and klt_shard_replace on a local shard (no peers) all fail with
    a message, without touching the feature arrays."""
    from kltamd.device import SelectDesc
    frames = synth(gpu, 77, 640, 480, 3)
    H, W = frames[0].shape
    dev = torch.device("cuda", 0)
    dfr = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    rk = _Rank(gpu, dfr, H, W, 4, 1, 0)
    assert not gpu.klt_shard_create_local(rk.ctx, 4, 4, H, 0)   # rank out of range
    assert b"bad arguments" in gpu.klt_shard_create_error()
    assert not gpu.klt_shard_create_local(rk.ctx, 0, 0, H, 0)   # no ranks
    assert not gpu.klt_shard_create_local(rk.ctx, 0, 2, H, -1)  # negative margin
    assert not gpu.klt_shard_create_local(rk.ctx, 0, 17, H, 0)  # past KLT_HIP_GATHER_MAX_RANKS
    assert b"KLT_HIP_GATHER_MAX_RANKS" in gpu.klt_shard_create_error()
    s = gpu.klt_shard_create_local(rk.ctx, 1, 4, H, 0)
    assert s and gpu.klt_shard_create_error() == b""
    x, y, v = (torch.from_numpy(a).to(dev) for a in _select(gpu, frames[0], 800))
    x0, y0, v0 = x.clone(), y.clone(), v.clone()
    ptrs = (C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), x.numel())
    assert gpu.klt_hip_frames_begin(rk.ctx, C.byref(rk.pd), C.c_void_p(dfr.data_ptr()), W) == 0
    from kltamd.device import PyrDesc
    bad = PyrDesc()
    gpu.klt_amd_pyr_desc(rk.tc, W, H - 32, rk.tc.contents.nPyramidLevels, 1, C.byref(bad))
    rc = gpu.klt_shard_track(s, C.byref(bad), C.byref(rk.td), C.c_void_p(dfr.data_ptr() + H * W), W, H * W, 2,
                             None, 0, *ptrs, None, None)
    assert rc < 0 and b"rows" in gpu.klt_shard_last_error(s)
    # margin 0 over two frames: some owned feature's window leaves the band -> escape; no callback -> error
    rc = gpu.klt_shard_track(s, C.byref(rk.pd), C.byref(rk.td), C.c_void_p(dfr.data_ptr() + H * W), W, H * W, 2,
                             None, 0, *ptrs, None, None)
    assert rc < 0 and b"callback" in gpu.klt_shard_last_error(s)
    # a whole-frame callback that fails: the rank still joins the redo's exchange, then reports it
    calls = [0]

    def broken(user, frames_out, stride_out):
        calls[0] += 1
        return 1
    cb = _FRAMES_FN(broken)
    x.copy_(x0), y.copy_(y0), v.copy_(v0)
    rc = gpu.klt_shard_track(s, C.byref(rk.pd), C.byref(rk.td), C.c_void_p(dfr.data_ptr() + H * W), W, H * W, 2,
                             None, 0, *ptrs, cb, None)
    assert rc < 0 and b"whole-frame callback failed" in gpu.klt_shard_last_error(s) and calls[0] == 1
    assert gpu.klt_hip_current_device() == 0
    tc = rk.tc.contents
    sd = SelectDesc(tc.window_width, tc.window_height, max(tc.borderx, 3), max(tc.bordery, 3), tc.nSkippedPixels)
    x.copy_(x0), y.copy_(y0), v.copy_(v0)
    rc = gpu.klt_shard_replace(s, C.byref(rk.pd), C.byref(sd), W, tc.mindist, tc.min_eigenvalue, *ptrs, None, None)
    assert rc < 0 and b"local" in gpu.klt_shard_last_error(s)
    assert torch.equal(x, x0) and torch.equal(v, v0)
    gpu.klt_shard_destroy(s)
    gpu.KLTFreeTrackingContext(rk.tc)


@pytest.mark.gpu
def test_c_shard_failure_agreement(gpu):
    """The failure agreement of klt_shard_track / klt_shard_replace over a real
    one-rank RCCL communicator, driven by klt_shard_inject_fault: a local
    failure still runs the exchange (agreement) and reports its own message;
    a failure count from a peer (phantom) makes the call fail with "1 peer
    rank(s) failed"; clearing the faults makes the shard work again; an
    exchange-buffer allocation failure aborts the communicator and the shard
    refuses every later call."""
    from kltamd.device import SelectDesc
    os.environ.pop("KLT_SHARD_TESTING", None)
    frames = synth(gpu, 91, 640, 480, 3)
    H, W = frames[0].shape
    dev = torch.device("cuda", 0)
    dfr = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    rk = _Rank(gpu, dfr, H, W, 1, 0, 64)
    uid = (C.c_ubyte * 128)()
    assert gpu.klt_shard_unique_id(uid) == 0
    s = gpu.klt_shard_create(rk.ctx, 0, 1, uid, H, 64)
    assert s
    assert gpu.klt_shard_inject_fault(s, 1) == -2  # test-only: inert without KLT_SHARD_TESTING=1
    os.environ["KLT_SHARD_TESTING"] = "1"
    assert gpu.klt_shard_inject_fault(s, 8) == -1  # unknown fault bit
    x, y, v = (torch.from_numpy(a).to(dev) for a in _select(gpu, frames[0], 600))
    x0, y0, v0 = x.clone(), y.clone(), v.clone()
    ptrs = (C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), x.numel())
    tc = rk.tc.contents
    sd = SelectDesc(tc.window_width, tc.window_height, max(tc.borderx, tc.window_width // 2),
                    max(tc.bordery, tc.window_height // 2), tc.nSkippedPixels)
    f1 = C.c_void_p(dfr.data_ptr() + H * W)

    def track():
        x.copy_(x0), y.copy_(y0), v.copy_(v0)
        assert gpu.klt_hip_frames_begin(rk.ctx, C.byref(rk.pd), C.c_void_p(dfr.data_ptr()), W) == 0
        return gpu.klt_shard_track(s, C.byref(rk.pd), C.byref(rk.td), f1, W, H * W, 1, None, 0, *ptrs, None, None)

    def replace():
        return gpu.klt_shard_replace(s, C.byref(rk.pd), C.byref(sd), W, tc.mindist, tc.min_eigenvalue, *ptrs,
                                     None, None)

    def err():
        return gpu.klt_shard_last_error(s).decode()

    assert track() == 0
    good = [t.clone() for t in (x, y, v)]
    assert gpu.klt_shard_inject_fault(s, 1) == 0  # LOCAL
    assert track() < 0 and err() == "shard_track: injected local fault"
    x.copy_(good[0]), y.copy_(good[1]), v.copy_(good[2])
    assert replace() < 0 and err() == "shard_replace: injected local fault"
    assert torch.equal(x, good[0]) and torch.equal(v, good[2])  # no selection ran
    assert gpu.klt_shard_inject_fault(s, 2) == 0  # PEER
    assert track() < 0 and err() == "shard_track: 1 peer rank(s) failed this chunk"
    x.copy_(good[0]), y.copy_(good[1]), v.copy_(good[2])
    assert replace() < 0 and err() == "shard_replace: 1 peer rank(s) failed the trackability map"
    assert torch.equal(x, good[0]) and torch.equal(v, good[2])
    assert gpu.klt_shard_inject_fault(s, 3) == 0  # both: this rank's own message wins
    assert track() < 0 and err() == "shard_track: injected local fault"
    assert gpu.klt_shard_inject_fault(s, 0) == 0  # cleared: the communicator still works
    assert track() == 0
    assert all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip((x, y, v), good))
    assert replace() == 0
    assert gpu.klt_shard_inject_fault(s, 4) == 0  # ALLOC: abort
    assert track() < 0 and "communicator aborted" in err() and "injected allocation failure" in err()
    assert gpu.klt_shard_inject_fault(s, 0) == 0
    assert track() < 0 and err() == "shard_track: the communicator was aborted"
    assert replace() < 0 and err() == "shard_replace: the communicator was aborted"
    assert gpu.klt_hip_current_device() == 0
    gpu.klt_shard_destroy(s)
    gpu.KLTFreeTrackingContext(rk.tc)


# ---------------------------------------------------------------------------
# GPU: kltamd.shard.ShardedSequence itself, one thread per rank on one GPU,
# the collectives done by a thread group (sum / copy between the ranks' tensors)
# ---------------------------------------------------------------------------
class _ThreadGroup:
    def __init__(self, world):
        import threading
        self.world, self.bar, self.slots, self.out = world, threading.Barrier(world), [None] * world, None

    def all_reduce(self, rank, t):
        torch.cuda.current_stream().synchronize()
        self.slots[rank] = t
        self.bar.wait()
        if rank == 0:
            acc = self.slots[0].clone()
            for o in self.slots[1:]:
                acc += o
            torch.cuda.current_stream().synchronize()
            self.out = acc
        self.bar.wait()
        t.copy_(self.out)
        torch.cuda.current_stream().synchronize()
        self.bar.wait()

    def all_gather(self, rank, out, inp):
        torch.cuda.current_stream().synchronize()
        self.slots[rank] = inp
        self.bar.wait()
        out.copy_(torch.cat(self.slots))
        torch.cuda.current_stream().synchronize()
        self.bar.wait()

    def broadcast(self, rank, t, src):
        torch.cuda.current_stream().synchronize()
        if rank == src:
            self.slots[src] = t
        self.bar.wait()
        if rank != src:
            t.copy_(self.slots[src])
            torch.cuda.current_stream().synchronize()
        self.bar.wait()


def threaded_sequence(gpu, frames, nfeat, world, chunk, margin, replace=False, band_only=False):
    """frames[0] selects; world ShardedSequence ranks (threads, one context
    each) track frames[1:] -- with replace: one frame per run() and
    ShardedSequence.replace after each, as the REPLACE harness does."""
    import threading
    from kltamd.device import D2D, PyrDesc, SelectDesc, TrackDesc, check, use_torch_stream
    from kltamd.shard import BandFrames, FullFrames, ShardedSequence, band_of
    H, W = frames[0].shape
    T = len(frames) - 1
    dev = torch.device("cuda", 0)
    dfr = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    sel = _select(gpu, frames[0], nfeat)
    grp = _ThreadGroup(world)
    tcs = [gpu.KLTCreateTrackingContext() for _ in range(world)]
    for tc in tcs:
        tc.contents.sequentialMode = 1
    ctxs = [gpu.klt_amd_device_context(tc) for tc in tcs]
    out, errs, stats = [None] * world, [], [None] * world

    def worker(rank):
        try:
            torch.cuda.set_device(dev)
            ctx, tc = ctxs[rank], tcs[rank]
            use_torch_stream(gpu, ctx, dev)
            pd, td = PyrDesc(), TrackDesc()
            gpu.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
            gpu.klt_amd_track_desc(tc, C.byref(td))
            x, y, v = (torch.from_numpy(a).to(dev) for a in sel)
            if band_only:
                def load(t0, n, row0, nrows, dst, stride):
                    part = dfr[t0:t0 + n, row0:row0 + nrows].contiguous()
                    for f in range(n):
                        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, C.c_void_p(dst + f * stride),
                                                           C.c_void_p(part[f].data_ptr()), nrows * W, D2D), "d2d")
                    gpu.klt_hip_sync(ctx)
                src = BandFrames(T + 1, H, W, band_of(H, world, rank, margin, row_edges(H, world, margin)), load,
                                 dev)
            else:
                src = FullFrames(dfr)
            seq = ShardedSequence(gpu, ctx, pd, td, src, x, y, v, rank, world,
                                  lambda o, i: grp.all_gather(rank, o, i),
                                  chunk=chunk, margin=margin)
            seq.begin(0)
            if replace:
                c = tc.contents
                sd = SelectDesc(c.window_width, c.window_height, max(c.borderx, c.window_width // 2),
                                max(c.bordery, c.window_height // 2), c.nSkippedPixels)
                for t in range(1, T + 1):
                    seq.run(t, 1)
                    seq.replace(sd, c.mindist, c.min_eigenvalue, lambda tt, s: grp.broadcast(rank, tt, s))
            else:
                seq.run(1, T)
            torch.cuda.current_stream().synchronize()
            out[rank] = (x.cpu().numpy(), y.cpu().numpy(), v.cpu().numpy())
            stats[rank] = (seq.redone, seq.rebuilt)
        except BaseException as e:  # surface in the main thread; release the others
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    for tc in tcs:
        gpu.KLTFreeTrackingContext(tc)
    if errs:
        raise errs[0]
    for r in range(1, world):  # every rank ends with the same list
        for a, b in zip(out[0], out[r]):
            assert np.array_equal(a.view(np.int32), b.view(np.int32))
    return out[0], stats


@pytest.mark.gpu
@pytest.mark.parametrize("world,chunk,margin,band_only", [(1, 4, 64, False), (3, 4, 64, False), (3, 3, 0, True),
                                                         (4, 5, 40, True)])
def test_sharded_sequence_threads_equal_oracle(gpu, oracle, world, chunk, margin, band_only):
    from kltabi import OracleTracker
    frames = synth(gpu, 2170 + world, 640, 480, 11)
    (x, y, v), stats = threaded_sequence(gpu, frames, 1500, world, chunk, margin, band_only=band_only)
    X, Y, V = OracleTracker(oracle).harness(frames, 1500, 11, first=frames[0])
    k = 11 - 2
    assert np.array_equal(v, V[:, k])
    assert np.array_equal(x.view(np.int32), X[:, k].view(np.int32))
    assert np.array_equal(y.view(np.int32), Y[:, k].view(np.int32))
    if margin == 0:
        assert stats[0][0] > 0  # chunks redone from whole frames


@pytest.mark.gpu
@pytest.mark.parametrize("world,margin,band_only", [(1, 64, False), (3, 64, True), (4, 0, False)])
def test_sharded_sequence_replace_equals_oracle(gpu, oracle, world, margin, band_only):
    """ShardedSequence.replace after every frame (the REPLACE harness): the
    ranks' trackability rows, broadcast per owner, and the same selection on
    every rank equal the oracle's list bit for bit."""
    from kltabi import OracleTracker
    frames = synth(gpu, 3170 + world, 640, 480, 9)
    (x, y, v), stats = threaded_sequence(gpu, frames, 800, world, 1, margin, replace=True, band_only=band_only)
    X, Y, V = OracleTracker(oracle).harness(frames, 800, 9, first=frames[0], replace=True)
    k = 9 - 2
    assert (V[:, k] > 0).any()  # some slots hold replacements (val = their eigenvalue)
    assert np.array_equal(v, V[:, k])
    assert np.array_equal(x.view(np.int32), X[:, k].view(np.int32))
    assert np.array_equal(y.view(np.int32), Y[:, k].view(np.int32))
