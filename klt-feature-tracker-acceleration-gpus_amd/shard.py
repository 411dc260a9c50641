"""Feature-sharded tracking across ranks (BASELINE config 4).

Row-band decomposition: rank r of N owns the features whose y lies in its band
[r*H/N, (r+1)*H/N) at the start of a chunk, builds pyramids only for its band
plus a margin (klt_hip_track_frames_band), and tracks its features through the
chunk.  After every chunk the ranks exchange results with one all-gather of
fixed per-rank slots: every rank holds the same chunk-start state, so every
rank knows every live feature's owner and its place among the owner's
features (klt_hip_gather_order); rank r packs its features' (x, y, val) bit
patterns in index order into its slot (klt_hip_gather_pack), the slots are
all-gathered, and every rank takes each feature from its owner's slot
(klt_hip_gather_unpack).  Lost features are nobody's and stay as they are,
the same on every rank.  A feature whose window would leave a rank's built
rows raises the chunk's escape flag (it rides in the slot's header); all
ranks then redo that chunk from full-frame pyramids, so the result never
depends on the margin.

The slot size is the largest owner's count, the same on every rank: the
counts are computed on the device right after the previous exchange and read
while the next chunk is already tracking.  The driver is speculative: chunk
c+1 is queued before chunk c's escape flag is read, and a chunk that escaped
(rare by design; never at the default margin on the synthetic sequences)
costs a drain, the redo and chunk c+1 again.  The next chunk's band pyramids
depend on frames only, so each call hands the library the next chunk's
frames: it builds them on its pyramid stream while this chunk is tracked and
exchanged.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

# level-0 rows built beyond the band: a level-1 row needs sigma-3.6 input 20
# rows above and 24 below its level-0 rows (the library marks exactly those
# rows valid), the level-1 window 4*(hh+1) more, plus a chunk of motion;
# tools/shard_sim.py: 48 and 64 never escaped at 4K/20k features (32- and
# 64-frame chunks), 32 did
DEFAULT_MARGIN = 64


@dataclass(frozen=True)
class Band:
    own_lo: float  # features with own_lo <= y < own_hi belong to the rank
    own_hi: float
    row_lo: int  # level-0 rows the rank builds
    row_hi: int


def band_of(nrows: int, world: int, rank: int, margin: int = DEFAULT_MARGIN, edges=None) -> Band:
    """Rank r's band: rows [r*H/N, (r+1)*H/N), or [edges[r], edges[r+1]) when
    edges (N+1 row boundaries, balanced_edges) are given."""
    if edges is not None:
        assert len(edges) == world + 1 and edges[0] == 0 and edges[-1] == nrows
        lo, hi = int(edges[rank]), int(edges[rank + 1])
    else:
        lo = rank * nrows // world
        hi = (rank + 1) * nrows // world
    own_lo = float("-inf") if rank == 0 else float(lo)
    own_hi = float("inf") if rank == world - 1 else float(hi)
    return Band(own_lo, own_hi, max(0, lo - margin), min(nrows, hi + margin))


def balanced_edges(y: torch.Tensor, v: torch.Tensor, nrows: int, world: int) -> list[int]:
    """Row boundaries that give every rank about the same number of live
    features (quantiles of their y), for the tracker's share of a rank's time:
    a rank with a dense band gets fewer rows.  Deterministic in (y, v), so
    every rank computes the same edges from the same list."""
    ys = torch.sort(y[v >= 0].float().cpu()).values
    m = ys.numel()
    edges = [0]
    for r in range(1, world):
        e = int(ys[min(m - 1, r * m // world)].item()) if m else r * nrows // world
        edges.append(min(max(e, edges[-1]), nrows))
    edges.append(nrows)
    return edges


def built_rows(nrows: int, band: Band, tile: int = 32) -> int:
    """Level-0 rows a rank's band build covers: its rows rounded out to whole tiles."""
    lo = (band.row_lo // tile) * tile
    hi = min(nrows, -(-band.row_hi // tile) * tile)
    return hi - lo


def row_edges(nrows: int, world: int, margin: int = DEFAULT_MARGIN, tile: int = 32) -> list[int]:
    """Row boundaries that give every rank about the same number of level-0
    rows to build (its band, the margins, whole tiles): the two edge ranks have
    one margin, so they own about a margin's rows more.  Inner boundaries on
    tile multiples (no partial tiles on either side); the candidate inner
    heights around (nrows - 2 margin) / world are scored by their largest
    build against equal bands.  Deterministic in its arguments."""
    eq = [r * nrows // world for r in range(world + 1)]
    if world < 3:
        return eq
    # equal bands first: a candidate must build strictly fewer rows to replace them
    best = (max(built_rows(nrows, band_of(nrows, world, r, margin, eq), tile) for r in range(world)), eq)
    ideal = (nrows - 2 * margin) / world
    for k in range(max(1, int(ideal // tile) - 2), int(ideal // tile) + 3):
        inner = k * tile
        rest = nrows - (world - 2) * inner
        if rest < 2 * tile:
            continue
        for first in sorted({(rest // 2 // tile) * tile, -(-(rest // 2) // tile) * tile}):
            edges = [0] + [first + i * inner for i in range(world - 1)] + [nrows]
            if any(b <= a for a, b in zip(edges, edges[1:])):
                continue
            cost = max(built_rows(nrows, band_of(nrows, world, r, margin, edges), tile) for r in range(world))
            if cost < best[0]:
                best = (cost, edges)
    return best[1]


def chunk_plan(t0: int, nframes: int, chunk: int, first: int | None = None) -> list[tuple[int, int]]:
    """(first frame, frames) of each chunk over frames t0 .. t0+nframes-1:
    `first` frames (default: chunk), then `chunk` each.  Deterministic, so
    every rank cuts the same chunks.  A short first chunk does not fill the
    build-ahead pipeline sooner: the second chunk's whole build is then
    exposed (tools/shard_sim.py --first-chunk 8 / 16 / 64 at 8 ranks: 10.04 /
    9.92 / 9.77 us per frame)."""
    first = chunk if first is None else max(1, min(first, chunk))
    out, c0, end = [], t0, t0 + nframes
    while c0 < end:
        n = min(first if not out else chunk, end - c0)
        out.append((c0, n))
        c0 += n
    return out


def cost_edges(y: torch.Tensor, v: torch.Tensor, nrows: int, world: int, margin: int = DEFAULT_MARGIN,
               feat_rows: float = 0.066, tile: int = 32) -> list[int]:
    """Row boundaries on tile multiples that minimise the largest rank cost
    built_rows + feat_rows * (live features owned), from the list (y, v) at
    the start: a rank's level-0 build and its tracker both grow with what it
    holds.  feat_rows prices one feature in level-0 rows (0.066: one 32-row
    tile of a 4K band build per ~480 features in tools/shard_sim.py's
    per-rank times).  Binary search on the cost, each rank taking the
    longest band that fits.  Deterministic in (y, v): every rank computes
    the same edges from the same list."""
    if world < 2:
        return [0, nrows]
    ys = torch.sort(y[v >= 0].float().cpu()).values
    bounds = list(range(0, nrows, tile)) + [nrows]  # candidate edges

    def owned(lo, hi, first, last):
        a = 0 if first else int(torch.searchsorted(ys, float(lo)).item())
        b = ys.numel() if last else int(torch.searchsorted(ys, float(hi)).item())
        return b - a

    def cost(lo, hi, r):
        e = [0] * (world + 1)
        e[r], e[r + 1], e[world] = lo, hi, nrows
        bd = Band(float("-inf") if r == 0 else float(lo), float("inf") if r == world - 1 else float(hi),
                  max(0, lo - margin), min(nrows, hi + margin))
        return built_rows(nrows, bd, tile) + feat_rows * owned(lo, hi, r == 0, r == world - 1)

    def fit(T):
        lo, edges = 0, [0]
        for r in range(world - 1):
            best = None
            for hi in bounds:
                if hi <= lo or hi > nrows - (world - 1 - r) * tile:  # a tile left for each rank after r
                    continue
                if cost(lo, hi, r) <= T:
                    best = hi
                else:
                    break
            if best is None:
                return None
            edges.append(best)
            lo = best
        if cost(lo, nrows, world - 1) > T:
            return None
        return edges + [nrows]

    lo_t, hi_t = 0.0, float(nrows + feat_rows * ys.numel() + 2 * margin + tile)
    best = fit(hi_t)
    for _ in range(40):
        mid = 0.5 * (lo_t + hi_t)
        e = fit(mid)
        if e is not None:
            best, hi_t = e, mid
        else:
            lo_t = mid
    return best if best is not None else row_edges(nrows, world, margin, tile)


def band_rows(nrows: int, band: Band, tile: int = 32, halo: int = 8) -> tuple[int, int]:
    """The u8 rows [ra, rb) a rank's band build reads: its level-0 build rows
    rounded out to whole tiles, plus the tiles' halo (k_pyr_l0 reads 5 rows
    above and 7 below a 32-row tile)."""
    lo = (band.row_lo // tile) * tile
    hi = -(-band.row_hi // tile) * tile
    return max(0, lo - halo), min(nrows, hi + halo)


class FullFrames:
    """Every frame whole in device memory (a uint8 tensor [T, H, W])."""

    def __init__(self, frames: torch.Tensor):
        self.frames = frames
        self.T, self.H, self.W = frames.shape
        self.stride = self.H * self.W  # bytes between band frames

    def band(self, t: int) -> int:
        """Device address of row 0 of frame t (only the band's rows are read)."""
        return self.frames.data_ptr() + t * self.stride

    def full(self, t0: int, n: int) -> tuple[int, int]:
        """Device address of frame t0 and the frame stride, frames t0 .. t0+n-1 whole."""
        return self.frames.data_ptr() + t0 * self.stride, self.stride


class BandFrames:
    """A rank's frames as SURVEY 8e has them: only the rows its band build
    reads (band_rows: its band, margin and tile halo), for every frame; whole
    frames only on demand -- the sequence start and a redone chunk -- into a
    scratch buffer.  load(t0, n, row0, nrows, dst, stride) writes rows row0 ..
    row0+nrows-1 of frames t0 .. t0+n-1 to the device address dst (frame
    stride `stride` bytes, pitch W): the rank's ingest (an H2D copy of its
    band of host frames, or synthesis)."""

    def __init__(self, T: int, H: int, W: int, band: Band, load, device):
        self.T, self.H, self.W, self.load = T, H, W, load
        self.ra, self.rb = band_rows(H, band)
        self.stride = (self.rb - self.ra) * W
        self.buf = torch.empty((T, self.rb - self.ra, W), dtype=torch.uint8, device=device)
        load(0, T, self.ra, self.rb - self.ra, self.buf.data_ptr(), self.stride)
        self._scratch = None

    def band(self, t: int) -> int:
        # row y of frame t is at this address + y*W for ra <= y < rb; the band
        # build reads no other rows
        return self.buf.data_ptr() + t * self.stride - self.ra * self.W

    def full(self, t0: int, n: int) -> tuple[int, int]:
        fb = self.H * self.W
        if self._scratch is None or self._scratch.numel() < n * fb:
            self._scratch = torch.empty(n * fb, dtype=torch.uint8, device=self.buf.device)
        self.load(t0, n, 0, self.H, self._scratch.data_ptr(), fb)
        return self._scratch.data_ptr(), fb


def owned_mask(y0: torch.Tensor, v0: torch.Tensor, band: Band) -> torch.Tensor:
    """The features klt_hip_track_frames_band tracks for this band (same tests as k_band_order)."""
    return (v0 >= 0) & (y0 >= band.own_lo) & (y0 < band.own_hi)


def band_edges(nrows: int, world: int, edges=None) -> list[float]:
    """The world+1 ownership edges of band_of: rank r owns edges[r] <= y < edges[r+1]."""
    out = [band_of(nrows, world, r, 0, edges).own_lo for r in range(world)]
    return out + [float("inf")]


SLOT_HDR = 4  # slot header: escape flag, failures, count, S (klt_hip.h KLT_HIP_GATHER_SLOT_WORDS)


def slot_words(S: int) -> int:
    return SLOT_HDR + 3 * S


def gather_order_ref(y0: torch.Tensor, v0: torch.Tensor, edges: list[float]):
    """Owner (-1: none) and place among the owner's features in index order of
    every feature, and every rank's count: what klt_hip_gather_order computes
    (torch, for the CPU tests)."""
    world = len(edges) - 1
    owner = torch.full(y0.shape, -1, dtype=torch.int64)
    for r in range(world):
        m = (v0 >= 0) & (y0 >= edges[r]) & (y0 < edges[r + 1]) & (owner < 0)
        owner[m] = r
    place = torch.zeros_like(owner)
    counts = []
    for r in range(world):
        m = owner == r
        place[m] = torch.arange(int(m.sum()))
        counts.append(int(m.sum()))
    return owner, place, counts


def gather_merge_ref(x, y, v, y0, v0, edges, rank: int, all_gather, escape: int = 0) -> int:
    """In place, after one chunk, with torch ops (CPU tests of the exchange
    over a real process group): this rank's slot of its owned features,
    all_gather(out, inp) of the world's slots, every feature from its owner's
    slot.  Same slots as klt_hip_gather_pack/unpack; returns the summed escape
    flags."""
    owner, place, counts = gather_order_ref(y0, v0, edges)
    S = max(1, max(counts))
    world = len(edges) - 1
    slot = torch.zeros(slot_words(S), dtype=torch.int32)
    slot[0], slot[1], slot[2], slot[3] = escape, 0, counts[rank], S
    m = owner == rank
    p = place[m] + SLOT_HDR
    slot[p] = x.view(torch.int32)[m]
    slot[p + S] = y.view(torch.int32)[m]
    slot[p + 2 * S] = v[m]
    out = torch.zeros(world * slot_words(S), dtype=torch.int32)
    all_gather(out, slot)
    sl = out.view(world, slot_words(S))
    m = owner >= 0
    q, p = owner[m], place[m] + SLOT_HDR
    x.view(torch.int32)[m] = sl[q, p]
    y.view(torch.int32)[m] = sl[q, p + S]
    v[m] = sl[q, p + 2 * S]
    return int(sl[:, 0].sum())


class Exchange:
    """The device side of the all-gather (klt_hip_gather_*) for one rank: the
    chunk-start order (which also saves the start state, alternating between
    two buffers, and zeroes the escape flag), this rank's slot, the gathered
    slots, and pinned host words the kernels write the counts and flags into,
    behind one event -- no copy-engine transfer on the stream between two
    chunks.  all_gather(out, inp) gathers the ranks' slots into out in rank
    order (torch.distributed.all_gather_into_tensor in production)."""

    def __init__(self, lib, ctx, n: int, edges: list[float], rank: int, all_gather, device):
        self.lib, self.ctx, self.n, self.rank, self.all_gather = lib, ctx, n, rank, all_gather
        self.world = len(edges) - 1
        self.edges = (C.c_float * (self.world + 1))(*edges)
        self.work = torch.zeros(lib.klt_hip_gather_work_ints(n, self.world), dtype=torch.int32, device=device)
        self.send = torch.empty(slot_words(max(n, 1)), dtype=torch.int32, device=device)
        self.recv = torch.empty(self.world * slot_words(max(n, 1)), dtype=torch.int32, device=device)
        self.flags = torch.zeros(2, dtype=torch.int32, device=device)
        self.save = torch.empty((2, 3, max(n, 1)), dtype=torch.int32, device=device)
        self.k = 0  # the save buffer the next order() fills
        self.h_counts = torch.zeros(self.world, dtype=torch.int32, pin_memory=True)
        self.h_flags = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        self.ev = torch.cuda.Event()
        self.timing = False  # tools/shard_sim.py: a timing event after every exchange
        self.timing_events = []

    def _check(self, rc, what):
        from .device import check
        check(self.lib, self.ctx, rc, what)

    def order(self, x, y, v, escape) -> int:
        """Ownership of the chunk-start state x/y/v, that state saved, the escape
        flag zeroed; the counts land in h_counts behind the event.  Returns the
        save buffer's index."""
        k = self.k
        self.k ^= 1
        self._check(self.lib.klt_hip_gather_order(
            self.ctx, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), self.n,
            self.edges, self.world, C.c_void_p(self.work.data_ptr()), C.c_void_p(self.save[k].data_ptr()),
            C.c_void_p(escape.data_ptr()), C.c_void_p(self.h_counts.data_ptr())), "gather_order")
        self.ev.record()
        return k

    def restore(self, k: int, x, y, v) -> None:
        """The state save buffer k holds, back into x/y/v."""
        x.view(torch.int32).copy_(self.save[k, 0, :self.n])
        y.view(torch.int32).copy_(self.save[k, 1, :self.n])
        v.copy_(self.save[k, 2, :self.n])

    def slot_size(self) -> int:
        """The largest count of the last order() (waits for its event)."""
        self.ev.synchronize()
        return max(1, int(self.h_counts.max()))

    def exchange(self, x, y, v, escape, S: int) -> int:
        """Pack, all-gather, unpack in place; then the next chunk's order()
        (whose save index is returned)."""
        W = slot_words(S)
        send, recv = self.send[:W], self.recv[:self.world * W]
        self._check(self.lib.klt_hip_gather_pack(
            self.ctx, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()),
            C.c_void_p(self.work.data_ptr()), self.n, self.world, self.rank, C.c_void_p(escape.data_ptr()), 0,
            C.c_void_p(send.data_ptr()), S), "gather_pack")
        self.all_gather(recv, send)
        # unpack and the next chunk's order (ownership, start-state save, escape reset, counts) in one launch
        k = self.k
        self.k ^= 1
        self._check(self.lib.klt_hip_gather_unpack_order(
            self.ctx, C.c_void_p(recv.data_ptr()), self.world, 0, C.c_void_p(self.work.data_ptr()), self.n,
            self.world, S, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()),
            C.c_void_p(self.flags.data_ptr()), C.c_void_p(self.h_flags.data_ptr()), self.edges,
            C.c_void_p(self.save[k].data_ptr()), C.c_void_p(escape.data_ptr()),
            C.c_void_p(self.h_counts.data_ptr())), "gather_unpack_order")
        self.ev.record()
        if self.timing:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.timing_events.append(e)
        return k

    def verdict(self) -> tuple[int, int]:
        """(escape flags summed, failures) of the last exchange (after slot_size or ev.synchronize)."""
        return int(self.h_flags[0]), int(self.h_flags[1])


class ShardedSequence:
    """Drives klt_hip_track_frames_band chunk by chunk for one rank.

    lib/ctx: the loaded library and a device context; pd/td: descriptors;
    frames: device u8 frames -- a uint8 tensor [T, H, W] (every rank holds
    them whole) or a BandFrames (the rank's rows only; build it with
    band_of(H, world, rank, margin, edges)); x/y/v: device feature arrays
    (identical on every rank at the start), on the stream the context uses.
    edges: row boundaries of the bands; default row_edges(H, world, margin),
    the bands klt_shard_create uses (equal level-0 rows built per rank).
    chunk / first_chunk: frames per band call, and of each run()'s first
    call (chunk_plan; default chunk).
    all_gather(out, inp) gathers a device int32 tensor of every rank into out
    in rank order (torch.distributed.all_gather_into_tensor in production).
    """

    def __init__(self, lib, ctx, pd, td, frames: torch.Tensor, x, y, v, rank: int, world: int, all_gather,
                 chunk: int = 64, margin: int = DEFAULT_MARGIN, edges=None, first_chunk: int | None = None):
        from .device import check
        self.lib, self.ctx, self.pd, self.td = lib, ctx, pd, td
        self.src = frames if isinstance(frames, (FullFrames, BandFrames)) else FullFrames(frames)
        self.x, self.y, self.v = x, y, v
        self.rank, self.world, self.chunk, self.first_chunk = rank, world, chunk, first_chunk
        H, W = self.src.H, self.src.W
        self.H, self.W = H, W
        # default: the C driver's bands (klt_shard_create), equal built rows per rank
        self.edges = edges = list(edges) if edges is not None else row_edges(H, world, margin)
        self.band = band_of(H, world, rank, margin, edges)
        if isinstance(self.src, BandFrames):
            ra, rb = band_rows(H, self.band)
            assert self.src.ra <= ra and self.src.rb >= rb, "BandFrames built for another band"
        self.escape = torch.zeros(1, dtype=torch.int32, device=x.device)
        # the frames are resident before run(): each build-ahead waits only for its bank
        check(lib, ctx, lib.klt_hip_set_ahead_ready(ctx, 1), "set_ahead_ready")
        self.xch = Exchange(lib, ctx, x.numel(), band_edges(H, world, edges), rank, all_gather, x.device)
        self.redone = 0
        self.rebuilt = 0  # replacements whose band pyramid was too short for the selection window
        self.t_last = None  # last tracked frame
        self._check = check

    def begin(self, t: int) -> None:
        self.t_last = t
        ptr, _ = self.src.full(t, 1)
        self._check(self.lib, self.ctx, self.lib.klt_hip_frames_begin(self.ctx, C.byref(self.pd), C.c_void_p(ptr),
                                                                      self.W), "frames_begin")

    def _band_call(self, ptr: int, stride: int, n: int, row_lo: int, row_hi: int, next_ptr: int = 0,
                   next_n: int = 0) -> None:
        b = self.band
        self._check(self.lib, self.ctx, self.lib.klt_hip_track_frames_band(
            self.ctx, C.byref(self.pd), C.byref(self.td), C.c_void_p(ptr), self.W, stride, n,
            C.c_void_p(self.x.data_ptr()), C.c_void_p(self.y.data_ptr()), C.c_void_p(self.v.data_ptr()),
            self.x.numel(), b.own_lo, b.own_hi, row_lo, row_hi, C.c_void_p(self.escape.data_ptr()),
            C.c_void_p(next_ptr) if next_n > 0 else None, next_n), "track_frames_band")

    def _redo(self, c0: int, n: int, k: int) -> None:
        """Chunk [c0, c0+n) again from whole frames and its start state (save
        buffer k), exchanged (every rank does it: they all read the same summed
        escape flag)."""
        torch.cuda.current_stream().synchronize()
        self.redone += 1
        self.xch.restore(k, self.x, self.y, self.v)
        self.xch.order(self.x, self.y, self.v, self.escape)
        S = self.xch.slot_size()
        ptr, fb = self.src.full(c0 - 1, n + 1)  # whole frames c0-1 .. c0+n-1
        self._check(self.lib, self.ctx, self.lib.klt_hip_frames_begin(
            self.ctx, C.byref(self.pd), C.c_void_p(ptr), self.W), "frames_begin")
        self._band_call(ptr + fb, fb, n, 0, self.H)
        self.xch.exchange(self.x, self.y, self.v, self.escape, S)
        self.xch.ev.synchronize()
        esc, bad = self.xch.verdict()
        if esc or bad:
            raise RuntimeError(f"a chunk redone from whole frames escaped ({esc}) or its exchange failed ({bad})")

    def run(self, t0: int, nframes: int) -> None:
        """Track frames t0 .. t0+nframes-1 (the pyramid of t0-1 must be current:
        begin(t0-1) first, or a previous run ending at t0-1).  Chunk c+1 is
        queued before chunk c's verdict is read; an escaped chunk c is redone
        and chunk c+1 runs again."""
        end = t0 + nframes
        chunks = chunk_plan(t0, nframes, self.chunk, self.first_chunk)
        k = self.xch.order(self.x, self.y, self.v, self.escape)  # the first chunk's ownership, start state, counts
        prev = None  # (c0, n, save index) of the chunk whose verdict is still unread
        i = 0
        while i < len(chunks):
            c0, n = chunks[i]
            nn = chunks[i + 1][1] if i + 1 < len(chunks) else 0  # the next chunk, built ahead
            src = self.src
            self._band_call(src.band(c0), src.stride, n, self.band.row_lo, self.band.row_hi,
                            src.band(c0 + n) if nn > 0 else 0, nn)
            S = self.xch.slot_size()  # this chunk's counts, with the previous chunk's verdict
            if prev is not None:
                esc, bad = self.xch.verdict()
                if bad:
                    raise RuntimeError(f"exchange failed on {bad} rank(s): the merged list would be wrong")
                if esc:  # the previous chunk escaped: this chunk ran from a wrong state
                    self._redo(*prev)
                    k = self.xch.k ^ 1  # the redo's exchange ordered (and saved) this chunk's start again
                    prev = None
                    continue
            k_next = self.xch.exchange(self.x, self.y, self.v, self.escape, S)
            prev = (c0, n, k)
            k = k_next
            i += 1
        self.xch.ev.synchronize()
        if prev is not None:
            esc, bad = self.xch.verdict()
            if bad:  # the unpack skipped a failed exchange: nothing was merged
                raise RuntimeError(f"exchange failed on {bad} rank(s): the merged list would be wrong")
            if esc:
                self._redo(*prev)
        self.t_last = end - 1

    # -- KLTReplaceLostFeatures across the ranks (selectGoodFeatures.c:514-541,
    # sequential mode: the last tracked frame's pyramid, :342-348) ------------
    def own_rows(self, rank: int | None = None) -> tuple[int, int]:
        """Pixel rows [lo, hi) whose trackability map rows rank computes."""
        b = self.band if rank is None else band_of(self.H, self.world, rank, 0, self.edges)
        lo = 0 if b.own_lo == float("-inf") else int(b.own_lo)
        hi = self.H if b.own_hi == float("inf") else int(b.own_hi)
        return lo, hi

    def _map_rows(self, sd, lo: int, hi: int, dev_map=None) -> tuple[int, int, int, int, int]:
        nx, ny, j0, j1 = (C.c_int() for _ in range(4))
        rc = self.lib.klt_hip_min_eigen_rows(self.ctx, C.byref(sd), lo, hi,
                                             C.c_void_p(dev_map) if dev_map is not None else None, C.byref(nx),
                                             C.byref(ny), C.byref(j0), C.byref(j1))
        if rc < 0:
            self._check(self.lib, self.ctx, rc, "min_eigen_rows")
        return rc, nx.value, ny.value, j0.value, j1.value

    def replace_rows(self, sd) -> torch.Tensor:
        """This rank's rows of the trackability map of the last tracked frame
        (a device int32 tensor in the whole map's layout; other rows 0).  A band
        pyramid too short for the selection window is rebuilt from the whole
        frame first (it becomes the previous pyramid; same values)."""
        _, nx, ny, _, _ = self._map_rows(sd, 0, 0)
        emap = torch.zeros(nx * ny, dtype=torch.int32, device=self.x.device)
        lo, hi = self.own_rows()
        rc = self._map_rows(sd, lo, hi, emap.data_ptr())[0]
        if rc == 1:
            self.rebuilt += 1
            self.begin(self.t_last)
            rc = self._map_rows(sd, lo, hi, emap.data_ptr())[0]
            assert rc == 0, "trackability rows still missing after a whole-frame build"
        return emap

    def replace_select(self, sd, mindist: int, min_eigenvalue: int, emap: torch.Tensor) -> None:
        """The host selection over the complete map (the same on every rank)."""
        self._check(self.lib, self.ctx, self.lib.klt_hip_select_map(
            self.ctx, self.W, self.H, C.byref(sd), mindist, min_eigenvalue, C.c_void_p(emap.data_ptr()),
            C.c_void_p(self.x.data_ptr()), C.c_void_p(self.y.data_ptr()), C.c_void_p(self.v.data_ptr()),
            self.x.numel()), "select_map")

    def replace(self, sd, mindist: int, min_eigenvalue: int, broadcast) -> None:
        """KLTReplaceLostFeatures between two run() calls: each rank's map rows
        to every rank (broadcast(tensor, src) in place, torch.distributed.broadcast
        in production), then the same selection everywhere."""
        emap = self.replace_rows(sd)
        _, nx, _, _, _ = self._map_rows(sd, 0, 0)
        for r in range(self.world):
            _, _, _, j0, j1 = self._map_rows(sd, *self.own_rows(r))
            if j1 > j0:
                part = emap[j0 * nx:j1 * nx]
                broadcast(part, r)
        self.replace_select(sd, mindist, min_eigenvalue, emap)
