"""End-to-end klt.h API on the GPU vs the reference's golden outputs and the
CPU oracle.  Exact mode: positions and status codes bit-identical in every
(feature, frame) cell except the never-written last column (example3.c:71)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import synth
from kltabi import GOLDEN, KLTRunner, OracleParams, OracleTracker, ft_bytes, parse_ft
from test_oracle import table_eq

pytestmark = pytest.mark.gpu


def test_v1_golden(gpu, frames):
    got = KLTRunner(gpu).harness(frames, 150, 10, first=frames[0])
    assert table_eq(got, parse_ft((GOLDEN / "v1_features2.ft").read_bytes()))


@pytest.mark.parametrize("n", [100, 150])
def test_config1_golden(gpu, frames, n):
    got = KLTRunner(gpu).harness(frames, n, 10)
    assert table_eq(got, parse_ft((GOLDEN / f"config1_{n}x10.ft").read_bytes()))


def test_config1_replace_golden(gpu, frames):
    got = KLTRunner(gpu).harness(frames, 150, 10, replace=True)
    assert table_eq(got, parse_ft((GOLDEN / "seq_config1_replace_150x10.ft").read_bytes()))


def test_synthetic_golden(gpu, syn640, syn333):
    got = KLTRunner(gpu).harness(syn640, 1000, 12)
    assert table_eq(got, parse_ft((GOLDEN / "seq_syn640_1000x12.ft").read_bytes()))
    got = KLTRunner(gpu).harness(syn333, 300, 8)
    assert table_eq(got, parse_ft((GOLDEN / "seq_syn333x251_300x8.ft").read_bytes()))


def test_non_sequential_mode(gpu, oracle, syn640):
    got = KLTRunner(gpu).harness(syn640, 500, 8, sequential=False)
    want = OracleTracker(oracle).harness(syn640, 500, 8)  # same results by construction
    assert table_eq(got, want)


def run_both(gpu, oracle, frames, n, nframes, setup, search=None, replace=False):
    tc = gpu.KLTCreateTrackingContext()
    setup(tc.contents)
    if search is not None:
        gpu.KLTChangeTCPyramid(tc, search)
    gpu.KLTUpdateTCBorder(tc)
    p = OracleParams.from_tc(tc.contents)
    t = tc.contents

    def full(tt):
        setup(tt)
        tt.nPyramidLevels, tt.subsampling = t.nPyramidLevels, t.subsampling
        tt.borderx, tt.bordery = t.borderx, t.bordery

    got = KLTRunner(gpu).harness(frames, n, nframes, tc_setup=full, replace=replace)
    gpu.KLTFreeTrackingContext(tc)
    want = OracleTracker(oracle, p).harness(frames, n, nframes, replace=replace)
    return got, want


CASES = {
    "win5": (lambda t: setattr(t, "window_width", 5) or setattr(t, "window_height", 5), None),
    "win9x7": (lambda t: setattr(t, "window_width", 9), None),
    "win15": (lambda t: setattr(t, "window_width", 15) or setattr(t, "window_height", 15), None),
    "ss2": (lambda t: None, 6),
    "levels3": (lambda t: None, 120),
    "lighting": (lambda t: setattr(t, "lighting_insensitive", 1), None),
    "step2": (lambda t: setattr(t, "step_factor", 2.0), None),
    "maxit3": (lambda t: setattr(t, "max_iterations", 3), None),
    "residue3": (lambda t: setattr(t, "max_residue", 3.0), None),
}


@pytest.mark.parametrize("name", list(CASES))
def test_nondefault_vs_oracle(gpu, oracle, syn333, name):
    setup, search = CASES[name]
    got, want = run_both(gpu, oracle, syn333, 200, 8, setup, search)
    assert table_eq(got, want), name


def test_replace_vs_oracle(gpu, oracle, syn640):
    got, want = run_both(gpu, oracle, syn640, 300, 12, lambda t: None, replace=True)
    assert table_eq(got, want)


def test_hd_vs_oracle(gpu, oracle):
    """BASELINE config 3 shape (1920x1080, 5000 features) on a few frames."""
    fr = synth(gpu, 1080, 1920, 1080, 4)
    got = KLTRunner(gpu).harness(fr, 5000, 4)
    want = OracleTracker(oracle).harness(fr, 5000, 4)
    assert table_eq(got, want)
    assert (got[2][:, 1] == 0).sum() > 4000


def test_device_numerics(gpu):
    """f64 sqrt and f32 division on gfx950 are correctly rounded (numpy == IEEE)."""
    import kltamd
    from kltamd.device import check
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.random(200000) * 10.0 ** rng.integers(-30, 30, 200000),
                        np.array([0.0, 1.0, 2.0, 4.0, 1e-310, 1.7e308])])
    out = np.empty_like(x)
    DP = C.POINTER(C.c_double)
    check(gpu, ctx, gpu.klt_hip_selftest_sqrt(ctx, x.ctypes.data_as(DP), out.ctypes.data_as(DP), x.size), "sqrt")
    assert np.array_equal(out, np.sqrt(x))
    a = (rng.standard_normal(200000) * 1e3).astype(np.float32)
    b = (rng.standard_normal(200000) * 1e-2).astype(np.float32)
    q = np.empty_like(a)
    FP = C.POINTER(C.c_float)
    check(gpu, ctx, gpu.klt_hip_selftest_div(ctx, a.ctypes.data_as(FP), b.ctypes.data_as(FP),
                                             q.ctypes.data_as(FP), a.size), "div")
    assert np.array_equal(q.view(np.int32), (a / b).view(np.int32))
    gpu.KLTFreeTrackingContext(tc)


def test_device_synth_matches_host(gpu):
    from kltamd.device import D2H, check
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    w, h, n = 333, 251, 3
    buf = gpu.klt_hip_malloc(ctx, w * h * n)
    check(gpu, ctx, gpu.klt_hip_synth_frames(ctx, 333, 0, n, w, h, buf, w, w * h), "synth")
    out = np.empty((n, h, w), np.uint8)
    check(gpu, ctx, gpu.klt_hip_memcpy(ctx, out.ctypes.data, buf, out.nbytes, D2H), "d2h")
    gpu.klt_hip_free(ctx, buf)
    host = synth(gpu, 333, w, h, n)
    for t in range(n):
        assert np.array_equal(out[t], host[t])
    gpu.KLTFreeTrackingContext(tc)


def test_stop_sequential_and_size_change(gpu, syn640):
    from kltabi import u8ptr
    lib = gpu
    tc = lib.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    fl = lib.KLTCreateFeatureList(50)
    a, b = syn640[0], syn640[1]
    lib.KLTSelectGoodFeatures(tc, u8ptr(a), 640, 480, fl)
    assert not tc.contents.pyramid_last
    lib.KLTTrackFeatures(tc, u8ptr(a), u8ptr(b), 640, 480, fl)
    assert tc.contents.pyramid_last and tc.contents.pyramid_last_gradx
    lib.KLTStopSequentialMode(tc)
    assert not tc.contents.pyramid_last and tc.contents.sequentialMode == 0
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)


def device_sequence(gpu, frames, nfeat, setup=None, reduction=0):
    """Select on frames[0], then klt_hip_track_sequence over frames[1:] with
    frames and features resident on the device (the path bench.py times)."""
    from kltabi import fl_to_arrays, u8ptr
    from kltamd.device import D2H, H2D, PyrDesc, TrackDesc, check
    h, w = frames[0].shape
    tc = gpu.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    if setup:
        setup(tc.contents)
    gpu.klt_amd_set_reduction(tc, reduction)
    ctx = gpu.klt_amd_device_context(tc)
    fl = gpu.KLTCreateFeatureList(nfeat)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(frames[0])), w, h, fl)
    x, y, v = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    stack = np.ascontiguousarray(np.stack(frames))
    dfr = gpu.klt_hip_malloc(ctx, stack.nbytes)
    dx, dy, dv = (gpu.klt_hip_malloc(ctx, 4 * nfeat) for _ in range(3))
    check(gpu, ctx, gpu.klt_hip_memcpy(ctx, dfr, stack.ctypes.data, stack.nbytes, H2D), "h2d")
    for d, a in ((dx, x), (dy, y), (dv, v)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, d, a.ctypes.data, a.nbytes, H2D), "h2d")
    pd, td = PyrDesc(), TrackDesc()
    gpu.klt_amd_pyr_desc(tc, w, h, tc.contents.nPyramidLevels, 1, C.byref(pd))
    gpu.klt_amd_track_desc(tc, C.byref(td))
    check(gpu, ctx, gpu.klt_hip_build_pyramid(ctx, 0, C.byref(pd), dfr, w, 0), "build")
    slot = C.c_int(0)
    check(gpu, ctx, gpu.klt_hip_track_sequence(ctx, C.byref(pd), C.byref(td), dfr, w, w * h, 1,
                                               len(frames) - 1, dx, dy, dv, nfeat, C.byref(slot)), "seq")
    for d, a in ((dx, x), (dy, y), (dv, v)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, a.ctypes.data, d, a.nbytes, D2H), "d2h")
    for d in (dfr, dx, dy, dv):
        gpu.klt_hip_free(ctx, d)
    gpu.KLTFreeTrackingContext(tc)
    return x, y, v


@pytest.mark.parametrize("shape,nfeat,nframes", [((480, 640), 1000, 12), ((251, 333), 300, 9),
                                                 ((1080, 1920), 5000, 6)])
def test_pipelined_device_sequence_vs_oracle(gpu, oracle, shape, nfeat, nframes):
    h, w = shape
    frames = synth(gpu, 4242 + w, w, h, nframes)
    x, y, v = device_sequence(gpu, frames, nfeat)
    X, Y, V = OracleTracker(oracle).harness(frames, nfeat, nframes, first=frames[0])
    k = nframes - 2  # column of the last tracked frame
    assert np.array_equal(x.view(np.int32), X[:, k].view(np.int32))
    assert np.array_equal(y.view(np.int32), Y[:, k].view(np.int32))
    assert np.array_equal(v, V[:, k])


def test_pipelined_generic_path_vs_oracle(gpu, oracle):
    """Non-default parameters: the pipeline drives the generic pyramid path."""
    frames = synth(gpu, 99, 333, 251, 7)

    def setup(t):
        t.window_width = t.window_height = 9

    x, y, v = device_sequence(gpu, frames, 200, setup)
    tc = gpu.KLTCreateTrackingContext()
    setup(tc.contents)
    p = OracleParams.from_tc(tc.contents)
    gpu.KLTFreeTrackingContext(tc)
    X, Y, V = OracleTracker(oracle, p).harness(frames, 200, 7, first=frames[0])
    assert np.array_equal(x.view(np.int32), X[:, 5].view(np.int32)) and np.array_equal(v, V[:, 5])


def batch_sequence(gpu, frames, nfeat, chunks, setup=None, calls=None, counts=None, ctx_hook=None):
    """Select on frames[0], then klt_hip_frames_begin + klt_hip_track_frames over
    frames[1:] (split into `calls` pieces, one chunk size per call), returning
    the device feature table: row j = the list after frame j+1.  counts (a
    list): the tracker's work counters (klt_hip_set_track_count) are appended.
    ctx_hook(ctx) runs before the first call and after the last (with
    done=True)."""
    from kltabi import fl_to_arrays, u8ptr
    from kltamd.device import D2H, H2D, PyrDesc, TrackDesc, check
    h, w = frames[0].shape
    tc = gpu.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    if setup:
        setup(tc.contents)
    ctx = gpu.klt_amd_device_context(tc)
    fl = gpu.KLTCreateFeatureList(nfeat)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(frames[0])), w, h, fl)
    x, y, v = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    stack = np.ascontiguousarray(np.stack(frames))
    T = len(frames) - 1
    dfr = gpu.klt_hip_malloc(ctx, stack.nbytes)
    dx, dy, dv = (gpu.klt_hip_malloc(ctx, 4 * nfeat) for _ in range(3))
    tx, ty, tv = (gpu.klt_hip_malloc(ctx, 4 * nfeat * T) for _ in range(3))
    check(gpu, ctx, gpu.klt_hip_memcpy(ctx, dfr, stack.ctypes.data, stack.nbytes, H2D), "h2d")
    for d, a in ((dx, x), (dy, y), (dv, v)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, d, a.ctypes.data, a.nbytes, H2D), "h2d")
    pd, td = PyrDesc(), TrackDesc()
    gpu.klt_amd_pyr_desc(tc, w, h, tc.contents.nPyramidLevels, 1, C.byref(pd))
    gpu.klt_amd_track_desc(tc, C.byref(td))
    check(gpu, ctx, gpu.klt_hip_frames_begin(ctx, C.byref(pd), dfr, w), "begin")
    if ctx_hook:
        ctx_hook(ctx)
    if counts is not None:
        check(gpu, ctx, gpu.klt_hip_set_track_count(ctx, 1), "count on")
    calls = calls or [T]
    assert sum(calls) == T and len(chunks) == len(calls)
    j0 = 0
    for nf, ch in zip(calls, chunks):
        off = 4 * nfeat * j0
        check(gpu, ctx, gpu.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), dfr + (1 + j0) * w * h, w, w * h,
                                                 nf, ch, dx, dy, dv, nfeat, tx + off, ty + off, tv + off,
                                                 nfeat), "frames")
        j0 += nf
    if ctx_hook:
        ctx_hook(ctx, done=True)
    if counts is not None:
        solves, passes = C.c_ulonglong(0), C.c_ulonglong(0)
        check(gpu, ctx, gpu.klt_hip_get_track_count(ctx, C.byref(solves), C.byref(passes), 1), "count")
        counts += [solves.value, passes.value]
        check(gpu, ctx, gpu.klt_hip_set_track_count(ctx, 0), "count off")
    X = np.empty((T, nfeat), np.float32)
    Y = np.empty((T, nfeat), np.float32)
    V = np.empty((T, nfeat), np.int32)
    for d, a in ((tx, X), (ty, Y), (tv, V)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, a.ctypes.data, d, a.nbytes, D2H), "d2h")
    for d, a in ((dx, x), (dy, y), (dv, v)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, a.ctypes.data, d, a.nbytes, D2H), "d2h")
    for d in (dfr, dx, dy, dv, tx, ty, tv):
        gpu.klt_hip_free(ctx, d)
    gpu.KLTFreeTrackingContext(tc)
    assert np.array_equal(X[-1], x) and np.array_equal(V[-1], v)  # final list == last table row
    return X, Y, V


def assert_table_equal(X, Y, V, OX, OY, OV):
    T = X.shape[0]
    for j in range(T):
        assert np.array_equal(V[j], OV[:, j]), f"val differs at frame {j + 1}"
        assert np.array_equal(X[j].view(np.int32), OX[:, j].view(np.int32)), f"x differs at frame {j + 1}"
        assert np.array_equal(Y[j].view(np.int32), OY[:, j].view(np.int32)), f"y differs at frame {j + 1}"


@pytest.mark.parametrize("chunks,calls", [([1], None), ([4], None), ([5], None), ([64], None),
                                          ([2, 7], [3, 8])])
def test_batched_frames_vs_oracle(gpu, oracle, chunks, calls):
    frames = synth(gpu, 5150, 640, 480, 12)
    X, Y, V = batch_sequence(gpu, frames, 1000, chunks, calls=calls)
    OX, OY, OV = OracleTracker(oracle).harness(frames, 1000, 12, first=frames[0])
    assert_table_equal(X, Y, V, OX, OY, OV)


@pytest.mark.parametrize("merge", [1, 0])
def test_track_counts_vs_oracle(gpu, oracle, merge):
    """klt_hip_set_track_count: the device's count of 2x2 systems formed equals
    the oracle's Newton loop bodies (both levels, SMALL_DET included) over the
    same sequence, with the deferred residue on and off; the gather passes are
    at least one per system."""
    frames = synth(gpu, 5150, 640, 480, 12)
    counts = []
    X, Y, V = batch_sequence_opts(gpu, frames, 1000, 5, dict(merge=merge), counts=counts)
    oracle.orc_solve_count(1)
    OX, OY, OV = OracleTracker(oracle).harness(frames, 1000, 12, first=frames[0])
    assert_table_equal(X, Y, V, OX, OY, OV)
    solves, passes = counts
    assert solves == oracle.orc_solve_count(1) and solves > 0
    assert passes >= solves


def test_batched_frames_odd_size_and_1080p(gpu, oracle):
    frames = synth(gpu, 333, 333, 251, 9)
    X, Y, V = batch_sequence(gpu, frames, 300, [3])
    assert_table_equal(X, Y, V, *OracleTracker(oracle).harness(frames, 300, 9, first=frames[0]))
    frames = synth(gpu, 1080, 1920, 1080, 6)
    X, Y, V = batch_sequence(gpu, frames, 5000, [16])
    assert_table_equal(X, Y, V, *OracleTracker(oracle).harness(frames, 5000, 6, first=frames[0]))


def test_batched_frames_generic_path(gpu, oracle):
    """Non-default window: pyramids come from the generic kernels, copied into the bank."""
    frames = synth(gpu, 98, 333, 251, 8)

    def setup(t):
        t.window_width = t.window_height = 9

    X, Y, V = batch_sequence(gpu, frames, 200, [3], setup)
    tc = gpu.KLTCreateTrackingContext()
    setup(tc.contents)
    p = OracleParams.from_tc(tc.contents)
    gpu.KLTFreeTrackingContext(tc)
    assert_table_equal(X, Y, V, *OracleTracker(oracle, p).harness(frames, 200, 8, first=frames[0]))


def test_batched_frames_errors(gpu):
    from kltamd.device import PyrDesc, TrackDesc
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    pd, td = PyrDesc(), TrackDesc()
    gpu.klt_amd_pyr_desc(tc, 64, 48, tc.contents.nPyramidLevels, 1, C.byref(pd))
    gpu.klt_amd_track_desc(tc, C.byref(td))
    # no klt_hip_frames_begin yet
    assert gpu.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), None, 64, 64 * 48, 0, 1, None, None, None,
                                    0, None, None, None, 0) < 0
    assert b"frames_begin" in gpu.klt_hip_last_error(ctx)
    gpu.KLTFreeTrackingContext(tc)


def test_reference_harness_relinked(gpu):
    """The reference's own example3.c, compiled unchanged and linked against
    libklt_amd.so (oracle/ref.mk -> oracle/_ref/example3_amd), reproduces the
    reference's config-1 output byte for byte."""
    import os
    import subprocess
    import tempfile
    from pathlib import Path
    exe = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "example3_amd"
    if not exe.exists():
        pytest.skip("oracle/_ref/example3_amd not built (needs /root/reference at build time)")
    for n in (100, 150):
        with tempfile.TemporaryDirectory() as d:
            run = Path(d) / "a" / "b"
            (run / "feat").mkdir(parents=True)
            (Path(d) / "data").mkdir()
            os.symlink(GOLDEN / "images_provided", Path(d) / "data" / "images_provided")
            subprocess.run([str(exe), "images_provided", str(n), "10"], cwd=run, check=True, capture_output=True,
                           timeout=120)
            got = (run / "feat" / "features2.ft").read_bytes()
            txt = (run / "feat" / "features2.txt").read_bytes()
        want = (GOLDEN / f"config1_{n}x10.ft").read_bytes()
        assert table_eq(parse_ft(got), parse_ft(want)), f"{n} features: .ft differs from the reference"
        assert txt.splitlines()[:2] == (GOLDEN / f"config1_{n}x10.txt").read_bytes().splitlines()[:2]


def _edge_positions():
    """Window centres where x+i / y+j round across an integer for some window
    pixel (just below a power of two), plus ordinary ones: exercises both the
    lane-patch gather and its per-pixel fallback."""
    f32 = np.float32
    xs, ys = [], []
    for base in (64.0, 128.0, 256.0, 512.0):
        for d in (-3, -2, -1, 1, 2):
            xs.append(np.nextafter(f32(base), f32(0)) if d == -1 else f32(base) + f32(d) * f32(1e-5))
            ys.append(f32(200.25) + f32(d))
    for d in range(8):
        xs.append(f32(300.5) + f32(d) * f32(0.37))
        ys.append(np.nextafter(f32(256.0), f32(0)) if d % 2 else f32(128.0) - f32(3e-6))
    return np.array(xs, np.float32), np.array(ys, np.float32)


@pytest.mark.parametrize("patch", [1, 0])
def test_patch_gather_edge_positions(gpu, oracle, patch):
    from kltabi import arrays_to_fl, fl_to_arrays, u8ptr
    frames = synth(gpu, 777, 640, 480, 2)
    x0, y0 = _edge_positions()
    n = len(x0)
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    assert gpu.klt_hip_set_track_patch(ctx, patch) == 0
    fl = gpu.KLTCreateFeatureList(n)
    arrays_to_fl(fl, x0, y0, np.zeros(n, np.int32))
    gpu.KLTTrackFeatures(tc, u8ptr(frames[0]), u8ptr(frames[1]), 640, 480, fl)
    gx, gy, gv = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    gpu.KLTFreeTrackingContext(tc)
    ox, oy, ov = x0.copy(), y0.copy(), np.zeros(n, np.int32)
    ot = OracleTracker(oracle)
    ot.params.sequentialMode = 0
    oracle.orc_set_params(ot.h, C.byref(ot.params))
    ot.track(frames[0], frames[1], ox, oy, ov)
    assert np.array_equal(gv, ov)
    assert np.array_equal(gx.view(np.int32), ox.view(np.int32))
    assert np.array_equal(gy.view(np.int32), oy.view(np.int32))


@pytest.mark.parametrize("opts", [dict(patch=0), dict(order=1, patch=1), dict(chunk=7), dict(merge=0),
                                  dict(merge=0, patch=0), dict(order=1, patch=0, chunk=3)])
def test_tracker_tuning_hooks_do_not_change_results(gpu, oracle, opts):
    """Lane patch, processing order, deferred residue and chunking only
    reorganise work."""
    frames = synth(gpu, 5151, 640, 480, 8)
    X, Y, V = batch_sequence_opts(gpu, frames, 3000, 4, opts)
    assert_table_equal(X, Y, V, *OracleTracker(oracle).harness(frames, 3000, 8, first=frames[0]))


@pytest.mark.parametrize("opts", [dict(overlap=1), dict(overlap=0), dict(overlap=1, merge=0), dict(overlap=1, prio=0)])
def test_overlapped_schedule_1080p(gpu, oracle, opts):
    """The bench's overlapped schedule -- pyramids of chunk c+1 built on their
    own stream while chunk c is tracked -- over several chunks (chunk 3, 10
    frames, 5000 features): bit-identical to the oracle, as one stream is."""
    frames = synth(gpu, 1080, 1920, 1080, 11)
    X, Y, V = batch_sequence_opts(gpu, frames, 5000, 3, opts)
    assert_table_equal(X, Y, V, *OracleTracker(oracle).harness(frames, 5000, 11, first=frames[0]))


def batch_sequence_opts(gpu, frames, nfeat, chunk, opts, counts=None):
    """batch_sequence with the tuning hooks applied to its device context."""
    orig = gpu.klt_amd_device_context

    def hooked(tc):
        ctx = orig(tc)
        assert gpu.klt_hip_set_track_patch(ctx, opts.get("patch", 1)) == 0
        assert gpu.klt_hip_set_track_order(ctx, opts.get("order", 0)) == 0
        assert gpu.klt_hip_set_frames_overlap(ctx, opts.get("overlap", 0)) == 0
        assert gpu.klt_hip_set_track_merge(ctx, opts.get("merge", 1)) == 0
        assert gpu.klt_hip_set_track_prio(ctx, opts.get("prio", 1)) == 0
        return ctx

    gpu.klt_amd_device_context = hooked
    try:
        return batch_sequence(gpu, frames, nfeat, [opts.get("chunk", chunk)], counts=counts)
    finally:
        gpu.klt_amd_device_context = orig


def _seq_via_api(gpu, frames, nfeat, sequential=True, first_call=False):
    """KLTTrackSequence over frames (selection on frames[0]); optionally one
    KLTTrackFeatures call first so that sequential mode starts from a kept pyramid."""
    from kltabi import fl_to_arrays, u8ptr
    h, w = frames[0].shape
    tc = gpu.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1 if sequential else 0
    fl = gpu.KLTCreateFeatureList(nfeat)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(frames[0])), w, h, fl)
    seq = frames
    if first_call:
        gpu.KLTTrackFeatures(tc, u8ptr(frames[0]), u8ptr(frames[1]), w, h, fl)
        seq = frames[1:]
    T = len(seq) - 1
    ft = gpu.KLTCreateFeatureTable(T, nfeat)
    keep = [np.ascontiguousarray(f) for f in seq]
    arr = (C.POINTER(C.c_ubyte) * len(keep))(*[u8ptr(f) for f in keep])
    gpu.KLTTrackSequence(tc, arr, len(keep), w, h, fl, ft, 0)
    X = np.array([[ft.contents.feature[j][i].contents.x for i in range(T)] for j in range(nfeat)], np.float32)
    Y = np.array([[ft.contents.feature[j][i].contents.y for i in range(T)] for j in range(nfeat)], np.float32)
    V = np.array([[ft.contents.feature[j][i].contents.val for i in range(T)] for j in range(nfeat)], np.int32)
    x, y, v = fl_to_arrays(fl)
    gpu.KLTFreeFeatureTable(ft)
    gpu.KLTFreeFeatureList(fl)
    gpu.KLTFreeTrackingContext(tc)
    return X, Y, V, (x, y, v)


@pytest.mark.parametrize("sequential,first_call", [(True, False), (False, False), (True, True)])
def test_track_sequence_api_vs_loop(gpu, oracle, sequential, first_call):
    """KLTTrackSequence == the per-frame KLTTrackFeatures + KLTStoreFeatureList loop (oracle)."""
    frames = synth(gpu, 6060, 640, 480, 40)  # > one 32-frame chunk
    X, Y, V, last = _seq_via_api(gpu, frames, 800, sequential, first_call)
    OX, OY, OV = OracleTracker(oracle).harness(frames, 800, 40, first=frames[0])
    off = 1 if first_call else 0
    T = X.shape[1]
    assert np.array_equal(V, OV[:, off:off + T])
    assert np.array_equal(X.view(np.int32), OX[:, off:off + T].view(np.int32))
    assert np.array_equal(Y.view(np.int32), OY[:, off:off + T].view(np.int32))
    assert np.array_equal(last[2], OV[:, off + T - 1])


def test_track_sequence_then_track_features(gpu, oracle):
    """Sequential mode: a KLTTrackFeatures call after KLTTrackSequence continues
    from the sequence's last pyramid, exactly like after the per-frame loop."""
    from kltabi import fl_to_arrays, u8ptr
    frames = synth(gpu, 6161, 333, 251, 9)
    h, w = frames[0].shape
    tc = gpu.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    fl = gpu.KLTCreateFeatureList(300)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(frames[0]), w, h, fl)
    keep = [np.ascontiguousarray(f) for f in frames[:6]]
    arr = (C.POINTER(C.c_ubyte) * 6)(*[u8ptr(f) for f in keep])
    gpu.KLTTrackSequence(tc, arr, 6, w, h, fl, None, 0)
    for t in range(6, 9):  # img1 is ignored in sequential mode: pass garbage
        junk = np.zeros_like(frames[0])
        gpu.KLTTrackFeatures(tc, u8ptr(junk), u8ptr(frames[t]), w, h, fl)
    x, y, v = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    gpu.KLTFreeTrackingContext(tc)
    OX, OY, OV = OracleTracker(oracle).harness(frames, 300, 9, first=frames[0])
    assert np.array_equal(v, OV[:, 7]) and np.array_equal(x.view(np.int32), OX[:, 7].view(np.int32))


@pytest.mark.parametrize("band", [False, True])
def test_processing_order_many_features(gpu, oracle, band):
    """k_band_order past its LDS bucket cache (40 000 features: a selected list
    repeated, every fifth copy lost): every live copy tracks exactly like the
    oracle's single list, lost copies are left alone; in band mode only the
    copies whose y lies in the band move."""
    from kltabi import fl_to_arrays, u8ptr
    from kltamd.device import D2H, H2D, PyrDesc, TrackDesc, check
    w, h, T, rep = 640, 480, 4, 27
    frames = synth(gpu, 4242, w, h, T + 1)
    tc = gpu.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    ctx = gpu.klt_amd_device_context(tc)
    fl = gpu.KLTCreateFeatureList(1500)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(frames[0])), w, h, fl)
    x1, y1, v1 = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    x, y, v = np.tile(x1, rep), np.tile(y1, rep), np.tile(v1, rep)
    m = len(x1)
    for c in range(0, rep, 5):
        v[c * m:(c + 1) * m] = -1
    n = len(x)
    assert n > 32768
    stack = np.ascontiguousarray(np.stack(frames))
    dfr = gpu.klt_hip_malloc(ctx, stack.nbytes)
    dx, dy, dv = (gpu.klt_hip_malloc(ctx, 4 * n) for _ in range(3))
    esc = gpu.klt_hip_malloc(ctx, 4)
    zero = np.zeros(1, np.int32)
    check(gpu, ctx, gpu.klt_hip_memcpy(ctx, dfr, stack.ctypes.data, stack.nbytes, H2D), "h2d")
    check(gpu, ctx, gpu.klt_hip_memcpy(ctx, esc, zero.ctypes.data, 4, H2D), "h2d")
    for d, a in ((dx, x), (dy, y), (dv, v)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, d, a.ctypes.data, a.nbytes, H2D), "h2d")
    pd, td = PyrDesc(), TrackDesc()
    gpu.klt_amd_pyr_desc(tc, w, h, tc.contents.nPyramidLevels, 1, C.byref(pd))
    gpu.klt_amd_track_desc(tc, C.byref(td))
    check(gpu, ctx, gpu.klt_hip_frames_begin(ctx, C.byref(pd), dfr, w), "begin")
    lo, hi = 120.0, 330.0
    if band:
        check(gpu, ctx, gpu.klt_hip_track_frames_band(ctx, C.byref(pd), C.byref(td), dfr + w * h, w, w * h, T, dx, dy,
                                                      dv, n, lo, hi, 0, h, esc, None, 0), "band")
    else:
        check(gpu, ctx, gpu.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), dfr + w * h, w, w * h, T, 2, dx, dy,
                                                 dv, n, None, None, None, 0), "frames")
    gx, gy, gv, ge = np.empty_like(x), np.empty_like(y), np.empty_like(v), np.zeros(1, np.int32)
    for d, a in ((dx, gx), (dy, gy), (dv, gv), (esc, ge)):
        check(gpu, ctx, gpu.klt_hip_memcpy(ctx, a.ctypes.data, d, a.nbytes, D2H), "d2h")
    for d in (dfr, dx, dy, dv, esc):
        gpu.klt_hip_free(ctx, d)
    gpu.KLTFreeTrackingContext(tc)
    ox, oy, ov = x1.copy(), y1.copy(), v1.copy()
    ot = OracleTracker(oracle)
    for j in range(T):
        ot.track(frames[j], frames[j + 1], ox, oy, ov)
    assert ge[0] == 0
    for c in range(rep):
        s = slice(c * m, (c + 1) * m)
        moved = v[s] >= 0
        if band:
            moved &= (y[s] >= lo) & (y[s] < hi)
        ex = np.where(moved, ox, x[s])
        ey = np.where(moved, oy, y[s])
        ev = np.where(moved, ov, v[s])
        assert np.array_equal(gv[s], ev), c
        assert np.array_equal(gx[s].view(np.int32), ex.view(np.int32)), c
        assert np.array_equal(gy[s].view(np.int32), ey.view(np.int32)), c
