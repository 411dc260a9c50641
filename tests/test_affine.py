"""The affine consistency check of KLTTrackFeatures (trackFeatures.c:503-1225,
:1438-1497; tc->affineConsistencyCheck 0 = translation, 1 = similarity,
2 = full affine).

Fixtures (tests/golden/affine_*.npz) are the reference's own outputs
(tests/golden/make_golden.py, oracle/_ref built from /root/reference): per
frame, the list's x/y/val and every feature's affine state -- aff_x, aff_y,
Axx, Ayx, Axy, Ayy and the crc32 of the stored img/gradx/grady window.  The
bar is bit-exact in every field (the last .ft column excepted, example3.c:71).
"""
from __future__ import annotations

import numpy as np
import pytest

from kltabi import (GOLDEN, OracleTracker, TrackingContextRec, affine_setup, load_dataset, run_affine)

import sys
sys.path.insert(0, str(GOLDEN))
from make_golden import AFFINE_CASES, affine_inputs  # noqa: E402

CASES = {c[0]: c for c in AFFINE_CASES}
FIELDS = ("X", "Y", "V", "AFF", "HAS", "CRC")


def mismatches(got, want) -> list[tuple[str, int]]:
    bad = []
    for name, a, b in zip(FIELDS, got, want):
        if name in "XYV":  # the never-written last column of the table
            a, b = a[:, :-1], b[:, :-1]
        a, b = np.asarray(a), np.asarray(b)
        if a.dtype == np.float32:  # bit patterns: -0.0 / NaN payloads count
            a, b = a.view(np.uint32), b.view(np.uint32)
        if a.shape != b.shape or not np.array_equal(a, b):
            bad.append((name, int((a != b).sum()) if a.shape == b.shape else -1))
    return bad


def golden(name):
    d = np.load(GOLDEN / f"{name}.npz")
    return tuple(d[k] for k in FIELDS)


def oracle_run(oracle, name):
    _, data, n, nf, replace, kw = CASES[name]
    tc = TrackingContextRec()
    affine_setup(**kw)(tc)
    o = OracleTracker(oracle)
    o.params.lighting_insensitive = tc.lighting_insensitive
    return o.harness_affine(affine_inputs(data), n, nf, tc, replace=replace)


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_affine_golden(oracle, name):
    assert mismatches(oracle_run(oracle, name), golden(name)) == []


def test_affine_fixtures_exercise_the_check():
    """The fixtures cover every branch worth pinning: windows stored and
    re-tracked, features lost by the affine stage, A moved off identity."""
    for name in ("affine_m1_100x10", "affine_m2_100x10", "affine_m2_warp_200x8"):
        X, Y, V, A, H, K = golden(name)
        assert H[-1].sum() > 20
        assert np.abs(A[-1][H[-1] == 1][:, 2:] - [1, 0, 0, 1]).max() > 0.02
        # a feature that had a window and lost it in a later frame
        assert ((H[:-1] == 1) & (H[1:] == 0)).any()
    X, Y, V, A, H, K = golden("affine_m0_100x10")
    assert (A[:, :, 2:] == np.array([1, 0, 0, 1], np.float32)).all()  # mode 0 keeps A


def test_oracle_affine_live_reference(oracle, ref, syn333):
    """A case no fixture holds, against the reference compiled here."""
    setup = affine_setup(mode=2, window=9, max_it=6, min_disp=0.05)
    want = run_affine(ref, syn333, 300, 8, setup)
    tc = TrackingContextRec()
    setup(tc)
    got = OracleTracker(oracle).harness_affine(syn333, 300, 8, tc)
    assert mismatches(got, want) == []


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_affine_golden(gpu, name):
    _, data, n, nf, replace, kw = CASES[name]
    got = run_affine(gpu, affine_inputs(data), n, nf, affine_setup(**kw), replace=replace)
    assert mismatches(got, golden(name)) == []


@pytest.mark.gpu
def test_gpu_affine_vs_oracle_synthetic(gpu, oracle, syn640):
    """640x480, 1000 features, mode 2 with a small window and a loose
    displacement bound: GPU == oracle in every field."""
    setup = affine_setup(mode=2, window=9, mdd=2.5)
    got = run_affine(gpu, syn640, 1000, 12, setup)
    tc = TrackingContextRec()
    setup(tc)
    want = OracleTracker(oracle).harness_affine(syn640, 1000, 12, tc)
    assert mismatches(got, want) == []


@pytest.mark.gpu
def test_gpu_affine_not_sequential(gpu, oracle, frames):
    """Non-sequential mode (both pyramids rebuilt per call) with mode 1."""
    setup = affine_setup(mode=1)

    def full(tc):
        setup(tc)
        tc.sequentialMode = 0

    from kltabi import KLTRunner, fl_affine
    A = []
    X, Y, V = KLTRunner(gpu).harness(frames, 100, 10, sequential=False, tc_setup=full,
                                     on_frame=lambda i, fl: A.append(fl_affine(fl)[0]))
    want = golden("affine_m1_100x10")
    assert np.array_equal(V[:, :-1], want[2][:, :-1])
    assert np.array_equal(np.stack(A).view(np.uint32), want[3].view(np.uint32))


@pytest.mark.gpu
def test_gpu_track_sequence_affine(gpu, oracle):
    """KLTTrackSequence with the affine check runs it in every call, like the
    KLTTrackFeatures + KLTStoreFeatureList loop (oracle), affine state included."""
    import ctypes as C
    from kltabi import fl_affine, fl_to_arrays, u8ptr
    frames = list(np.load(GOLDEN / "warp_frames.npz")["frames"])
    setup = affine_setup(mode=2)
    h, w = frames[0].shape
    tc = gpu.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    setup(tc.contents)
    fl = gpu.KLTCreateFeatureList(200)
    gpu.KLTSelectGoodFeatures(tc, u8ptr(frames[0]), w, h, fl)
    keep = [np.ascontiguousarray(f) for f in frames]
    arr = (C.POINTER(C.c_ubyte) * len(keep))(*[u8ptr(f) for f in keep])
    gpu.KLTTrackSequence(tc, arr, len(keep), w, h, fl, None, 0)
    x, y, v = fl_to_arrays(fl)
    aff, has, crc = fl_affine(fl)
    gpu.KLTFreeFeatureList(fl)
    gpu.KLTFreeTrackingContext(tc)
    t = TrackingContextRec()
    setup(t)
    X, Y, V, A, H, K = OracleTracker(oracle).harness_affine(frames, 200, len(frames), t, first=frames[0])
    assert np.array_equal(v, V[:, -2]) and np.array_equal(x.view(np.int32), X[:, -2].view(np.int32))
    assert np.array_equal(aff.view(np.int32), A[-1].view(np.int32))
    assert np.array_equal(has, H[-1]) and np.array_equal(crc, K[-1])


@pytest.mark.gpu
def test_gpu_affine_window_upload(gpu, frames):
    """A stored window the device does not hold (here: the list's windows
    handed to a fresh tracking context mid-sequence) is uploaded from aff_img;
    the run continues exactly as the uninterrupted one."""
    from kltabi import fl_affine, fl_to_arrays, u8ptr
    setup = affine_setup(mode=2)
    h, w = frames[0].shape

    def run(switch_at):
        tc = gpu.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        setup(tc.contents)
        fl = gpu.KLTCreateFeatureList(100)
        gpu.KLTSelectGoodFeatures(tc, u8ptr(frames[1]), w, h, fl)
        img1 = frames[1]
        for i in range(1, 10):
            if i == switch_at:  # new context: no sequential pyramid, an empty window store
                gpu.KLTFreeTrackingContext(tc)
                tc = gpu.KLTCreateTrackingContext()
                tc.contents.sequentialMode = 1
                setup(tc.contents)
            gpu.KLTTrackFeatures(tc, u8ptr(np.ascontiguousarray(img1)), u8ptr(np.ascontiguousarray(frames[i])),
                                 w, h, fl)
            img1 = frames[i]
        out = fl_to_arrays(fl) + fl_affine(fl)
        gpu.KLTFreeFeatureList(fl)
        gpu.KLTFreeTrackingContext(tc)
        return out

    a, b = run(None), run(5)
    for p, q in zip(a, b):
        assert np.array_equal(np.asarray(p).view(np.uint8), np.asarray(q).view(np.uint8))
    assert a[4].sum() > 20  # windows were held throughout
