"""Degenerate and boundary inputs of the hot path: empty feature lists,
images smaller than the tracking border, flat images (zero trackability,
singular 2x2 systems), every lost-feature status code, all-lost lists, and
sizes on the edge of the fused kernels' tiles.

CPU tests pin the oracle on these inputs against the reference compiled here
(oracle/_ref, skipped without it); GPU tests hold libklt_amd to the oracle,
bit for bit (positions, status codes), the never-written last table column
excepted (example3.c:71).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import synth
from kltabi import KLTRunner, OracleParams, OracleTracker
from test_oracle import table_eq

# name -> (frames builder(amd), n_features, n_frames, tc setup)
def _flat(amd):
    return [np.full((120, 160), 128, np.uint8) for _ in range(4)]


def _tiny(amd):
    return synth(amd, 7, 40, 30, 4)          # smaller than 2 x border (24)


def _strip(amd):
    return synth(amd, 9, 300, 49, 5)         # one border-wide row band


def _edge_tiles(amd):
    return synth(amd, 11, 65, 33, 5)         # one pixel past a 64x32 tile


def _noisy(amd):
    rng = np.random.default_rng(5)           # uncorrelated frames: residues and losses
    return [rng.integers(0, 256, (96, 128), dtype=np.uint8) for _ in range(4)]


def _default(amd):
    return synth(amd, 333, 333, 251, 6)


def _set(**kw):
    def f(t):
        for k, v in kw.items():
            setattr(t, k, v)
    return f


EDGE = {
    "empty_list": (_default, 0, 4, _set()),
    "one_feature": (_default, 1, 6, _set()),
    "flat_images": (_flat, 50, 4, _set()),
    "smaller_than_border": (_tiny, 20, 4, _set()),
    "border_strip": (_strip, 40, 5, _set()),
    "tile_edge_sizes": (_edge_tiles, 30, 5, _set()),
    "uncorrelated_frames": (_noisy, 60, 4, _set()),
    "small_det": (_default, 100, 4, _set(min_determinant=1e9)),
    "max_iterations": (_default, 100, 4, _set(max_iterations=1, min_displacement=1e-6)),
    "large_residue": (_default, 100, 4, _set(max_residue=0.05)),
    "more_features_than_found": (_tiny, 500, 4, _set(mindist=2, window_width=3, window_height=3)),
    "zero_mindist": (_default, 300, 4, _set(mindist=0)),
    "min_eigenvalue_high": (_default, 200, 4, _set(min_eigenvalue=1 << 20)),
}


def _run(lib_runner, frames, n, nf, setup):
    return lib_runner.harness(frames, n, nf, tc_setup=setup)


def _oracle_run(oracle, amd, frames, n, nf, setup):
    tc = amd.KLTCreateTrackingContext()
    setup(tc.contents)
    p = OracleParams.from_tc(tc.contents)
    amd.KLTFreeTrackingContext(tc)
    return OracleTracker(oracle, p).harness(frames, n, nf)


@pytest.mark.parametrize("name", list(EDGE))
def test_oracle_edge_vs_reference(oracle, ref, amd, name):
    build, n, nf, setup = EDGE[name]
    frames = build(amd)
    want = _run(KLTRunner(ref), frames, n, nf, setup)
    got = _oracle_run(oracle, amd, frames, n, nf, setup)
    assert table_eq(got, want), name


def test_edge_cases_reach_every_status(oracle, amd):
    """Across the cases every status code of klt.h:28-33 occurs."""
    seen = set()
    for name, (build, n, nf, setup) in EDGE.items():
        if n == 0:
            continue
        X, Y, V = _oracle_run(oracle, amd, build(amd), n, nf, setup)
        seen |= set(np.unique(V[:, :-1]).tolist())
    assert {0, -1, -2, -3, -4, -5} <= seen, seen


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(EDGE))
def test_gpu_edge_vs_oracle(gpu, oracle, name):
    build, n, nf, setup = EDGE[name]
    frames = build(gpu)
    got = _run(KLTRunner(gpu), frames, n, nf, setup)
    want = _oracle_run(oracle, gpu, frames, n, nf, setup)
    assert table_eq(got, want), name


@pytest.mark.gpu
def test_gpu_all_lost_list_is_untouched(gpu):
    """Features with val < 0 are not tracked and keep their fields
    (trackFeatures.c:1346), including on the batched device path."""
    from kltabi import arrays_to_fl, fl_to_arrays, u8ptr
    frames = synth(gpu, 21, 160, 120, 3)
    h, w = frames[0].shape
    tc = gpu.KLTCreateTrackingContext()
    fl = gpu.KLTCreateFeatureList(10)
    x = np.arange(10, dtype=np.float32) * 7.25
    y = np.arange(10, dtype=np.float32) * 3.5
    v = -np.arange(1, 11, dtype=np.int32)
    arrays_to_fl(fl, x, y, v)
    gpu.KLTTrackFeatures(tc, u8ptr(frames[0]), u8ptr(frames[1]), w, h, fl)
    gx, gy, gv = fl_to_arrays(fl)
    gpu.KLTFreeFeatureList(fl)
    gpu.KLTFreeTrackingContext(tc)
    assert np.array_equal(gx, x) and np.array_equal(gy, y) and np.array_equal(gv, v)


@pytest.mark.gpu
def test_gpu_8k_frame_pyramid_and_tracking(gpu, oracle):
    """The largest size class: a 7680x4320 pair (33 Mpx, 132 MB per f32
    plane) -- the fused pyramid bit-identical to the oracle, and 2000
    features tracked over it bit-identically."""
    from gpu_helpers import Dev
    from test_gpu_pyramid import assert_planes_equal, oracle_for
    h, w = 4320, 7680
    frames = synth(gpu, 4320, w, h, 3)
    dev = Dev(gpu)
    dev.build(frames[0])
    assert dev.path(0) == 1
    assert_planes_equal(dev.levels(0, 2), oracle_for(oracle, dev.tc).frame_pyramid(frames[0]), "8k")
    got = KLTRunner(gpu).harness(frames, 2000, 3)
    want = OracleTracker(oracle).harness(frames, 2000, 3)
    assert table_eq(got, want)
    assert (got[2][:, 1] == 0).sum() > 1500
