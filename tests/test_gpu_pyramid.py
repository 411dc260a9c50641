"""Pyramid kernels (fused gfx950 path and generic path) vs the CPU oracle,
bit for bit, per plane (_KLTComputeSmoothedImage + _KLTComputePyramid +
_KLTComputeGradients, trackFeatures.c:1296-1307)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import synth
from gpu_helpers import Dev, bits
from kltamd.device import check
from kltabi import OracleParams, OracleTracker

pytestmark = pytest.mark.gpu

SHAPES = [(240, 320), (480, 640), (251, 333), (67, 129), (31, 40), (1080, 1920), (113, 517)]


def oracle_for(oracle, tc):
    return OracleTracker(oracle, OracleParams.from_tc(tc.contents))


def assert_planes_equal(got, want, tag):
    assert len(got) == len(want)
    for lv, (g, w) in enumerate(zip(got, want)):
        for kind, a, b in zip(("img", "gx", "gy"), g, w):
            assert a.shape == b.shape, (tag, lv, kind)
            bad = np.flatnonzero(bits(a) != bits(b))
            assert bad.size == 0, f"{tag} L{lv} {kind}: {bad.size} mismatches, first at {np.unravel_index(bad[0], a.shape)}"


@pytest.mark.parametrize("shape", SHAPES)
def test_fused_pyramid_bit_exact(gpu, oracle, shape):
    h, w = shape
    img = synth(gpu, 1000 + h, w, h, 1)[0]
    dev = Dev(gpu)
    dev.build(img)
    assert dev.path(0) == 1, "default parameters must take the fused gfx950 kernels"
    got = dev.levels(0, 2)
    want = oracle_for(oracle, dev.tc).frame_pyramid(img)
    assert_planes_equal(got, want, f"fused {shape}")


def test_fused_pyramid_real_frames(gpu, oracle, frames):
    dev = Dev(gpu)
    ot = oracle_for(oracle, dev.tc)
    for img in frames[:4]:
        dev.build(img)
        assert_planes_equal(dev.levels(0, 2), ot.frame_pyramid(img), "images_provided")


# (2001, 2100), (2003, 2050), (2160, 3840): whole frames of >= 2000 rows run
# the 64-row level-0 tiles (pyramid.hip kL0WideMinRows), with a partial last
# tile row, a partial last tile column and (2050) no 4-byte row alignment
STRIP_SHAPES = [(480, 640), (1080, 1920), (67, 136), (31, 40), (9, 64), (200, 72), (2160, 3840), (2001, 2100),
                (2003, 2050)]


@pytest.mark.parametrize("shape", STRIP_SHAPES)
def test_fused_pyramid_shapes_vs_oracle(gpu, oracle, shape):
    """k_pyr_l0 + k_pyr_l1 at odd, tiny, tall and 4K shapes == oracle, bit for bit."""
    h, w = shape
    img = synth(gpu, 4242 + w, w, h, 1)[0]
    dev = Dev(gpu)
    dev.build(img)
    assert_planes_equal(dev.levels(0, 2), oracle_for(oracle, dev.tc).frame_pyramid(img), f"tiles {shape}")


@pytest.mark.parametrize("shape", [(240, 320), (251, 333), (67, 129)])
def test_generic_equals_fused(gpu, shape):
    h, w = shape
    img = synth(gpu, 77, w, h, 1)[0]
    dev = Dev(gpu)
    dev.build(img, slot=0)
    dev.build(img, slot=1, force_generic=True)
    assert dev.path(0) == 1 and dev.path(1) == 0
    assert_planes_equal(dev.levels(1, 2), dev.levels(0, 2), f"generic {shape}")


def setups():
    def win9(t):
        t.window_width = t.window_height = 9

    def ss2(t):
        t.window_width = t.window_height = 9

    def grad15(t):
        t.grad_sigma = 1.5

    def pyr_sf(t):
        t.pyramid_sigma_fact = 0.7

    return [("win9", win9, None), ("ss2", ss2, 9), ("ss8", None, 30), ("levels3", None, 200),
            ("grad1.5", grad15, None), ("pyr0.7", pyr_sf, None)]


@pytest.mark.parametrize("name,fn,search", setups(), ids=[s[0] for s in setups()])
def test_generic_nondefault_bit_exact(gpu, oracle, name, fn, search):
    img = synth(gpu, 9, 320, 240, 1)[0]

    def setup(t):
        if fn:
            fn(t)

    dev = Dev(gpu, setup)
    if search is not None:
        gpu.KLTChangeTCPyramid(dev.tc, search)
    gpu.KLTUpdateTCBorder(dev.tc)
    n = dev.tc.contents.nPyramidLevels
    dev.build(img)
    want = oracle_for(oracle, dev.tc).frame_pyramid(img)
    assert_planes_equal(dev.levels(0, n), want, name)


def test_selection_images_no_presmoothing(gpu, oracle):
    img = synth(gpu, 5, 200, 150, 1)[0]

    def setup(t):
        t.smoothBeforeSelecting = 0

    dev = Dev(gpu, setup)
    dev.build(img, nlevels=1, smooth=0)
    a, gx, gy = oracle_for(oracle, dev.tc).select_images(img)
    assert_planes_equal(dev.levels(0, 1), [(a, gx, gy)], "no-presmooth")


def test_level_layout_api(gpu):
    """klt_hip_level_interleaved / klt_hip_level_ptr: fused levels are one
    {gx, gy, img} record per pixel at the base (gx/gy queries return NULL),
    generic levels are three planes; both de-interleave to the same planes."""
    import ctypes as C
    h, w = 67, 129
    img = synth(gpu, 31, w, h, 1)[0]
    dev = Dev(gpu)
    dev.build(img, slot=0)
    dev.build(img, slot=1, force_generic=True)
    lib, ctx = gpu, dev.ctx
    want = dev.levels(1, 2)
    for lv in range(2):
        assert lib.klt_hip_level_interleaved(ctx, 0, lv) == 1
        assert lib.klt_hip_level_interleaved(ctx, 1, lv) == 0
        base = lib.klt_hip_level_ptr(ctx, 0, lv, 0)
        assert base and not lib.klt_hip_level_ptr(ctx, 0, lv, 1) and not lib.klt_hip_level_ptr(ctx, 0, lv, 2)
        assert all(lib.klt_hip_level_ptr(ctx, 1, lv, k) for k in range(3))
        lw, lh = want[lv][0].shape[1], want[lv][0].shape[0]
        rec = np.empty((lh, lw, 3), np.float32)
        check(lib, ctx, lib.klt_hip_sync(ctx), "sync")
        check(lib, ctx, lib.klt_hip_memcpy(ctx, rec.ctypes.data, C.c_void_p(base), rec.nbytes, 2), "d2h")
        for k, plane in enumerate((1, 2, 0)):  # record {gx, gy, img} (klt_dev.h kRec*)
            assert np.array_equal(bits(rec[:, :, k]), bits(want[lv][plane])), (lv, k)
    assert lib.klt_hip_level_interleaved(ctx, 0, 5) == -1
