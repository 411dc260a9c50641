"""Trackability map + selection on the GPU vs the oracle and the reference's
golden selection lists (selectGoodFeatures.c:297-495)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import synth
from gpu_helpers import Dev
from kltabi import GOLDEN, OracleParams, OracleTracker, fl_to_arrays, u8ptr
from test_oracle import read_fl

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(240, 320), (480, 640), (251, 333), (1080, 1920)])
def test_eigen_map_bit_exact(gpu, oracle, shape):
    h, w = shape
    img = synth(gpu, 31 + w, w, h, 1)[0]
    dev = Dev(gpu)
    dev.build(img, nlevels=1)
    vals, nx, ny = dev.eigen(0)
    ot = OracleTracker(oracle, OracleParams.from_tc(dev.tc.contents))
    _, gx, gy = ot.select_images(img)
    pts = ot.eigen_points(gx, gy)
    assert pts.shape[0] == nx * ny
    assert np.array_equal(vals, pts[:, 2])
    b = dev.tc.contents.borderx
    assert pts[0, 0] == b and pts[0, 1] == b and pts[nx, 1] == b + 1


@pytest.mark.parametrize("skip,window", [(1, 7), (2, 7), (0, 9), (1, 5)])
def test_eigen_map_skipped_pixels(gpu, oracle, skip, window):
    """Grid steps and windows: the tiled 7x7 kernel serves steps 1-2
    (k_min_eigen7), the per-point kernel every other case; both equal the
    oracle value for value."""
    img = synth(gpu, 3 + skip, 333, 251, 1)[0]

    def setup(t):
        t.nSkippedPixels = skip
        t.window_width = t.window_height = window

    dev = Dev(gpu, setup)
    dev.build(img, nlevels=1)
    vals, nx, ny = dev.eigen(0)
    ot = OracleTracker(oracle, OracleParams.from_tc(dev.tc.contents))
    pts = ot.eigen_points(*ot.select_images(img)[1:])
    assert np.array_equal(vals, pts[:, 2])


def select(lib, img, n, setup=None):
    h, w = img.shape
    tc = lib.KLTCreateTrackingContext()
    if setup:
        setup(tc.contents)
    fl = lib.KLTCreateFeatureList(n)
    lib.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(img)), w, h, fl)
    out = fl_to_arrays(fl)
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)
    return out


@pytest.mark.parametrize("name,img,n", [("select_img0_150.fl", 0, 150),
                                        ("select_img5_1000.fl", 5, 1000)])
def test_select_golden(gpu, frames, name, img, n):
    x, y, v = select(gpu, frames[img], n)
    gx, gy, gv = read_fl(GOLDEN / name)
    assert np.array_equal(x, gx) and np.array_equal(y, gy) and np.array_equal(v, gv)


def test_select_golden_synthetic(gpu, syn640):
    x, y, v = select(gpu, syn640[0], 1000)
    gx, gy, gv = read_fl(GOLDEN / "select_syn640_1000.fl")
    assert np.array_equal(x, gx) and np.array_equal(y, gy) and np.array_equal(v, gv)


@pytest.mark.parametrize("shape,n", [((1080, 1920), 5000), ((251, 333), 400)])
def test_select_vs_oracle(gpu, oracle, shape, n):
    h, w = shape
    img = synth(gpu, 1080, w, h, 1)[0]
    x, y, v = select(gpu, img, n)
    ox, oy, ov = OracleTracker(oracle).select(img, n)
    assert np.array_equal(x, ox) and np.array_equal(y, oy) and np.array_equal(v, ov)


def test_select_nondefault(gpu, oracle):
    img = synth(gpu, 8, 320, 240, 1)[0]

    def setup(t):
        t.mindist = 4
        t.window_width = t.window_height = 5
        t.smoothBeforeSelecting = 0
        t.min_eigenvalue = 50

    x, y, v = select(gpu, img, 700, setup)
    tc = gpu.KLTCreateTrackingContext()
    setup(tc.contents)
    ot = OracleTracker(oracle, OracleParams.from_tc(tc.contents))
    gpu.KLTFreeTrackingContext(tc)
    ox, oy, ov = ot.select(img, 700)
    assert np.array_equal(x, ox) and np.array_equal(y, oy) and np.array_equal(v, ov)
