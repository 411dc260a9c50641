"""The CPU oracle (oracle/klt_oracle.c) pinned against the reference.

Golden vectors: src/V1/feat/features2.ft (committed by the reference authors)
and the reference-generated fixtures in tests/golden/ (make_golden.py).  When
oracle/_ref is present (build container) the oracle is also compared live with
the reference on fresh inputs.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest

from kltabi import (GOLDEN, KLTRunner, OracleParams, OracleTracker, fl_to_arrays, ft_bytes,
                    parse_ft, u8ptr)
import ctypes as C


def table_eq(a, b, skip_last=True):
    sl = slice(0, -1) if skip_last else slice(None)
    return all(np.array_equal(x[:, sl], y[:, sl]) for x, y in zip(a, b))


def test_v1_golden_features2(oracle, frames):
    """src/V1/example3.c: img0 first, 150 features, 10 frames (V1 feat/features2.ft)."""
    got = OracleTracker(oracle).harness(frames, 150, 10, first=frames[0])
    gold = parse_ft((GOLDEN / "v1_features2.ft").read_bytes())
    assert ft_bytes(*got) == (GOLDEN / "v1_features2.ft").read_bytes() or table_eq(got, gold)
    assert table_eq(got, gold)


@pytest.mark.parametrize("n", [100, 150])
def test_config1_golden(oracle, frames, n):
    """src/V3 `make run_cpu images_provided n 10` (BASELINE config 1)."""
    got = OracleTracker(oracle).harness(frames, n, 10)
    gold = parse_ft((GOLDEN / f"config1_{n}x10.ft").read_bytes())
    assert table_eq(got, gold)
    assert not np.any(gold[2][:, :-1] > 0)  # vals are 0 or negative status codes


def test_config1_status_histogram(oracle, frames):
    got = OracleTracker(oracle).harness(frames, 100, 10)
    vals, counts = np.unique(got[2][:, 8], return_counts=True)
    assert dict(zip(vals.tolist(), counts.tolist())) == {-5: 9, -4: 11, 0: 80}


def test_replace_golden(oracle, frames):
    got = OracleTracker(oracle).harness(frames, 150, 10, replace=True)
    gold = parse_ft((GOLDEN / "seq_config1_replace_150x10.ft").read_bytes())
    assert table_eq(got, gold)


def test_synthetic_sequences_golden(oracle, syn640, syn333):
    got = OracleTracker(oracle).harness(syn640, 1000, 12)
    assert table_eq(got, parse_ft((GOLDEN / "seq_syn640_1000x12.ft").read_bytes()))
    got = OracleTracker(oracle).harness(syn333, 300, 8)
    assert table_eq(got, parse_ft((GOLDEN / "seq_syn333x251_300x8.ft").read_bytes()))


def read_fl(path):
    data = path.read_bytes()
    assert data[:6] == b"KLTFL1"
    n = int(np.frombuffer(data[6:10], "<i4")[0])
    rec = np.frombuffer(data[10:], dtype=[("x", "<f4"), ("y", "<f4"), ("v", "<i4")])
    assert len(rec) == n
    return rec["x"], rec["y"], rec["v"]


@pytest.mark.parametrize("name,img,n", [("select_img0_150.fl", 0, 150),
                                        ("select_img5_1000.fl", 5, 1000)])
def test_selection_golden(oracle, frames, name, img, n):
    x, y, v = OracleTracker(oracle).select(frames[img], n)
    gx, gy, gv = read_fl(GOLDEN / name)
    assert np.array_equal(x, gx) and np.array_equal(y, gy) and np.array_equal(v, gv)


def test_selection_golden_synthetic(oracle, syn640):
    x, y, v = OracleTracker(oracle).select(syn640[0], 1000)
    gx, gy, gv = read_fl(GOLDEN / "select_syn640_1000.fl")
    assert np.array_equal(x, gx) and np.array_equal(y, gy) and np.array_equal(v, gv)


def test_stage_hashes(oracle, frames, syn640, syn333):
    """Every pyramid plane (img/gx/gy per level) hashes like the reference's."""
    stages = json.loads((GOLDEN / "stages.json").read_text())
    ot = OracleTracker(oracle)
    for name, img in (("img0", frames[0]), ("syn640_t0", syn640[0]), ("syn333x251_t0", syn333[0])):
        for lv, planes in enumerate(ot.frame_pyramid(img)):
            for kind, a in zip(("img", "gx", "gy"), planes):
                ref = stages[f"{name}/L{lv}/{kind}"]
                assert list(a.shape) == ref["shape"]
                assert hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() == ref["sha256"], \
                    f"{name}/L{lv}/{kind}"


def test_default_params(oracle):
    p = OracleParams()
    oracle.orc_default_params(C.byref(p))
    assert (p.borderx, p.bordery, p.nPyramidLevels, p.subsampling) == (24, 24, 2, 4)


def test_quicksort_matches_reference_symbol(oracle, ref):
    """oracle quicksort == the reference's exported _quicksort, tie-heavy data."""
    fn = ref._quicksort
    fn.restype = None
    fn.argtypes = [C.POINTER(C.c_int), C.c_int]
    rng = np.random.default_rng(7)
    for n in (0, 1, 2, 3, 10, 257, 5000):
        a = np.zeros((n, 3), np.int32)
        a[:, 0] = np.arange(n)
        a[:, 1] = rng.integers(0, 100, n)
        a[:, 2] = rng.integers(0, 7, n)
        b = a.copy()
        oracle.orc_quicksort(a.ctypes.data_as(C.POINTER(C.c_int)), n)
        fn(b.ctypes.data_as(C.POINTER(C.c_int)), n)
        assert np.array_equal(a, b)


def test_live_vs_reference_nondefault(oracle, ref, syn333):
    """Non-default parameters exercise the generic paths: window 9, ss 2, no presmoothing."""
    def setup(tc):
        tc.window_width = tc.window_height = 9
        tc.smoothBeforeSelecting = 0

    runner = KLTRunner(ref)

    def both(setup_fn, search=None):
        lib = runner.lib
        tc = lib.KLTCreateTrackingContext()
        setup_fn(tc.contents)
        if search is not None:
            lib.KLTChangeTCPyramid(tc, search)
        lib.KLTUpdateTCBorder(tc)
        p = OracleParams.from_tc(tc.contents)
        lib.KLTFreeTrackingContext(tc)

        def full_setup(t):
            setup_fn(t)
            t.nPyramidLevels, t.subsampling = p.nPyramidLevels, p.subsampling
            t.borderx, t.bordery = p.borderx, p.bordery

        r = runner.harness(syn333, 150, 6, tc_setup=full_setup)
        o = OracleTracker(oracle, p).harness(syn333, 150, 6)
        return r, o

    r, o = both(setup, search=9)
    assert table_eq(r, o)

    def li(tc):
        tc.lighting_insensitive = 1

    r, o = both(li)
    assert table_eq(r, o)


@pytest.mark.parametrize("seed", ["1081", "1087"])
def test_oracle_config5_prefix(oracle, amd, seed):
    """The oracle against the reference's config-5 fixtures (long_config5.json,
    1080p/5000, seeds 1081 .. 1087): the first three columns of two seeds --
    the CPU half of the pinning whose GPU half is
    test_gpu_long.py::test_config5_seeds_vs_reference."""
    cfg = json.loads((GOLDEN / "long_config5.json").read_text())["seeds"][seed]
    w, h, n = cfg["w"], cfg["h"], cfg["features"]
    frames = []
    for t in range(4):
        a = np.empty((h, w), np.uint8)
        amd.klt_synth_frame(int(seed), t, w, h, a.ctypes.data)
        frames.append(a)
    X, Y, V = OracleTracker(oracle).harness(frames, n, 4, first=frames[0])
    for c in range(3):
        hh = hashlib.sha256()
        for a, dt in ((X[:, c], "<f4"), (Y[:, c], "<f4"), (V[:, c], "<i4")):
            hh.update(np.ascontiguousarray(a, dt).tobytes())
        assert hh.hexdigest() == cfg["columns"][c], f"seed {seed} column {c}"
