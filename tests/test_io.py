"""Host-side parts of libklt_amd.so on the CPU (no GPU needed): feature
list/history/table persistence (writeFeatures.c), PGM/PPM I/O (pnmio.c),
store/extract (storeFeatures.c), the lazy exact quicksort behind selection
(selectGoodFeatures.c:45-96), and the synthetic frame generator.

Byte-level expectations come from the reference's own outputs committed under
tests/golden/ (config1_*x10.ft/.txt were written by the reference harness),
and -- where oracle/_ref is built -- from the reference library writing the
same data side by side.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json

import numpy as np
import pytest

from kltabi import GOLDEN, fl_to_arrays, parse_ft, u8ptr
from test_oracle import table_eq


def _table_from_ft(lib, path):
    ft = lib.KLTReadFeatureTable(None, str(path).encode())
    assert ft
    return ft


def _table_arrays(ft):
    t = ft.contents
    X = np.empty((t.nFeatures, t.nFrames), np.float32)
    Y = np.empty_like(X)
    V = np.empty((t.nFeatures, t.nFrames), np.int32)
    for j in range(t.nFeatures):
        for i in range(t.nFrames):
            f = t.feature[j][i].contents
            X[j, i], Y[j, i], V[j, i] = f.x, f.y, f.val
    return X, Y, V


@pytest.mark.parametrize("n", [100, 150])
def test_table_read_write_reproduces_reference_files(amd, tmp_path, n):
    """Read the reference's binary .ft, write it back binary and as text:
    both byte-identical to what the reference wrote (KLTWriteFeatureTable)."""
    src = GOLDEN / f"config1_{n}x10.ft"
    ft = _table_from_ft(amd, src)
    amd.KLTWriteFeatureTable(ft, str(tmp_path / "t.ft").encode(), None)
    amd.KLTWriteFeatureTable(ft, str(tmp_path / "t.txt").encode(), b"%5.1f")
    assert (tmp_path / "t.ft").read_bytes() == src.read_bytes()
    assert (tmp_path / "t.txt").read_bytes() == (GOLDEN / f"config1_{n}x10.txt").read_bytes()
    assert table_eq(_table_arrays(ft), parse_ft(src.read_bytes()), skip_last=False)
    amd.KLTFreeFeatureTable(ft)


def test_text_table_reads_back(amd, tmp_path):
    src = GOLDEN / "config1_100x10.txt"
    ft = amd.KLTReadFeatureTable(None, str(src).encode())
    X, Y, V = _table_arrays(ft)
    want = parse_ft((GOLDEN / "config1_100x10.ft").read_bytes())
    assert np.array_equal(V, want[2])
    # the text holds one decimal: equal to the binary values rounded the same way
    assert np.allclose(X, want[0], atol=0.051) and np.allclose(Y, want[1], atol=0.051)
    amd.KLTFreeFeatureTable(ft)


@pytest.mark.parametrize("name", ["select_img0_150.fl", "select_img5_1000.fl", "select_syn640_1000.fl"])
def test_list_binary_roundtrip(amd, tmp_path, name):
    src = GOLDEN / name
    fl = amd.KLTReadFeatureList(None, str(src).encode())
    assert fl
    amd.KLTWriteFeatureList(fl, str(tmp_path / "l.fl").encode(), None)
    assert (tmp_path / "l.fl").read_bytes() == src.read_bytes()
    amd.KLTFreeFeatureList(fl)


def _both(amd, ref):
    return [("amd", amd)] + ([("ref", ref)] if ref is not None else [])


@pytest.fixture
def ref_or_none():
    import kltabi
    if not kltabi.REF_LIB.exists():
        return None
    return kltabi.bind_klt(kltabi.REF_LIB)


def _fill_list(lib, x, y, v):
    fl = lib.KLTCreateFeatureList(len(x))
    for k in range(len(x)):
        f = fl.contents.feature[k].contents
        f.x, f.y, f.val = float(x[k]), float(y[k]), int(v[k])
    return fl


def _sample_features(n=37, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 640, n).astype(np.float32)
    y = rng.uniform(0, 480, n).astype(np.float32)
    v = rng.integers(-5, 2000, n).astype(np.int32)
    x[v < 0] = -1.0
    y[v < 0] = -1.0
    return x, y, v


@pytest.mark.parametrize("fmt", [None, b"%5.1f", b"%7.3f"])
def test_list_and_history_writes_match_reference(amd, ref_or_none, tmp_path, fmt):
    if ref_or_none is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    x, y, v = _sample_features()
    outs = {}
    for tag, lib in _both(amd, ref_or_none):
        fl = _fill_list(lib, x, y, v)
        lib.KLTWriteFeatureList(fl, str(tmp_path / f"{tag}.fl").encode(), fmt)
        ft = lib.KLTCreateFeatureTable(4, len(x))
        for i in range(4):
            lib.KLTStoreFeatureList(fl, ft, i)
        fh = lib.KLTCreateFeatureHistory(4)
        lib.KLTExtractFeatureHistory(fh, ft, 5)
        lib.KLTWriteFeatureHistory(fh, str(tmp_path / f"{tag}.fh").encode(), fmt)
        lib.KLTWriteFeatureTable(ft, str(tmp_path / f"{tag}.ft").encode(), fmt)
        outs[tag] = [(tmp_path / f"{tag}.{e}").read_bytes() for e in ("fl", "fh", "ft")]
        lib.KLTFreeFeatureHistory(fh)
        lib.KLTFreeFeatureTable(ft)
        lib.KLTFreeFeatureList(fl)
    assert outs["amd"] == outs["ref"]


def test_store_extract_and_count(amd):
    x, y, v = _sample_features(20, 9)
    fl = _fill_list(amd, x, y, v)
    assert amd.KLTCountRemainingFeatures(fl) == int((v >= 0).sum())
    ft = amd.KLTCreateFeatureTable(3, 20)
    amd.KLTStoreFeatureList(fl, ft, 2)
    fl2 = amd.KLTCreateFeatureList(20)
    amd.KLTExtractFeatureList(fl2, ft, 2)
    gx, gy, gv = fl_to_arrays(fl2)
    assert np.array_equal(gx, x) and np.array_equal(gy, y) and np.array_equal(gv, v)
    fh = amd.KLTCreateFeatureHistory(3)
    amd.KLTExtractFeatureHistory(fh, ft, 4)
    assert fh.contents.feature[2].contents.val == v[4]
    for p in (fh,):
        amd.KLTFreeFeatureHistory(p)
    amd.KLTFreeFeatureTable(ft)
    amd.KLTFreeFeatureList(fl)
    amd.KLTFreeFeatureList(fl2)


def test_pgm_roundtrip_and_bytes(amd, ref_or_none, tmp_path):
    img = np.random.default_rng(1).integers(0, 256, (37, 53)).astype(np.uint8)
    for tag, lib in _both(amd, ref_or_none):
        lib.pgmWriteFile(str(tmp_path / f"{tag}.pgm").encode(), u8ptr(img), 53, 37)
    data = (tmp_path / "amd.pgm").read_bytes()
    if ref_or_none is not None:
        assert data == (tmp_path / "ref.pgm").read_bytes()
    w, h = C.c_int(0), C.c_int(0)
    out = np.zeros_like(img)
    amd.pgmReadFile(str(tmp_path / "amd.pgm").encode(), u8ptr(out), C.byref(w), C.byref(h))
    assert (w.value, h.value) == (53, 37) and np.array_equal(out, img)


def test_ppm_overlay_matches_reference(amd, ref_or_none, tmp_path, frames):
    if ref_or_none is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    fl_src = GOLDEN / "select_img0_150.fl"
    img = np.ascontiguousarray(frames[0])
    h, w = img.shape
    for tag, lib in _both(amd, ref_or_none):
        fl = lib.KLTReadFeatureList(None, str(fl_src).encode())
        lib.KLTWriteFeatureListToPPM(fl, u8ptr(img), w, h, str(tmp_path / f"{tag}.ppm").encode())
        lib.KLTFreeFeatureList(fl)
    assert (tmp_path / "amd.ppm").read_bytes() == (tmp_path / "ref.ppm").read_bytes()


def test_lazy_quicksort_is_the_reference_permutation(amd, oracle):
    """klt_select.c's partition-on-demand sort, run to completion, yields the
    same order as the oracle's restatement of _quicksort (pinned against the
    reference symbol in test_oracle.py) -- ties included."""
    rng = np.random.default_rng(11)
    for n in (0, 1, 2, 3, 17, 256, 4097):
        for hi in (3, 1000, 2**31 - 1):
            val = rng.integers(0, hi, n).astype(np.int32)
            idx = np.arange(n, dtype=np.int32)
            a = np.zeros((n, 3), np.int32)
            a[:, 0], a[:, 2] = idx, val
            oracle.orc_quicksort(a.ctypes.data_as(C.POINTER(C.c_int)), n)
            v2, i2 = val.copy(), idx.copy()
            amd.klt_sort_pairs_full(v2.ctypes.data_as(C.POINTER(C.c_int)), i2.ctypes.data_as(C.POINTER(C.c_int)),
                                    n)
            assert np.array_equal(i2, a[:, 0]) and np.array_equal(v2, a[:, 2])


def test_synthetic_generator_is_pinned(amd):
    """include/klt_synth.h on the host reproduces the committed fixture hash."""
    man = json.loads((GOLDEN / "manifest.json").read_text())
    for key, (seed, w, h) in {"frame_syn640_t0.u8": (640480, 640, 480),
                              "frame_syn333x251_t0.u8": (333, 333, 251)}.items():
        a = np.empty((h, w), np.uint8)
        amd.klt_synth_frame(seed, 0, w, h, a.ctypes.data)
        assert hashlib.sha256(a.tobytes()).hexdigest() == man[key]
