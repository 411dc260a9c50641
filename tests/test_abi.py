"""The drop-in boundary: struct layouts, exported symbols, parameter logic.

Runs without a GPU (loading libklt_amd.so needs no device)."""
from __future__ import annotations

import ctypes as C
import re
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

from kltabi import ROOT, TrackingContextRec, OracleParams

INCLUDE = ROOT / "include"

PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "klt.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(KLT_TrackingContextRec),
         offsetof(KLT_TrackingContextRec, pyramid_last), offsetof(KLT_TrackingContextRec, subsampling),
         sizeof(KLT_FeatureRec), offsetof(KLT_FeatureRec, aff_img), offsetof(KLT_FeatureRec, aff_x),
         sizeof(KLT_FeatureListRec), sizeof(KLT_FeatureHistoryRec), sizeof(KLT_FeatureTableRec));
  return 0;
}
"""


def probe_layout(include_dir: Path) -> list[int]:
    with tempfile.TemporaryDirectory() as d:
        src = Path(d) / "probe.c"
        src.write_text(PROBE)
        exe = Path(d) / "probe"
        subprocess.run(["gcc", f"-I{include_dir}", str(src), "-o", str(exe)], check=True)
        return [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                               check=True).stdout.split()]


def test_klt_h_layout():
    """include/klt.h compiles to the reference's x86-64 layout."""
    assert probe_layout(INCLUDE) == [136, 112, 80, 64, 16, 40, 16, 16, 16]


def test_klt_h_layout_equals_reference_header():
    ref_inc = Path("/root/reference/src/V3")
    if not ref_inc.exists():
        pytest.skip("reference headers not present")
    assert probe_layout(INCLUDE) == probe_layout(ref_inc)


def declared_functions() -> dict[str, list[str]]:
    out = {}
    for h in sorted(INCLUDE.glob("*.h")):
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"#[^\n]*", "", text)
        text = re.sub(r"typedef[^;]*;", "", text, flags=re.S)
        names = re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", text)
        # drop things that are not prototypes (macros removed above, typedef'd structs gone)
        names = [n for n in names if n not in {"if", "while", "for", "return", "sizeof"}]
        # header-only inline helpers (klt_synth.h) are not library symbols
        inline = set(re.findall(r"KLT_SYNTH_FN\s+\w+\s+(\w+)\s*\(", h.read_text()))
        out[h.name] = sorted(set(names) - inline)
    return out


def test_every_declared_symbol_is_exported(amd):
    decl = declared_functions()
    assert "KLTTrackFeatures" in decl["klt.h"] and "klt_hip_track" in decl["klt_hip.h"]
    missing = [(h, n) for h, names in decl.items() for n in names if not hasattr(amd, n)]
    assert not missing, missing
    assert C.c_int.in_dll(amd, "KLT_verbose") is not None


def test_reference_surface_is_exported(amd, ref):
    """Every KLT*/pnm/_KLT public function the reference library defines."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(ROOT / "oracle/_ref/libklt_ref.so")],
                         capture_output=True, text=True, check=True).stdout
    names = {l.split()[-1] for l in out.splitlines() if " T " in l}
    public = {n for n in names if n.startswith(("KLT", "pgm", "ppm", "pnm"))}
    public |= {"_KLTComputeSmoothSigma", "_KLTCreateFloatImage", "_KLTFreeFloatImage",
               "_KLTWriteFloatImageToPGM"}
    missing = sorted(n for n in public if not hasattr(amd, n))
    assert not missing, missing


def tc_fields(lib, tc):
    t = tc.contents
    return {n: getattr(t, n) for n, _ in TrackingContextRec._fields_ if not n.startswith("pyramid_last")}


def test_defaults_match_reference(amd, ref):
    a, r = amd.KLTCreateTrackingContext(), ref.KLTCreateTrackingContext()
    assert tc_fields(amd, a) == tc_fields(ref, r)
    assert tc_fields(amd, a)["borderx"] == 24
    assert not a.contents.pyramid_last
    amd.KLTFreeTrackingContext(a)
    ref.KLTFreeTrackingContext(r)


@pytest.mark.parametrize("win", [3, 4, 5, 7, 8, 9, 11, 15, 21])
@pytest.mark.parametrize("search", [1, 4, 6, 10, 15, 30, 60, 200])
def test_pyramid_and_border_derivation(amd, oracle, win, search):
    """KLTChangeTCPyramid / KLTUpdateTCBorder (klt.c:288-431) vs the oracle."""
    tc = amd.KLTCreateTrackingContext()
    tc.contents.window_width = tc.contents.window_height = win
    amd.KLTSetVerbosity(0)
    amd.KLTChangeTCPyramid(tc, search)
    amd.KLTUpdateTCBorder(tc)
    p = OracleParams()
    oracle.orc_default_params(C.byref(p))
    p.window_width = p.window_height = win
    oracle.orc_change_pyramid(C.byref(p), search)
    oracle.orc_update_border(C.byref(p))
    t = tc.contents
    assert (t.nPyramidLevels, t.subsampling, t.borderx, t.bordery, t.window_width) == \
           (p.nPyramidLevels, p.subsampling, p.borderx, p.bordery, p.window_width)
    amd.KLTFreeTrackingContext(tc)


def test_smooth_sigma(amd):
    tc = amd.KLTCreateTrackingContext()
    assert amd._KLTComputeSmoothSigma(tc) == np.float32(np.float32(0.1) * np.float32(7))
    amd.KLTFreeTrackingContext(tc)


def test_no_gpu_path_fails_loudly():
    """Without a device the tracker must exit via KLTError, not fall back to a CPU path."""
    code = ("import sys; sys.path.insert(0, %r); import kltamd, numpy as np; lib = kltamd.load();"
            "lib.KLTSetVerbosity(0);"
            "n = lib.klt_hip_device_count();"
            "sys.exit(3) if n > 0 else None;"
            "tc = lib.KLTCreateTrackingContext(); fl = lib.KLTCreateFeatureList(5);"
            "a = np.zeros((64, 64), np.uint8);"
            "lib.KLTSelectGoodFeatures(tc, a.ctypes.data_as(kltamd.abi.U8P), 64, 64, fl)") % str(ROOT)
    import os
    import sys
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env)
    if r.returncode == 3:
        pytest.skip("a GPU is visible")
    assert r.returncode == 1 and "KLT Error" in r.stderr, (r.returncode, r.stderr[-500:])


@pytest.mark.parametrize("workers", [0, 1, 3, 4, 8])
def test_copy_pool_selftest(amd, workers):
    """Host-only: the copy pool behind KLTTrackSequence's pinned staging copies
    every byte of many back-to-back groups (random sizes and piece lengths),
    with the job list refilled between groups while the workers are parked."""
    assert amd.klt_hip_selftest_copy_pool(workers, 400, 1 << 20) == 0
    assert amd.klt_hip_selftest_copy_pool(workers, 2000, 4096) == 0
