#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Needs oracle/_ref/ (built from /root/reference by `make -C oracle ref`), so it
only runs in the build container.  Everything it writes is data: inputs and the
reference's outputs on them.

  python tests/golden/make_golden.py

Outputs
  config1_<n>x10.ft / .txt   src/V3 example3 (`make run_cpu images_provided n 10`)
  select_*.fl                 KLTSelectGoodFeatures + KLTWriteFeatureList (binary)
  seq_*.ft                    example3-style sequences on synthetic frames
  stages.json                 sha256 of every pyramid plane the reference builds
  affine_*.npz                the affine consistency check (affineConsistencyCheck
                              0/1/2): per-frame x/y/val and the features' affine
                              state (aff_x, aff_y, A, stored-window crc32);
                              warp_frames.npz holds the warped input sequence
  manifest.json               sha256 of every fixture file
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
from kltabi import (GOLDEN, REF_LIB, ROOT, KLTRunner, affine_setup, bind_klt, ft_bytes,  # noqa: E402
                    load_dataset, run_affine, u8ptr)

REF_BIN = ROOT / "oracle" / "_ref" / "example3_ref"


def synth_frames(seed: int, w: int, h: int, n: int) -> list[np.ndarray]:
    import kltamd
    lib = kltamd.load()
    out = []
    for t in range(n):
        a = np.empty((h, w), np.uint8)
        lib.klt_synth_frame(seed, t, w, h, a.ctypes.data)
        out.append(a)
    return out


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def run_example3(n_features: int, n_frames: int) -> tuple[bytes, bytes]:
    with tempfile.TemporaryDirectory() as d:
        run = Path(d) / "a" / "b"
        (run / "feat").mkdir(parents=True)
        (Path(d) / "data").mkdir()
        os.symlink(GOLDEN / "images_provided", Path(d) / "data" / "images_provided")
        subprocess.run([str(REF_BIN), "images_provided", str(n_features), str(n_frames)], cwd=run,
                       check=True, capture_output=True)
        return (run / "feat" / "features2.ft").read_bytes(), (run / "feat" / "features2.txt").read_bytes()


class RefStages:
    """Per-stage planes from the reference's own internal functions."""

    class Pyr(C.Structure):
        _fields_ = [("subsampling", C.c_int), ("nLevels", C.c_int),
                    ("img", C.POINTER(C.c_void_p)), ("ncols", C.POINTER(C.c_int)),
                    ("nrows", C.POINTER(C.c_int))]

    class FImg(C.Structure):
        _fields_ = [("ncols", C.c_int), ("nrows", C.c_int), ("data", C.POINTER(C.c_float))]

    def __init__(self):
        self.lib = lib = bind_klt(REF_LIB)
        V = C.c_void_p
        for name, res, args in [
            ("_KLTCreateFloatImage", V, [C.c_int, C.c_int]),
            ("_KLTFreeFloatImage", None, [V]),
            ("_KLTToFloatImage", None, [V, C.c_int, C.c_int, V]),
            ("_KLTComputeSmoothedImage", None, [V, C.c_float, V]),
            ("_KLTComputeGradients", None, [V, C.c_float, V, V]),
            ("_KLTCreatePyramid", C.POINTER(self.Pyr), [C.c_int, C.c_int, C.c_int, C.c_int]),
            ("_KLTComputePyramid", None, [C.POINTER(self.Pyr), V, C.c_float]),
            ("_KLTFreePyramid", None, [C.POINTER(self.Pyr)]),
        ]:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        lib._KLTComputePyramid.argtypes = [V, C.POINTER(self.Pyr), C.c_float]

    def plane(self, fimg) -> np.ndarray:
        r = C.cast(fimg, C.POINTER(self.FImg)).contents
        return np.ctypeslib.as_array(r.data, shape=(r.nrows, r.ncols)).copy()

    def pyramid(self, img: np.ndarray):
        """trackFeatures.c:1296-1307 with default parameters."""
        lib = self.lib
        tc = lib.KLTCreateTrackingContext()
        t = tc.contents
        h, w = img.shape
        tmp = lib._KLTCreateFloatImage(w, h)
        f = lib._KLTCreateFloatImage(w, h)
        lib._KLTToFloatImage(u8ptr(np.ascontiguousarray(img)), w, h, tmp)
        lib._KLTComputeSmoothedImage(tmp, lib._KLTComputeSmoothSigma(tc), f)
        p = lib._KLTCreatePyramid(w, h, t.subsampling, t.nPyramidLevels)
        lib._KLTComputePyramid(f, p, t.pyramid_sigma_fact)
        gx = lib._KLTCreatePyramid(w, h, t.subsampling, t.nPyramidLevels)
        gy = lib._KLTCreatePyramid(w, h, t.subsampling, t.nPyramidLevels)
        out = []
        for lv in range(t.nPyramidLevels):
            lib._KLTComputeGradients(p.contents.img[lv], t.grad_sigma, gx.contents.img[lv],
                                     gy.contents.img[lv])
            out.append(tuple(self.plane(q.contents.img[lv]) for q in (p, gx, gy)))
        for q in (p, gx, gy):
            lib._KLTFreePyramid(q)
        lib._KLTFreeFloatImage(tmp)
        lib._KLTFreeFloatImage(f)
        lib.KLTFreeTrackingContext(tc)
        return out


def write_select(lib, img: np.ndarray, n: int, path: Path) -> None:
    h, w = img.shape
    tc = lib.KLTCreateTrackingContext()
    fl = lib.KLTCreateFeatureList(n)
    lib.KLTSelectGoodFeatures(tc, u8ptr(np.ascontiguousarray(img)), w, h, fl)
    lib.KLTWriteFeatureList(fl, str(path).encode(), None)
    lib.KLTFreeFeatureList(fl)
    lib.KLTFreeTrackingContext(tc)


def warp_frames(seed: int = 2004, w: int = 224, h: int = 176, n: int = 8) -> list[np.ndarray]:
    """A sequence with rotation and zoom (the motion the affine check models):
    frame t samples a larger synthetic frame bilinearly (float64) at
    R(0.6 deg * t) (u, v) / (1 + 0.012 t) + (0.5 t, 0.2 t) around the centre."""
    base = synth_frames(seed, w + 96, h + 96, 1)[0].astype(np.float64)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    u, v = xx - (w - 1) / 2.0, yy - (h - 1) / 2.0
    out = []
    for t in range(n):
        th, s = np.deg2rad(0.6 * t), 1.0 + 0.012 * t
        sx = (np.cos(th) * u - np.sin(th) * v) / s + (w + 95) / 2.0 + 0.5 * t
        sy = (np.sin(th) * u + np.cos(th) * v) / s + (h + 95) / 2.0 + 0.2 * t
        x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
        ax, ay = sx - x0, sy - y0
        val = ((1 - ax) * (1 - ay) * base[y0, x0] + ax * (1 - ay) * base[y0, x0 + 1] +
               (1 - ax) * ay * base[y0 + 1, x0] + ax * ay * base[y0 + 1, x0 + 1])
        out.append(np.clip(np.floor(val + 0.5), 0, 255).astype(np.uint8))
    return out


# (fixture name, dataset, features, frames, replace, affine_setup kwargs)
AFFINE_CASES = [
    ("affine_m0_100x10", "images_provided", 100, 10, False, dict(mode=0)),
    ("affine_m1_100x10", "images_provided", 100, 10, False, dict(mode=1)),
    ("affine_m2_100x10", "images_provided", 100, 10, False, dict(mode=2)),
    ("affine_m2_replace_150x10", "images_provided", 150, 10, True, dict(mode=2)),
    ("affine_m2_w11_100x10", "images_provided", 100, 10, False, dict(mode=2, window=11, mdd=3.0, max_res=20.0)),
    ("affine_m0_li_warp_200x8", "warp", 200, 8, False, dict(mode=0, li=1)),
    ("affine_m1_warp_200x8", "warp", 200, 8, False, dict(mode=1)),
    ("affine_m2_warp_200x8", "warp", 200, 8, False, dict(mode=2, max_it=20)),
]


def affine_inputs(name: str):
    if name == "warp":
        return list(np.load(GOLDEN / "warp_frames.npz")["frames"])
    return load_dataset()


def write_affine(ref) -> None:
    np.savez_compressed(GOLDEN / "warp_frames.npz", frames=np.stack(warp_frames()))
    for name, data, n, nf, replace, kw in AFFINE_CASES:
        X, Y, V, A, H, K = run_affine(ref, affine_inputs(data), n, nf, affine_setup(**kw), replace=replace)
        np.savez_compressed(GOLDEN / f"{name}.npz", X=X, Y=Y, V=V, AFF=A, HAS=H, CRC=K)


def main() -> None:
    if not REF_LIB.exists() or not REF_BIN.exists():
        sys.exit("oracle/_ref is not built: run `make -C oracle ref` (needs /root/reference)")
    frames = load_dataset()
    ref = bind_klt(REF_LIB)
    ref.KLTSetVerbosity(0)
    runner = KLTRunner(ref)
    files: dict[str, str] = {}

    # 1. the reference harness itself (config 1 and the 150-feature default)
    for n in (100, 150):
        ft, txt = run_example3(n, 10)
        (GOLDEN / f"config1_{n}x10.ft").write_bytes(ft)
        (GOLDEN / f"config1_{n}x10.txt").write_bytes(txt)

    # 2. selection lists
    write_select(ref, frames[0], 150, GOLDEN / "select_img0_150.fl")
    write_select(ref, frames[5], 1000, GOLDEN / "select_img5_1000.fl")
    syn = synth_frames(640480, 640, 480, 12)
    write_select(ref, syn[0], 1000, GOLDEN / "select_syn640_1000.fl")

    # 3. sequences on synthetic frames (example3 semantics, frames[1] first)
    X, Y, V = runner.harness(syn, 1000, 12)
    (GOLDEN / "seq_syn640_1000x12.ft").write_bytes(ft_bytes(X, Y, V))
    odd = synth_frames(333, 333, 251, 8)
    X, Y, V = runner.harness(odd, 300, 8)
    (GOLDEN / "seq_syn333x251_300x8.ft").write_bytes(ft_bytes(X, Y, V))
    X, Y, V = runner.harness(frames, 150, 10, replace=True)
    (GOLDEN / "seq_config1_replace_150x10.ft").write_bytes(ft_bytes(X, Y, V))

    # 4. the affine consistency check
    write_affine(ref)

    # 5. per-stage planes
    st = RefStages()
    stages = {}
    for name, img in (("img0", frames[0]), ("syn640_t0", syn[0]), ("syn333x251_t0", odd[0])):
        for lv, planes in enumerate(st.pyramid(img)):
            for kind, a in zip(("img", "gx", "gy"), planes):
                stages[f"{name}/L{lv}/{kind}"] = {"shape": list(a.shape), "sha256": sha(a.tobytes())}
    (GOLDEN / "stages.json").write_text(json.dumps(stages, indent=1, sort_keys=True) + "\n")

    for p in sorted(GOLDEN.iterdir()):
        if p.is_file() and p.name != "manifest.json":
            files[p.name] = sha(p.read_bytes())
    files["frame_syn640_t0.u8"] = sha(syn[0].tobytes())
    files["frame_syn333x251_t0.u8"] = sha(odd[0].tobytes())
    (GOLDEN / "manifest.json").write_text(json.dumps(files, indent=1, sort_keys=True) + "\n")
    print(f"wrote {len(files)} fixtures to {GOLDEN}")


if __name__ == "__main__":
    main()
