#!/usr/bin/env python3
"""Full-length BASELINE sequences (configs 2, 3 and 4) through the REFERENCE.

Needs oracle/_ref/libklt_ref.so (the reference compiled from /root/reference by
`make -C oracle ref`), so it only runs in the build container.  It writes data
only: the sequence parameters and, per feature-table column, a sha256 of the
reference's output -- the frames themselves are regenerated bit-identically
from the seed by include/klt_synth.h, here and on the GPU box.

Harness (src/V3/example3.c:44-76 with the synthetic sequence): select on frame
0, then for i = 1 .. frames-1: KLTTrackFeatures(frame i-1 -> frame i) in
sequential mode and KLTStoreFeatureList into column i-1.  Column c's digest is
sha256(x[c] f32 LE || y[c] f32 LE || val[c] i32 LE) over all features, so a
test may check any prefix of the sequence.

  python tests/golden/make_long.py [config2 config3 config4]

Output: tests/golden/long_<name>.json
  config2: 640x480,   1000 features,  100 frames, seed 640480  (BASELINE configs[1])
  config3: 1920x1080, 5000 features,  500 frames, seed 1080    (configs[2])
  config4: 3840x2160, 20000 features, 1000 frames, seed 2160   (configs[3]; the
           single-GPU result the sharded run must equal)
  config3r: config 3's sequence (60 frames) through the REPLACE harness:
           KLTReplaceLostFeatures after every KLTTrackFeatures
  config5: configs[4]'s other per-GPU sequences -- 1920x1080, 5000 features,
           100 frames each at seeds 1081 .. 1087 (bench.py's rank r runs seed
           1080 + r; seed 1080 is config3's) -- one entry per seed
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
from kltabi import REF_LIB, bind_klt, u8ptr  # noqa: E402

CONFIGS = {
    "config2": dict(w=640, h=480, features=1000, frames=100, seed=640480),
    "config3": dict(w=1920, h=1080, features=5000, frames=500, seed=1080),
    "config4": dict(w=3840, h=2160, features=20000, frames=1000, seed=2160),
    # the REPLACE harness (example3.c:67-69: KLTReplaceLostFeatures after every
    # KLTTrackFeatures, before KLTStoreFeatureList) at the config-3 size
    "config3r": dict(w=1920, h=1080, features=5000, frames=60, seed=1080, replace=True),
    "config5": dict(w=1920, h=1080, features=5000, frames=100, seeds=list(range(1081, 1088))),
}


def column_digest(x: np.ndarray, y: np.ndarray, v: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(x, "<f4").tobytes())
    h.update(np.ascontiguousarray(y, "<f4").tobytes())
    h.update(np.ascontiguousarray(v, "<i4").tobytes())
    return h.hexdigest()


def list_view(fl):
    """(x, y, val) views of a klt.h list whose records are one contiguous block
    (KLTCreateFeatureList allocates them so, klt.c:143-170), 64-byte stride."""
    n = fl.contents.nFeatures
    base = C.addressof(fl.contents.feature[0].contents)
    for k in (1, n - 1):
        assert C.addressof(fl.contents.feature[k].contents) == base + 64 * k, "records not contiguous"
    raw = np.ctypeslib.as_array((C.c_uint8 * (64 * n)).from_address(base)).view(np.int32).reshape(n, 16)
    return raw[:, 0].view(np.float32), raw[:, 1].view(np.float32), raw[:, 2]


def run(name: str, p: dict | None = None) -> dict:
    import kltamd
    amd = kltamd.load()  # host-side synthetic generator only (klt_synth_frame)
    p = dict(p or CONFIGS[name])
    if "seeds" in p:  # one sequence per seed, each a fixture of its own
        seeds = p.pop("seeds")
        per = {str(sd): run(f"{name} seed {sd}", dict(p, seed=sd)) for sd in seeds}
        return {"config": name, **p, "seeds": per,
                "produced_by": "oracle/_ref/libklt_ref.so (reference src/V3 compiled from its own sources)"}
    w, h, nf, nframes, seed = p["w"], p["h"], p["features"], p["frames"], p["seed"]
    ref = bind_klt(REF_LIB)
    ref.KLTSetVerbosity(0)

    def frame(t):
        a = np.empty((h, w), np.uint8)
        amd.klt_synth_frame(seed, t, w, h, a.ctypes.data)
        return a

    tc = ref.KLTCreateTrackingContext()
    tc.contents.sequentialMode = 1
    fl = ref.KLTCreateFeatureList(nf)
    img1 = frame(0)
    t0 = time.time()
    ref.KLTSelectGoodFeatures(tc, u8ptr(img1), w, h, fl)
    x, y, v = list_view(fl)
    cols = []
    live = []
    for i in range(1, nframes):
        img2 = frame(i)
        ref.KLTTrackFeatures(tc, u8ptr(img1), u8ptr(img2), w, h, fl)
        if p.get("replace"):
            ref.KLTReplaceLostFeatures(tc, u8ptr(img2), w, h, fl)
        cols.append(column_digest(x, y, v))
        live.append(int((v >= 0).sum()))
        img1 = img2
        if i % 50 == 0:
            print(f"{name}: frame {i}/{nframes - 1}, {live[-1]} live, {time.time() - t0:.0f}s", flush=True)
    final = {"x": hashlib.sha256(x.tobytes()).hexdigest(), "y": hashlib.sha256(y.tobytes()).hexdigest(),
             "val": hashlib.sha256(v.tobytes()).hexdigest()}
    ref.KLTFreeFeatureList(fl)
    ref.KLTFreeTrackingContext(tc)
    return {"config": name, **p, "select_frame": 0, "generator": "include/klt_synth.h",
            "produced_by": "oracle/_ref/libklt_ref.so (reference src/V3 compiled from its own sources)",
            "column_digest": "sha256(x f32 LE || y f32 LE || val i32 LE), column c = list after frame c+1",
            "columns": cols, "live": live, "final": final, "cpu_seconds": round(time.time() - t0, 1)}


def main() -> None:
    if not REF_LIB.exists():
        sys.exit("oracle/_ref is not built: run `make -C oracle ref` (needs /root/reference)")
    for name in sys.argv[1:] or list(CONFIGS):
        out = run(name)
        (HERE / f"long_{name}.json").write_text(json.dumps(out, indent=0) + "\n")
        print(f"wrote long_{name}.json")


if __name__ == "__main__":
    main()
