"""The per-call frame upload's schedules (round 6, DESIGN §5 "Frame uploads of
the per-call API"): a KLTTrackFeatures frame from pageable memory goes
through the host pool into pinned staging and is DMAed in groups -- by
default two, the first a quarter of the frame, each queued as soon as its
pieces are copied (runtime.hip HostPool::parallel_groups).  The knobs are
read once per process, so each configuration runs in a child process; every
configuration, and the registered-buffer path (one DMA from the caller's
pages), must leave the same feature lists, at a size above the 1 MB split
threshold (1080p), one below it (640x480, one group), and one whose frame is
not a whole number of copy pieces (1000x700)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import ctypes as C, hashlib, json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import kltamd
lib = kltamd.load()
lib.KLTSetVerbosity(0)
U8P = C.POINTER(C.c_ubyte)
u8 = lambda a: a.ctypes.data_as(U8P)
out = {}
for W, H, NF in ((1920, 1080, 1500), (640, 480, 400), (1000, 700, 600)):
    fr = []
    for t in range(6):
        a = np.empty((H, W), np.uint8)
        lib.klt_synth_frame(W + H, t, W, H, a.ctypes.data)
        fr.append(a)
    def run(register):
        tc = lib.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        fl = lib.KLTCreateFeatureList(NF)
        if register:
            img1, img2 = np.empty((H, W), np.uint8), np.empty((H, W), np.uint8)
            for b in (img1, img2):
                assert lib.klt_amd_register_buffer(tc, b.ctypes.data_as(C.c_void_p), b.nbytes) == 0
            img1[:] = fr[0]
            lib.KLTSelectGoodFeatures(tc, u8(img1), W, H, fl)
            for t in range(1, len(fr)):
                img2[:] = fr[t]
                lib.KLTTrackFeatures(tc, u8(img1), u8(img2), W, H, fl)
                img1[:] = img2
        else:
            lib.KLTSelectGoodFeatures(tc, u8(fr[0]), W, H, fl)
            for t in range(1, len(fr)):
                lib.KLTTrackFeatures(tc, u8(fr[t - 1]), u8(fr[t]), W, H, fl)
        h = hashlib.sha256()
        live = 0
        for k in range(NF):
            f = fl.contents.feature[k].contents
            h.update(np.array([f.x, f.y], "<f4").tobytes() + np.array([f.val], "<i4").tobytes())
            live += f.val >= 0
        lib.KLTFreeFeatureList(fl)
        lib.KLTFreeTrackingContext(tc)
        return h.hexdigest(), int(live)
    out[f"{W}x{H}"] = {"pageable": run(False), "registered": run(True)}
print(json.dumps(out), flush=True)
"""

CONFIGS = [
    {},  # the default: pipelined, two groups, the first a quarter
    {"KLT_AMD_UPLOAD_PIPE": "0", "KLT_AMD_UPLOAD_GROUPS": "4"},  # round 5's schedule
    {"KLT_AMD_UPLOAD_GROUPS": "1"},
    {"KLT_AMD_UPLOAD_GROUPS": "3", "KLT_AMD_UPLOAD_FIRST": "0.1"},
    {"KLT_AMD_UPLOAD_GROUPS": "2", "KLT_AMD_UPLOAD_FIRST": "0", "KLT_AMD_COPY_PIECE": "4096"},
    {"KLT_AMD_HOST_THREADS": "0"},  # no pool: the caller copies alone
]


def test_upload_schedules_same_lists(tmp_path):
    script = tmp_path / "upload_child.py"
    script.write_text(CHILD)
    results = []
    for cfg in CONFIGS:
        env = {k: v for k, v in os.environ.items() if not k.startswith("KLT_AMD_")}
        env.update(cfg)
        r = subprocess.run([sys.executable, str(script), str(ROOT)], capture_output=True, text=True, timeout=180,
                           env=env)
        assert r.returncode == 0, (cfg, r.stdout[-2000:], r.stderr[-2000:])
        results.append((cfg, json.loads(r.stdout.strip().splitlines()[-1])))
    ref = results[0][1]
    for size, d in ref.items():
        assert d["pageable"] == d["registered"], (size, d)
        assert d["pageable"][1] > 0, (size, d)  # something is still tracked after five frames
    for cfg, got in results[1:]:
        assert got == ref, (cfg, got, ref)
