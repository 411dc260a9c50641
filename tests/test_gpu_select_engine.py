"""The device half of selection (csrc/select.hip): the reference's quicksort
order (selectGoodFeatures.c:62-96) produced lazily with its top-level
partition steps split on the device by the parallel form of the same step.
Pinned against klt_sort_pairs_full (the host restatement, itself pinned to
the oracle's quicksort in test_abi / test_select_host) on tie-heavy, sorted,
constant and random inputs, with the device/host threshold forced small so
that many device steps run; then the selection walk itself against the
oracle's selection and REPLACE harness at sizes where device steps happen."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import synth
from kltabi import KLTRunner, OracleTracker

pytestmark = pytest.mark.gpu


def host_order(gpu, vals):
    v = np.ascontiguousarray(vals, np.int32).copy()
    i = np.arange(len(v), dtype=np.int32)
    gpu.klt_sort_pairs_full(v.ctypes.data_as(C.POINTER(C.c_int)), i.ctypes.data_as(C.POINTER(C.c_int)), len(v))
    return v, i


def device_order(gpu, ctx, vals, threshold):
    from kltamd.device import check
    v = np.ascontiguousarray(vals, np.int32)
    ov = np.empty(len(v), np.int32)
    oi = np.empty(len(v), np.int32)
    check(gpu, ctx, gpu.klt_hip_select_tune(ctx, threshold), "tune")
    check(gpu, ctx, gpu.klt_hip_select_sort_test(ctx, v.ctypes.data, len(v), ov.ctypes.data, oi.ctypes.data), "sort")
    d, s, vis = C.c_long(), C.c_long(), C.c_long()
    check(gpu, ctx, gpu.klt_hip_select_stats(ctx, C.byref(d), C.byref(s), C.byref(vis), None), "stats")
    return ov, oi, s.value


CASES = {
    "ties3": lambda rng, n: rng.integers(0, 3, n),
    "ties50": lambda rng, n: rng.integers(0, 50, n),
    "random": lambda rng, n: rng.integers(-2**31, 2**31 - 1, n),
    "constant": lambda rng, n: np.full(n, 7),
    "ascending": lambda rng, n: np.arange(n),
    "descending": lambda rng, n: np.arange(n)[::-1].copy(),
    "eigen_like": lambda rng, n: np.maximum(0, (rng.exponential(2000, n) - 500)).astype(np.int64),
}


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("n,threshold", [(1, 1), (2, 1), (7, 2), (1000, 64), (100_000, 1000), (300_001, 20_000)])
def test_device_order_equals_host(gpu, case, n, threshold):
    rng = np.random.default_rng(n * 7 + len(case))
    vals = CASES[case](rng, n).astype(np.int32)
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    try:
        hv, hi = host_order(gpu, vals)
        dv, di, steps = device_order(gpu, ctx, vals, threshold)
        assert np.array_equal(hv, dv) and np.array_equal(hi, di), f"{case} n={n}: order differs"
        if n > threshold:
            assert steps > 0
    finally:
        gpu.klt_hip_select_tune(ctx, 32768)
        gpu.KLTFreeTrackingContext(tc)


@pytest.mark.parametrize("threshold", [64, 4096, 32768])
def test_selection_with_device_steps_vs_oracle(gpu, oracle, threshold):
    """KLTSelectGoodFeatures and the REPLACE harness through klt_hip_select, with
    the device/host split at several thresholds, against the oracle."""
    frames = synth(gpu, 777, 640, 480, 8)

    def setup(t):
        ctx = gpu.klt_amd_device_context(C.pointer(t))
        assert gpu.klt_hip_select_tune(ctx, threshold) == 0

    X, Y, V = KLTRunner(gpu).harness(frames, 1000, 8, first=frames[0], replace=True, tc_setup=setup)
    OX, OY, OV = OracleTracker(oracle).harness(frames, 1000, 8, first=frames[0], replace=True)
    T = 7
    assert np.array_equal(V[:, :T], OV[:, :T])
    assert np.array_equal(X[:, :T].view(np.int32), OX[:, :T].view(np.int32))
    assert np.array_equal(Y[:, :T].view(np.int32), OY[:, :T].view(np.int32))


EXIT_CHILD = r"""
import ctypes as C, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import kltamd
lib = kltamd.load()
lib.KLTSetVerbosity(0)
W, H, NF = 1280, 720, 3000
u8 = lambda a: a.ctypes.data_as(C.POINTER(C.c_ubyte))
fr = []
for t in range(5):
    a = np.empty((H, W), np.uint8)
    lib.klt_synth_frame(720, t, W, H, a.ctypes.data)
    fr.append(a)
parked = lib.KLTCreateTrackingContext()  # freed below: its device context is parked, graphs and all
tc = lib.KLTCreateTrackingContext()      # never freed: live at exit
for c in (parked, tc):
    c.contents.sequentialMode = 1
fl = lib.KLTCreateFeatureList(NF)
for c in (parked, tc):
    lib.KLTSelectGoodFeatures(c, u8(fr[0]), W, H, fl)
    for t in range(1, 5):
        lib.KLTTrackFeatures(c, u8(fr[t - 1]), u8(fr[t]), W, H, fl)
        lib.KLTReplaceLostFeatures(c, u8(fr[t]), W, H, fl)
lib.KLTFreeTrackingContext(parked)
print("child done", flush=True)
"""


def test_exit_after_replace_is_clean(tmp_path):
    """The process exits cleanly after REPLACE calls whose partition steps were
    graph launches, with one tracking context freed (its device context
    parked) and one never freed: the library's exit hook (runtime.hip
    exit_hook) drains the device, releases the instantiated graphs and joins
    the host sort pool before the code object's own exit-time
    unregistration.  A crash inside exit() after such a run was seen once
    under rocprofv3 in round 4."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    script = tmp_path / "exit_child.py"
    script.write_text(EXIT_CHILD)
    r = subprocess.run([sys.executable, str(script), str(root)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "child done" in r.stdout
