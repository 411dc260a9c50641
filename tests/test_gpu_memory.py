"""Device memory bounds of the batched path:
the bank budget (klt_hip_set_bank_budget) caps the chunk of a plain
klt_hip_track_frames call -- with results identical to the uncapped run, the
tracker being chunk-independent -- and fails a band call or a one-frame
over-budget request cleanly, before allocating; a parked device context is
trimmed and restored to its defaults (klt_hip_ctx_reset), and
klt_amd_release_cached_devices frees the parked ones."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import pytest

from conftest import synth
from kltabi import OracleTracker
from test_gpu_track import assert_table_equal, batch_sequence

pytestmark = pytest.mark.gpu


def test_budget_caps_chunk_results_unchanged(gpu, oracle):
    frames = synth(gpu, 5151, 640, 480, 14)
    seen = {}

    def hook(ctx, done=False):
        if not done:
            # room for three banks of 5 frames, not of the 13 asked for
            from kltamd.device import PyrDesc
            one = 3 * (640 * 480 * 12 + 160 * 120 * 12 + 160 * 480 * 4) + 14 * (64 << 10)
            assert gpu.klt_hip_set_bank_budget(ctx, 5 * one) == 0
            assert gpu.klt_hip_get_bank_budget(ctx) == 5 * one
        else:
            seen["chunk"] = gpu.klt_hip_frames_chunk(ctx)
            seen["foot"] = gpu.klt_hip_ctx_footprint(ctx)

    X, Y, V = batch_sequence(gpu, frames, 1000, [13], ctx_hook=hook)
    assert 1 <= seen["chunk"] < 13, seen
    OX, OY, OV = OracleTracker(oracle).harness(frames, 1000, 14, first=frames[0])
    assert_table_equal(X, Y, V, OX, OY, OV)
    X2, Y2, V2 = batch_sequence(gpu, frames, 1000, [13])
    assert np.array_equal(X.view(np.int32), X2.view(np.int32)) and np.array_equal(V, V2)


def test_budget_errors_are_clean(gpu):
    from kltamd.device import PyrDesc, TrackDesc, check
    W, H = 640, 480
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    pd, td = PyrDesc(), TrackDesc()
    gpu.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    gpu.klt_amd_track_desc(tc, C.byref(td))
    fr = gpu.klt_hip_malloc(ctx, 9 * W * H)
    check(gpu, ctx, gpu.klt_hip_synth_frames(ctx, 7, 0, 9, W, H, fr, W, W * H), "synth")
    check(gpu, ctx, gpu.klt_hip_frames_begin(ctx, C.byref(pd), fr, W), "begin")
    foot0 = gpu.klt_hip_ctx_footprint(ctx)
    # not even one frame per bank
    assert gpu.klt_hip_set_bank_budget(ctx, 1 << 20) == 0
    assert gpu.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), fr + W * H, W, W * H, 8, 8, None, None, None, 0,
                                    None, None, None, 0) < 0
    assert b"bank budget" in gpu.klt_hip_last_error(ctx)
    assert gpu.klt_hip_ctx_footprint(ctx) == foot0  # nothing was allocated
    # a band call whose chunk does not fit fails instead of shortening its exchange span
    one = 3 * (W * H * 12 + (W // 4) * (H // 4) * 12 + (W // 4) * H * 4) + 14 * (64 << 10)
    assert gpu.klt_hip_set_bank_budget(ctx, 3 * one) == 0
    esc = gpu.klt_hip_malloc(ctx, 4)
    check(gpu, ctx, gpu.klt_hip_memcpy(ctx, esc, np.zeros(1, np.int32).ctypes.data, 4, 1), "h2d")
    assert gpu.klt_hip_track_frames_band(ctx, C.byref(pd), C.byref(td), fr + W * H, W, W * H, 8, None, None, None,
                                         0, 0.0, float(H), 0, H, esc, None, 0) < 0
    assert b"over the budget" in gpu.klt_hip_last_error(ctx)
    # within the budget the same call runs
    assert gpu.klt_hip_set_bank_budget(ctx, 0) == 0
    check(gpu, ctx, gpu.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), fr + W * H, W, W * H, 8, 8, None, None,
                                             None, 0, None, None, None, 0), "frames")
    assert gpu.klt_hip_frames_chunk(ctx) == 8
    gpu.klt_hip_free(ctx, esc)
    gpu.klt_hip_free(ctx, fr)
    gpu.KLTFreeTrackingContext(tc)


def test_reset_trims_and_restores_defaults(gpu):
    """A context holding more than 2 GiB is trimmed when parked; a host-thread
    setting does not leak into the next tracking context."""
    from kltamd.device import PyrDesc, TrackDesc, check
    gpu.klt_amd_release_cached_devices()
    W, H = 1920, 1080
    tc = gpu.KLTCreateTrackingContext()
    ctx = gpu.klt_amd_device_context(tc)
    check(gpu, ctx, gpu.klt_hip_set_host_threads(ctx, 2), "threads")
    pd, td = PyrDesc(), TrackDesc()
    gpu.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    gpu.klt_amd_track_desc(tc, C.byref(td))
    n = 34
    fr = gpu.klt_hip_malloc(ctx, n * W * H)
    check(gpu, ctx, gpu.klt_hip_synth_frames(ctx, 7, 0, n, W, H, fr, W, W * H), "synth")
    check(gpu, ctx, gpu.klt_hip_frames_begin(ctx, C.byref(pd), fr, W), "begin")
    check(gpu, ctx, gpu.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), fr + W * H, W, W * H, n - 1, 32, None,
                                             None, None, 0, None, None, None, 0), "frames")
    assert gpu.klt_hip_ctx_footprint(ctx) > (2 << 30)
    gpu.klt_hip_free(ctx, fr)
    gpu.KLTFreeTrackingContext(tc)  # parked, trimmed
    tc2 = gpu.KLTCreateTrackingContext()
    ctx2 = gpu.klt_amd_device_context(tc2)
    assert ctx2 == ctx  # the parked context is handed on
    assert gpu.klt_hip_ctx_footprint(ctx2) <= (2 << 30)
    env = os.environ.get("KLT_AMD_HOST_THREADS")  # the library's default (runtime.hip), clamped to 0..16
    assert gpu.klt_hip_get_host_threads(ctx2) == (min(max(int(env), 0), 16) if env else 7)
    gpu.KLTFreeTrackingContext(tc2)
    assert gpu.klt_amd_release_cached_devices() >= 1
    assert gpu.klt_amd_release_cached_devices() == 0


def test_registered_buffers_bit_identical(gpu):
    """klt_amd_register_buffer (klt_amd.h): example3.c's two reused buffers,
    page-locked once, give the same lists as the staged upload; overlapping
    registrations and unknown pointers are refused with a warning."""
    from kltabi import fl_to_arrays, u8ptr
    frames = synth(gpu, 4242, 640, 480, 6)
    H, W = frames[0].shape

    def loop(register):
        img1, img2 = np.empty((H, W), np.uint8), np.empty((H, W), np.uint8)
        tc = gpu.KLTCreateTrackingContext()
        tc.contents.sequentialMode = 1
        if register:
            assert gpu.klt_amd_register_buffer(tc, img1.ctypes.data, img1.nbytes) == 0
            assert gpu.klt_amd_register_buffer(tc, img2.ctypes.data, img2.nbytes) == 0
            assert gpu.klt_amd_register_buffer(tc, img2.ctypes.data + 16, 64) == -1  # overlaps img2
        fl = gpu.KLTCreateFeatureList(500)
        img1[:] = frames[0]
        gpu.KLTSelectGoodFeatures(tc, u8ptr(img1), W, H, fl)
        cols = []
        for t in range(1, len(frames)):
            img2[:] = frames[t]
            gpu.KLTTrackFeatures(tc, u8ptr(img1), u8ptr(img2), W, H, fl)
            gpu.KLTReplaceLostFeatures(tc, u8ptr(img2), W, H, fl)
            cols.append(fl_to_arrays(fl))
            img1[:] = img2
        if register:
            assert gpu.klt_amd_unregister_buffer(tc, img1.ctypes.data) == 0
            assert gpu.klt_amd_unregister_buffer(tc, img1.ctypes.data) == -1  # no longer registered
        gpu.KLTFreeFeatureList(fl)
        gpu.KLTFreeTrackingContext(tc)  # img2 is released with the context
        return cols

    a, b = loop(False), loop(True)
    for ca, cb in zip(a, b):
        for p, q in zip(ca, cb):
            assert np.array_equal(p.view(np.int32), q.view(np.int32))


def test_reset_drains_the_callers_stream(gpu):
    """a context parked (klt_hip_ctx_reset) while the caller's
    stream (klt_hip_set_stream) still runs its work waits for that work before
    its buffers are freed and the context is handed on -- for the stream
    still set, for one the context switched away from, and for
    stream A after A -> own -> B, where B's record must not replace A's."""
    import torch
    from kltamd.device import check
    W, H, n = 1920, 1080, 96
    dev = torch.device("cuda", 0)
    for mode in ("still_set", "switch_away", "a_own_b"):
        tc = gpu.KLTCreateTrackingContext()
        ctx = gpu.klt_amd_device_context(tc)
        s = torch.cuda.Stream(dev)
        check(gpu, ctx, gpu.klt_hip_set_stream(ctx, C.c_void_p(s.cuda_stream)), "set_stream")
        fr = torch.empty((n, H, W), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        check(gpu, ctx, gpu.klt_hip_synth_frames(ctx, 9, 0, n, W, H, C.c_void_p(fr.data_ptr()), W, W * H), "synth")
        if mode != "still_set":
            check(gpu, ctx, gpu.klt_hip_set_stream(ctx, None), "own stream")
        if mode == "a_own_b":
            b = torch.cuda.Stream(dev)  # idle: only A holds the context's work
            check(gpu, ctx, gpu.klt_hip_set_stream(ctx, C.c_void_p(b.cuda_stream)), "set_stream B")
        gpu.KLTFreeTrackingContext(tc)  # parks the device context: klt_hip_ctx_reset
        assert s.query(), f"{mode}: the reset returned while the caller's stream still ran the context's work"
        del fr
    assert gpu.klt_amd_release_cached_devices() >= 1


SEQ_EXIT_CHILD = r"""
import ctypes as C, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import kltamd
lib = kltamd.load()
lib.KLTSetVerbosity(0)
W, H, NF, n = 1280, 720, 2000, 40
U8P = C.POINTER(C.c_ubyte)
fr = []
for t in range(n):
    a = np.empty((H, W), np.uint8)
    lib.klt_synth_frame(720, t, W, H, a.ctypes.data)
    fr.append(a)
arr = (U8P * n)(*[a.ctypes.data_as(U8P) for a in fr])
ft = lib.KLTCreateFeatureTable(n - 1, NF)
parked = lib.KLTCreateTrackingContext()  # freed below: parked with its copy pool, streams and staging
tc = lib.KLTCreateTrackingContext()      # never freed: live at exit
for c in (parked, tc):
    c.contents.sequentialMode = 1
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(c, arr[0], W, H, fl)
    lib.KLTTrackSequence(c, arr, n, W, H, fl, ft, 0)
img = np.empty((H, W), np.uint8)  # a registered caller buffer, still registered at exit
assert lib.klt_amd_register_buffer(tc, img.ctypes.data_as(C.c_void_p), img.nbytes) == 0
img[:] = fr[-1]
lib.KLTTrackFeatures(tc, arr[n - 1], img.ctypes.data_as(U8P), W, H, fl)
lib.KLTFreeTrackingContext(parked)
print("child done", flush=True)
"""


def test_exit_after_sequence_with_live_context(tmp_path):
    """a process that ran KLTTrackSequence (copy pool,
    copy streams, pinned staging) and a registered-buffer KLTTrackFeatures
    exits with one tracking context live and one parked: rc 0, promptly.  The
    exit hook (runtime.hip exit_release_host) drains the device and releases
    the host pipeline of every context before the HIP runtime's teardown."""
    import subprocess
    import sys
    import time
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    script = tmp_path / "seq_exit_child.py"
    script.write_text(SEQ_EXIT_CHILD)
    a = time.perf_counter()
    r = subprocess.run([sys.executable, str(script), str(root)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "child done" in r.stdout
    assert time.perf_counter() - a < 60
