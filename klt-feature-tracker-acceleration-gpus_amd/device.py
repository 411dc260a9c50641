"""ctypes binding of the device C ABI (include/klt_hip.h) of libklt_amd.so.

Used by bench.py and the GPU tests for device-resident work (frames and
feature arrays kept in HBM); the klt.h API (abi.py) is the drop-in surface.
"""
from __future__ import annotations

import ctypes
import ctypes as C
import os

MAX_TAPS = 71
MAX_LEVELS = 8
EXACT, FAST = 0, 1


class Taps(C.Structure):
    _fields_ = [("width", C.c_int), ("k", C.c_float * MAX_TAPS)]


class PyrDesc(C.Structure):
    _fields_ = [("ncols", C.c_int), ("nrows", C.c_int), ("nlevels", C.c_int),
                ("subsampling", C.c_int), ("smooth_input", C.c_int), ("smooth", Taps),
                ("pyr", Taps), ("grad_gauss", Taps), ("grad_deriv", Taps)]


class TrackDesc(C.Structure):
    _fields_ = [("window_width", C.c_int), ("window_height", C.c_int),
                ("max_iterations", C.c_int), ("min_determinant", C.c_float),
                ("min_displacement", C.c_float), ("max_residue", C.c_float),
                ("step_factor", C.c_float), ("borderx", C.c_int), ("bordery", C.c_int),
                ("lighting_insensitive", C.c_int), ("reduction", C.c_int)]


class SelectDesc(C.Structure):
    _fields_ = [("window_width", C.c_int), ("window_height", C.c_int), ("borderx", C.c_int),
                ("bordery", C.c_int), ("nSkippedPixels", C.c_int)]


class Timing(C.Structure):
    _fields_ = [("n_pyr_l0", C.c_int), ("n_pyr_l1", C.c_int), ("n_track", C.c_int),
                ("n_eigen", C.c_int), ("n_generic", C.c_int), ("ms_pyr_l0", C.c_double),
                ("ms_pyr_l1", C.c_double), ("ms_track", C.c_double), ("ms_eigen", C.c_double),
                ("ms_generic", C.c_double), ("frames_pyr_l0", C.c_long), ("frames_pyr_l1", C.c_long),
                ("frames_track", C.c_long)]


V = C.c_void_p
FP = C.POINTER(C.c_float)
IP = C.POINTER(C.c_int)
DP = C.POINTER(C.c_double)

DEVICE_PROTOS = {
    "klt_hip_ctx_create": (V, [C.c_int]),
    "klt_hip_ctx_destroy": (None, [V]),
    "klt_hip_last_error": (C.c_char_p, [V]),
    "klt_hip_track_kernel": (C.c_char_p, [V]),
    "klt_hip_set_stream": (C.c_int, [V, V]),
    "klt_hip_get_stream": (V, [V]),
    "klt_hip_sync": (C.c_int, [V]),
    "klt_hip_device_count": (C.c_int, []),
    "klt_hip_current_device": (C.c_int, []),
    "klt_hip_upload_frame": (C.c_int, [V, C.c_int, V, C.c_int, C.c_int]),
    "klt_hip_build_pyramid": (C.c_int, [V, C.c_int, C.POINTER(PyrDesc), V, C.c_long, C.c_int]),
    "klt_hip_pyramid_path": (C.c_int, [V, C.c_int]),
    "klt_hip_fused_path": (C.c_int, [V, C.POINTER(PyrDesc)]),
    "klt_hip_set_track_order": (C.c_int, [V, C.c_int]),
    "klt_hip_set_track_merge": (C.c_int, [V, C.c_int]),
    "klt_hip_set_track_prio": (C.c_int, [V, C.c_int]),
    "klt_hip_set_track_impl": (C.c_int, [V, C.c_int]),
    "klt_hip_set_track_patch": (C.c_int, [V, C.c_int]),
    "klt_hip_set_track_count": (C.c_int, [V, C.c_int]),
    "klt_hip_get_track_count": (C.c_int, [V, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), C.c_int]),
    "klt_hip_set_prof": (C.c_int, [V, V]),
    "klt_hip_set_frames_overlap": (C.c_int, [V, C.c_int]),
    "klt_hip_set_host_threads": (C.c_int, [V, C.c_int]),
    "klt_hip_get_host_threads": (C.c_int, [V]),
    "klt_hip_set_path": (C.c_int, [V, C.c_int]),
    "klt_hip_set_bank_budget": (C.c_int, [V, C.c_size_t]),
    "klt_hip_get_bank_budget": (C.c_size_t, [V]),
    "klt_hip_frames_chunk": (C.c_int, [V]),
    "klt_hip_ctx_footprint": (C.c_size_t, [V]),
    "klt_hip_ctx_reset": (C.c_int, [V]),
    "klt_hip_level_dims": (C.c_int, [V, C.c_int, C.c_int, IP, IP]),
    "klt_hip_download_level": (C.c_int, [V, C.c_int, C.c_int, C.c_int, V]),
    "klt_hip_level_ptr": (V, [V, C.c_int, C.c_int, C.c_int]),
    "klt_hip_level_interleaved": (C.c_int, [V, C.c_int, C.c_int]),
    "klt_hip_track": (C.c_int, [V, C.c_int, C.c_int, C.POINTER(TrackDesc), V, V, V, C.c_int, C.c_int]),
    "klt_hip_track_sequence": (C.c_int, [V, C.POINTER(PyrDesc), C.POINTER(TrackDesc), V, C.c_long,
                                         C.c_long, C.c_int, C.c_int, V, V, V, C.c_int, IP]),
    "klt_hip_frames_begin": (C.c_int, [V, C.POINTER(PyrDesc), V, C.c_long]),
    "klt_hip_frames_begin_slot": (C.c_int, [V, C.c_int]),
    "klt_hip_frames_end_slot": (C.c_int, [V, C.c_int]),
    "klt_hip_track_frames": (C.c_int, [V, C.POINTER(PyrDesc), C.POINTER(TrackDesc), V, C.c_long, C.c_long,
                                       C.c_int, C.c_int, V, V, V, C.c_int, V, V, V, C.c_long]),
    "klt_hip_track_frames_band": (C.c_int, [V, C.POINTER(PyrDesc), C.POINTER(TrackDesc), V, C.c_long, C.c_long,
                                            C.c_int, V, V, V, C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, V,
                                            V, C.c_int]),
    "klt_shard_unique_id": (C.c_int, [V]),
    "klt_shard_band_edges": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "klt_shard_create": (V, [V, C.c_int, C.c_int, V, C.c_int, C.c_int]),
    "klt_shard_create_local": (V, [V, C.c_int, C.c_int, C.c_int, C.c_int]),
    "klt_shard_destroy": (None, [V]),
    "klt_shard_last_error": (C.c_char_p, [V]),
    "klt_shard_create_error": (C.c_char_p, []),
    "klt_shard_inject_fault": (C.c_int, [V, C.c_int]),
    "klt_shard_rows": (C.c_int, [V, IP, IP]),
    "klt_shard_track": (C.c_int, [V, C.POINTER(PyrDesc), C.POINTER(TrackDesc), V, C.c_long, C.c_long, C.c_int, V,
                                  C.c_int, V, V, V, C.c_int, V, V]),
    "klt_hip_select_map": (C.c_int, [V, C.c_int, C.c_int, V, C.c_int, C.c_int, V, V, V, V, C.c_int]),
    "klt_hip_min_eigen_rows": (C.c_int, [V, V, C.c_int, C.c_int, V, IP, IP, IP, IP]),
    "klt_hip_gather_order": (C.c_int, [V, V, V, V, C.c_int, FP, C.c_int, V, V, V, V]),
    "klt_hip_gather_pack": (C.c_int, [V, V, V, V, V, C.c_int, C.c_int, C.c_int, V, C.c_int, V, C.c_int]),
    "klt_hip_gather_unpack": (C.c_int, [V, V, C.c_int, C.c_int, V, C.c_int, C.c_int, C.c_int, V, V, V, V, V]),
    "klt_hip_gather_work_ints": (C.c_long, [C.c_int, C.c_int]),
    "klt_hip_gather_unpack_order": (C.c_int, [V, V, C.c_int, C.c_int, V, C.c_int, C.c_int, C.c_int, V, V, V, V, V,
                                              FP, V, V, V]),
    "klt_hip_set_ahead_ready": (C.c_int, [V, C.c_int]),
    "klt_shard_eigen": (C.c_int, [V, C.POINTER(PyrDesc), V, C.c_long, V, V, V]),
    "klt_shard_select": (C.c_int, [V, C.POINTER(PyrDesc), V, C.c_int, C.c_int, V, V, V, V, C.c_int]),
    "klt_shard_replace": (C.c_int, [V, C.POINTER(PyrDesc), V, C.c_long, C.c_int, C.c_int, V, V, V, C.c_int, V, V]),
    "klt_hip_min_eigen": (C.c_int, [V, C.c_int, C.POINTER(SelectDesc), V, IP, IP]),
    "klt_hip_select": (C.c_int, [V, C.c_int, C.POINTER(SelectDesc), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 V, V, V, V, C.c_int]),
    "klt_hip_select_dev_map": (C.c_int, [V, V, C.c_int, C.c_int, C.POINTER(SelectDesc), C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.c_int, V, V, V, V, C.c_int]),
    "klt_hip_select_tune": (C.c_int, [V, C.c_int]),
    "klt_hip_select_stats": (C.c_int, [V, C.POINTER(C.c_long), C.POINTER(C.c_long), C.POINTER(C.c_long), DP]),
    "klt_hip_select_sort_test": (C.c_int, [V, V, C.c_int, V, V]),
    "klt_hip_synth_rows": (C.c_int, [V, C.c_ulonglong, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, V,
                                     C.c_long, C.c_long]),
    "klt_hip_synth_frames": (C.c_int, [V, C.c_ulonglong, C.c_int, C.c_int, C.c_int, C.c_int, V,
                                       C.c_long, C.c_long]),
    "klt_hip_malloc": (V, [V, C.c_size_t]),
    "klt_hip_free": (None, [V, V]),
    "klt_hip_memcpy": (C.c_int, [V, V, V, C.c_size_t, C.c_int]),
    "klt_hip_set_timing": (C.c_int, [V, C.c_int]),
    "klt_hip_get_timing": (C.c_int, [V, C.POINTER(Timing)]),
    "klt_hip_selftest_sqrt": (C.c_int, [V, DP, DP, C.c_int]),
    "klt_hip_selftest_div": (C.c_int, [V, FP, FP, FP, C.c_int]),
    "klt_hip_selftest_copy_pool": (C.c_int, [C.c_int, C.c_int, C.c_size_t]),
    # klt_api.c hooks
    "klt_amd_device_context": (V, [V]),
    "klt_amd_pyr_desc": (None, [V, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(PyrDesc)]),
    "klt_amd_track_desc": (None, [V, C.POINTER(TrackDesc)]),
    "klt_amd_set_reduction": (None, [V, C.c_int]),
    "klt_amd_release_cached_devices": (C.c_int, []),
    "klt_amd_register_buffer": (C.c_int, [V, V, C.c_size_t]),
    "klt_amd_unregister_buffer": (C.c_int, [V, V]),
    "klt_hip_register_host": (C.c_int, [V, V, C.c_size_t]),
    "klt_hip_unregister_host": (C.c_int, [V, V]),
    # host helpers
    "klt_synth_frame": (None, [C.c_uint64, C.c_int, C.c_int, C.c_int, V]),
    "klt_sort_pairs_full": (None, [IP, IP, C.c_int]),
}

H2D, D2H, D2D = 1, 2, 3  # hipMemcpyKind


def bind_device(lib: C.CDLL) -> C.CDLL:
    # KLT_AMD_LIB may name an older build (same-box A/B tools): its missing
    # extensions stay unbound; the shipped library exports all of them
    # (tests/test_abi.py)
    alt = bool(os.environ.get("KLT_AMD_LIB"))
    for name, (res, args) in DEVICE_PROTOS.items():
        if alt and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


class DeviceError(RuntimeError):
    pass


def check(lib: C.CDLL, ctx, rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.klt_hip_last_error(ctx)
        raise DeviceError(f"{what}: {msg.decode() if msg else 'error'}")


def use_torch_stream(lib, ctx, device=None):
    """Run the library and torch on one stream.  torch's default stream is the
    null stream (handle 0), which klt_hip_set_stream reads as "the context's
    own non-blocking stream" -- unordered with torch.  So make a dedicated
    torch stream current and hand that to the library.  Returns the stream."""
    import torch
    s = torch.cuda.current_stream(device)
    if s.cuda_stream == 0:
        s = torch.cuda.Stream(device)
        torch.cuda.set_stream(s)
    check(lib, ctx, lib.klt_hip_set_stream(ctx, ctypes.c_void_p(s.cuda_stream)), "set_stream")
    return s
