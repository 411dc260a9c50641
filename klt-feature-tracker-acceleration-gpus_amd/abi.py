"""ctypes mirror of the klt.h C ABI (include/klt.h == reference src/V3/klt.h layout).

Pure definitions -- importing this module never loads a library, so tests can
bind the same ABI to the product (libklt_amd.so) and to the reference build.
Layouts (x86-64): KLT_TrackingContextRec 136 B with pyramid_last at 112,
KLT_FeatureRec 64 B, KLT_FeatureList/History/Table 16 B.
"""
from __future__ import annotations

import ctypes as C

KLT_TRACKED, KLT_NOT_FOUND, KLT_SMALL_DET = 0, -1, -2
KLT_MAX_ITERATIONS, KLT_OOB, KLT_LARGE_RESIDUE = -3, -4, -5


class FloatImageRec(C.Structure):
    _fields_ = [("ncols", C.c_int), ("nrows", C.c_int), ("data", C.POINTER(C.c_float))]


class TrackingContextRec(C.Structure):
    _fields_ = [
        ("mindist", C.c_int), ("window_width", C.c_int), ("window_height", C.c_int),
        ("sequentialMode", C.c_int), ("smoothBeforeSelecting", C.c_int),
        ("writeInternalImages", C.c_int), ("lighting_insensitive", C.c_int),
        ("min_eigenvalue", C.c_int), ("min_determinant", C.c_float),
        ("min_displacement", C.c_float), ("max_iterations", C.c_int),
        ("max_residue", C.c_float), ("grad_sigma", C.c_float),
        ("smooth_sigma_fact", C.c_float), ("pyramid_sigma_fact", C.c_float),
        ("step_factor", C.c_float), ("nSkippedPixels", C.c_int),
        ("borderx", C.c_int), ("bordery", C.c_int), ("nPyramidLevels", C.c_int),
        ("subsampling", C.c_int), ("affine_window_width", C.c_int),
        ("affine_window_height", C.c_int), ("affineConsistencyCheck", C.c_int),
        ("affine_max_iterations", C.c_int), ("affine_max_residue", C.c_float),
        ("affine_min_displacement", C.c_float),
        ("affine_max_displacement_differ", C.c_float),
        ("pyramid_last", C.c_void_p), ("pyramid_last_gradx", C.c_void_p),
        ("pyramid_last_grady", C.c_void_p),
    ]


class FeatureRec(C.Structure):
    _fields_ = [
        ("x", C.c_float), ("y", C.c_float), ("val", C.c_int),
        ("aff_img", C.POINTER(FloatImageRec)), ("aff_img_gradx", C.POINTER(FloatImageRec)),
        ("aff_img_grady", C.POINTER(FloatImageRec)),
        ("aff_x", C.c_float), ("aff_y", C.c_float), ("aff_Axx", C.c_float),
        ("aff_Ayx", C.c_float), ("aff_Axy", C.c_float), ("aff_Ayy", C.c_float),
    ]


class FeatureListRec(C.Structure):
    _fields_ = [("nFeatures", C.c_int), ("feature", C.POINTER(C.POINTER(FeatureRec)))]


class FeatureHistoryRec(C.Structure):
    _fields_ = [("nFrames", C.c_int), ("feature", C.POINTER(C.POINTER(FeatureRec)))]


class FeatureTableRec(C.Structure):
    _fields_ = [("nFrames", C.c_int), ("nFeatures", C.c_int),
                ("feature", C.POINTER(C.POINTER(C.POINTER(FeatureRec))))]


assert C.sizeof(TrackingContextRec) == 136 and TrackingContextRec.pyramid_last.offset == 112
assert C.sizeof(FeatureRec) == 64 and FeatureRec.aff_img.offset == 16
assert C.sizeof(FeatureListRec) == 16 and C.sizeof(FeatureTableRec) == 16

TC = C.POINTER(TrackingContextRec)
FL = C.POINTER(FeatureListRec)
FH = C.POINTER(FeatureHistoryRec)
FT = C.POINTER(FeatureTableRec)
U8P = C.POINTER(C.c_ubyte)

# name -> (restype, argtypes); the full klt.h surface (src/V3/klt.h:130-233)
KLT_PROTOS = {
    "KLTCreateTrackingContext": (TC, []),
    "KLTCreateFeatureList": (FL, [C.c_int]),
    "KLTCreateFeatureHistory": (FH, [C.c_int]),
    "KLTCreateFeatureTable": (FT, [C.c_int, C.c_int]),
    "KLTFreeTrackingContext": (None, [TC]),
    "KLTFreeFeatureList": (None, [FL]),
    "KLTFreeFeatureHistory": (None, [FH]),
    "KLTFreeFeatureTable": (None, [FT]),
    "KLTSelectGoodFeatures": (None, [TC, U8P, C.c_int, C.c_int, FL]),
    "KLTTrackFeatures": (None, [TC, U8P, U8P, C.c_int, C.c_int, FL]),
    "KLTReplaceLostFeatures": (None, [TC, U8P, C.c_int, C.c_int, FL]),
    "KLTCountRemainingFeatures": (C.c_int, [FL]),
    "KLTPrintTrackingContext": (None, [TC]),
    "KLTChangeTCPyramid": (None, [TC, C.c_int]),
    "KLTUpdateTCBorder": (None, [TC]),
    "KLTStopSequentialMode": (None, [TC]),
    "KLTSetVerbosity": (None, [C.c_int]),
    "_KLTComputeSmoothSigma": (C.c_float, [TC]),
    "KLTStoreFeatureList": (None, [FL, FT, C.c_int]),
    "KLTExtractFeatureList": (None, [FL, FT, C.c_int]),
    "KLTStoreFeatureHistory": (None, [FH, FT, C.c_int]),
    "KLTExtractFeatureHistory": (None, [FH, FT, C.c_int]),
    "KLTWriteFeatureListToPPM": (None, [FL, U8P, C.c_int, C.c_int, C.c_char_p]),
    "KLTWriteFeatureList": (None, [FL, C.c_char_p, C.c_char_p]),
    "KLTWriteFeatureHistory": (None, [FH, C.c_char_p, C.c_char_p]),
    "KLTWriteFeatureTable": (None, [FT, C.c_char_p, C.c_char_p]),
    "KLTReadFeatureList": (FL, [FL, C.c_char_p]),
    "KLTReadFeatureHistory": (FH, [FH, C.c_char_p]),
    "KLTReadFeatureTable": (FT, [FT, C.c_char_p]),
    # pnmio.h
    "pgmReadFile": (U8P, [C.c_char_p, U8P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pgmWriteFile": (None, [C.c_char_p, U8P, C.c_int, C.c_int]),
    "ppmWriteFileRGB": (None, [C.c_char_p, U8P, U8P, U8P, C.c_int, C.c_int]),
}


# libklt_amd.so extensions of the klt.h surface (include/klt_amd.h)
AMD_KLT_PROTOS = {
    "KLTTrackSequence": (None, [TC, C.POINTER(U8P), C.c_int, C.c_int, C.c_int, FL, FT, C.c_int]),
}


def bind_klt(lib: C.CDLL, extensions: bool = False) -> C.CDLL:
    """Attach the klt.h prototypes (and, for libklt_amd.so, its extensions)."""
    protos = dict(KLT_PROTOS, **AMD_KLT_PROTOS) if extensions else KLT_PROTOS
    for name, (res, args) in protos.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
