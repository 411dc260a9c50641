"""Helpers for the -m gpu tests: drive libklt_amd.so's device ABI directly."""
from __future__ import annotations

import ctypes as C

import numpy as np

import kltamd
from kltamd.device import PyrDesc, SelectDesc, TrackDesc, check


def bits(a: np.ndarray) -> np.ndarray:
    """Compare floats by bit pattern (catches -0.0 vs +0.0 and NaN payloads)."""
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


class Dev:
    """A tracking context plus its device context, for stage-level tests."""

    def __init__(self, lib, setup=None):
        self.lib = lib
        self.tc = lib.KLTCreateTrackingContext()
        if setup:
            setup(self.tc.contents)
        self.ctx = lib.klt_amd_device_context(self.tc)

    def close(self):
        if self.tc:
            self.lib.KLTFreeTrackingContext(self.tc)
            self.tc = None

    def __del__(self):
        self.close()

    def desc(self, w, h, nlevels=None, smooth=1):
        d = PyrDesc()
        n = self.tc.contents.nPyramidLevels if nlevels is None else nlevels
        self.lib.klt_amd_pyr_desc(self.tc, w, h, n, smooth, C.byref(d))
        return d

    def build(self, img: np.ndarray, slot=0, nlevels=None, smooth=1, force_generic=False):
        lib, ctx = self.lib, self.ctx
        h, w = img.shape
        d = self.desc(w, h, nlevels, smooth)
        img = np.ascontiguousarray(img)
        check(lib, ctx, lib.klt_hip_set_path(ctx, 1 if force_generic else 0), "set_path")
        check(lib, ctx, lib.klt_hip_upload_frame(ctx, 0, img.ctypes.data, w, h), "upload")
        check(lib, ctx, lib.klt_hip_build_pyramid(ctx, slot, C.byref(d), None, 0, 0), "build")
        return d

    def levels(self, slot, nlevels):
        lib, ctx = self.lib, self.ctx
        out = []
        for lv in range(nlevels):
            w, h = C.c_int(), C.c_int()
            check(lib, ctx, lib.klt_hip_level_dims(ctx, slot, lv, C.byref(w), C.byref(h)), "dims")
            planes = []
            for which in range(3):
                a = np.empty((h.value, w.value), np.float32)
                check(lib, ctx, lib.klt_hip_download_level(ctx, slot, lv, which, a.ctypes.data), "dl")
                planes.append(a)
            out.append(tuple(planes))
        return out

    def path(self, slot):
        return self.lib.klt_hip_pyramid_path(self.ctx, slot)

    def eigen(self, slot, setup_desc=None):
        t = self.tc.contents
        sd = SelectDesc(t.window_width, t.window_height,
                        max(t.borderx, t.window_width // 2), max(t.bordery, t.window_height // 2),
                        t.nSkippedPixels)
        nx, ny = C.c_int(), C.c_int()
        lib, ctx = self.lib, self.ctx
        check(lib, ctx, lib.klt_hip_min_eigen(ctx, slot, C.byref(sd), None, C.byref(nx), C.byref(ny)), "eig")
        out = np.empty(nx.value * ny.value, np.int32)
        check(lib, ctx, lib.klt_hip_min_eigen(ctx, slot, C.byref(sd), out.ctypes.data, C.byref(nx),
                                              C.byref(ny)), "eig")
        return out, nx.value, ny.value
