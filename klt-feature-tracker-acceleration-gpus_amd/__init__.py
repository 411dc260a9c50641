"""MI355X-native pyramidal KLT tracker (klt.h drop-in, HIP/CDNA4 kernels).

The product is the C-ABI shared library lib/libklt_amd.so (built from csrc/ by
`make -C csrc`, or __graft_entry__.build()).  This package only binds it:

    import kltamd                       # repo-root shim for this hyphenated dir
    lib = kltamd.load()                 # klt.h + klt_hip_* prototypes attached
    tc = lib.KLTCreateTrackingContext()

There is no Python or CPU fallback: load() raises if the library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

from . import abi, device  # noqa: F401

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "lib" / "libklt_amd.so"

_lib: C.CDLL | None = None


def load() -> C.CDLL:
    """Load libklt_amd.so once and attach every prototype."""
    global _lib
    if _lib is None:
        path = LIB_PATH
        alt = os.environ.get("KLT_AMD_LIB")  # tools only: e.g. the instrumented build lib/prof/
        if alt:
            path = Path(alt)
        if not path.exists():
            raise ImportError(f"{path} is missing: build it with `make -C {PKG_DIR / 'csrc'}` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
        abi.bind_klt(lib, extensions=True)
        device.bind_device(lib)
        _lib = lib
    return _lib
