"""Shared fixtures.  `-m gpu` tests need a real MI355X (run through gpurun);
everything else runs on the CPU-only build container."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import kltabi  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    if not kltabi.ORACLE_LIB.exists():
        pytest.fail(f"{kltabi.ORACLE_LIB} missing: run `make -C oracle` (or __graft_entry__.build())")
    return kltabi.load_oracle()


@pytest.fixture(scope="session")
def ref():
    """The reference compiled from /root/reference (oracle/_ref); optional."""
    if not kltabi.REF_LIB.exists():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    return kltabi.bind_klt(kltabi.REF_LIB)


@pytest.fixture(scope="session")
def amd():
    import kltamd
    lib = kltamd.load()
    lib.KLTSetVerbosity(0)
    return lib


@pytest.fixture(scope="session")
def gpu(amd):
    if amd.klt_hip_device_count() <= 0:
        pytest.fail("no HIP device visible: -m gpu tests must run on the GPU box")
    return amd


@pytest.fixture(scope="session")
def frames():
    return kltabi.load_dataset()


def synth(amd, seed: int, w: int, h: int, n: int, t0: int = 0):
    out = []
    for t in range(t0, t0 + n):
        a = np.empty((h, w), np.uint8)
        amd.klt_synth_frame(seed, t, w, h, a.ctypes.data)
        out.append(a)
    return out


@pytest.fixture(scope="session")
def syn640(amd):
    return synth(amd, 640480, 640, 480, 12)


@pytest.fixture(scope="session")
def syn333(amd):
    return synth(amd, 333, 333, 251, 8)
