"""The C examples (examples/): built by __graft_entry__.build(), run on the
GPU.  shard_world1 drives include/klt_shard.h from C over a one-rank RCCL
communicator with lost-feature replacement after every frame and compares the
list with the plain klt.h loop's, cell for cell."""
from __future__ import annotations

import subprocess
from pathlib import Path

import pytest

EX = Path(__file__).resolve().parents[1] / "examples"


def test_example_compiles_as_c():
    """The example compiles against the public headers as C (gcc, no HIP)."""
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", "-std=c99", f"-I{EX.parent / 'include'}",
                        str(EX / "shard_world1.c")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("args", [[], ["320", "240", "300", "7"], ["1920", "1080", "3000", "5"]])
def test_shard_world1_equals_klt_loop(tmp_path, args):
    exe = EX / "shard_world1"
    r = subprocess.run([str(exe), *args], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cells differing 0" in r.stdout
    replaced = int(r.stdout.split("replaced-in-last-frame")[1].split()[0])
    assert replaced > 0, r.stdout  # the replacement path ran
