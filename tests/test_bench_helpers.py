"""bench.py's host helpers of the sharded_4k leg, on the CPU: the list digest
is the reference fixtures' column digest (tests/golden/long_config*.json:
sha256(x f32 LE || y f32 LE || val i32 LE)), and gather_floats -- the
per-rank timing and state exchange every rank takes part in at N > 1 -- over a
real world-size-2 gloo group."""
from __future__ import annotations

import hashlib
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_state_digest_is_the_fixture_column_digest():
    rng = np.random.default_rng(7)
    x = rng.random(1000, dtype=np.float32) * 3840
    y = rng.random(1000, dtype=np.float32) * 2160
    v = rng.integers(-4, 1, 1000).astype(np.int32)
    h = hashlib.sha256()
    h.update(x.astype("<f4").tobytes())
    h.update(y.astype("<f4").tobytes())
    h.update(v.astype("<i4").tobytes())
    got = bench.state_digest(torch.from_numpy(x), torch.from_numpy(y), torch.from_numpy(v))
    assert got == h.hexdigest()
    # bit patterns, not values: -0.0 and +0.0 digest differently
    x2 = x.copy()
    x2[0] = -0.0 if x[0] == 0.0 else x[0]
    x2[1] = -0.0
    x3 = x2.copy()
    x3[1] = 0.0
    assert bench.state_digest(torch.from_numpy(x2), torch.from_numpy(y), torch.from_numpy(v)) != \
        bench.state_digest(torch.from_numpy(x3), torch.from_numpy(y), torch.from_numpy(v))


def test_gather_floats_without_a_process_group():
    assert bench.gather_floats([1.5, 2.0], 1, torch.device("cpu")) == [[1.5, 2.0]]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, bench.gather_floats([float(rank), 10.0 + rank, 2.0 ** 40 + rank], world, torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def test_gather_floats_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [[0.0, 10.0, 2.0 ** 40], [1.0, 11.0, 2.0 ** 40 + 1]]
    assert [r[1] for r in res] == [want, want]  # every rank holds every rank's values, in rank order
