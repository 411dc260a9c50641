#!/usr/bin/env python3
"""Kernel times of the exchange kernels alone (klt_hip_gather_order / pack /
unpack_order, 20 000 features, 8 ranks): HIP events over 200 launches each."""
import ctypes as C
import sys
from pathlib import Path
import numpy as np
import torch
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import kltamd
from kltamd.device import check, use_torch_stream
from kltamd.shard import band_edges, slot_words

lib = kltamd.load()
dev = torch.device("cuda", 0)
tc = lib.KLTCreateTrackingContext()
ctx = lib.klt_amd_device_context(tc)
use_torch_stream(lib, ctx, dev)
n, world, H = 20000, 8, 2160
rng = np.random.default_rng(1)
x = torch.from_numpy(rng.uniform(0, 3840, n).astype(np.float32)).to(dev)
y = torch.from_numpy(rng.uniform(0, H, n).astype(np.float32)).to(dev)
v = torch.from_numpy(np.where(rng.uniform(size=n) < 0.1, -1, 0).astype(np.int32)).to(dev)
E = (C.c_float * (world + 1))(*band_edges(H, world))
work = torch.zeros(lib.klt_hip_gather_work_ints(n, world), dtype=torch.int32, device=dev)
save = torch.zeros(3 * n, dtype=torch.int32, device=dev)
esc = torch.zeros(1, dtype=torch.int32, device=dev)
flags = torch.zeros(2, dtype=torch.int32, device=dev)
hc = torch.zeros(world, dtype=torch.int32).pin_memory()
hf = torch.zeros(2, dtype=torch.int32).pin_memory()
P = lambda t: C.c_void_p(t.data_ptr())


def timeit(name, fn, reps=200):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(f"{name}: {1e3 * a.elapsed_time(b) / reps:.1f} us per launch (back to back)", flush=True)


timeit("gather_order", lambda: check(lib, ctx, lib.klt_hip_gather_order(ctx, P(x), P(y), P(v), n, E, world, P(work),
                                                                         P(save), P(esc), P(hc)), "order"))
S = max(1, int(work[n:n + world].max().item()))
W = slot_words(S)
slots = torch.zeros(world * W, dtype=torch.int32, device=dev)
for r in range(world):
    check(lib, ctx, lib.klt_hip_gather_pack(ctx, P(x), P(y), P(v), P(work), n, world, r, P(esc), 0,
                                            C.c_void_p(slots[r * W:].data_ptr()), S), "pack")
timeit("gather_pack", lambda: check(lib, ctx, lib.klt_hip_gather_pack(ctx, P(x), P(y), P(v), P(work), n, world, 3,
                                                                       P(esc), 0, P(slots), S), "pack"))
timeit("gather_unpack_order", lambda: check(lib, ctx, lib.klt_hip_gather_unpack_order(
    ctx, P(slots), world, 0, P(work), n, world, S, P(x), P(y), P(v), P(flags), P(hf), E, P(save), P(esc), P(hc)),
    "unpack_order"))
lib.KLTFreeTrackingContext(tc)
