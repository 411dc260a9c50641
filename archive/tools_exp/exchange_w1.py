"""What the exchange of include/klt_shard.h costs a rank, measured at world 1
(one GPU cannot run RCCL over xGMI): klt_shard_track per 64-frame chunk (band
call + k_shard_pack + ncclAllReduce of 3n+2 int32 + the flag read + unpack)
against klt_hip_track_frames_band + the same host read of the escape flag,
4K frames, 20 000 features, alternating, after a warm-up.  The difference per
chunk is the exchange's fixed cost on this rank; the xGMI transfer of an
8-rank ring (2*(N-1)/N * 240 KB per rank) is on top of it."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import kltamd  # noqa: E402
from kltamd.device import PyrDesc, TrackDesc, check, use_torch_stream  # noqa: E402
from kltabi import fl_to_arrays, u8ptr  # noqa: E402

W, H, NF, CH, T = 3840, 2160, 20000, 64, 192
lib = kltamd.load()
lib.KLTSetVerbosity(0)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
fr = torch.empty((T + 1, H, W), dtype=torch.uint8, device=dev)
tc = lib.KLTCreateTrackingContext()
tc.contents.sequentialMode = 1
ctx = lib.klt_amd_device_context(tc)
use_torch_stream(lib, ctx, dev)
check(lib, ctx, lib.klt_hip_synth_frames(ctx, 2160, 0, T + 1, W, H, C.c_void_p(fr.data_ptr()), W, W * H), "synth")
f0 = np.ascontiguousarray(fr[0].cpu().numpy())
fl = lib.KLTCreateFeatureList(NF)
lib.KLTSelectGoodFeatures(tc, u8ptr(f0), W, H, fl)
x0, y0, v0 = (torch.from_numpy(np.asarray(a)).to(dev) for a in fl_to_arrays(fl))
lib.KLTFreeFeatureList(fl)
pd, td = PyrDesc(), TrackDesc()
lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
lib.klt_amd_track_desc(tc, C.byref(td))
uid = (C.c_ubyte * 128)()
assert lib.klt_shard_unique_id(uid) == 0
s = lib.klt_shard_create(ctx, 0, 1, uid, H, 64)
assert s
esc = torch.zeros(1, dtype=torch.int32, device=dev)
ptr = lambda t: C.c_void_p(fr.data_ptr() + t * H * W)  # noqa: E731
res = {"shard_track": [], "band_call": []}
for rep in range(4):
    for mode in ("shard_track", "band_call"):
        x, y, v = x0.clone(), y0.clone(), v0.clone()
        check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), ptr(0), W), "begin")
        torch.cuda.synchronize()
        per = []
        for c0 in range(1, 1 + T, CH):
            nn = CH if c0 + CH < 1 + T else 0
            t0 = time.perf_counter()
            if mode == "shard_track":
                rc = lib.klt_shard_track(s, C.byref(pd), C.byref(td), ptr(c0), W, H * W, CH, ptr(c0 + CH) if nn else None,
                                         nn, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                                         C.c_void_p(v.data_ptr()), NF, None, None)
                assert rc == 0, lib.klt_shard_last_error(s)
            else:
                esc.zero_()
                check(lib, ctx, lib.klt_hip_track_frames_band(
                    ctx, C.byref(pd), C.byref(td), ptr(c0), W, H * W, CH, C.c_void_p(x.data_ptr()),
                    C.c_void_p(y.data_ptr()), C.c_void_p(v.data_ptr()), NF, C.c_float(-np.inf), C.c_float(np.inf),
                    0, H, C.c_void_p(esc.data_ptr()), ptr(c0 + CH) if nn else None, nn), "band")
                assert int(esc.item()) == 0
            per.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        if rep > 0:  # the first round warms up both paths
            res[mode].append(1e6 * float(np.median(per)))
out = {"workload": f"{W}x{H}, {NF} features, {CH}-frame chunks, world 1 (real RCCL communicator)",
       "us_per_chunk_median": {k: sorted(v) for k, v in res.items()},
       "exchange_us_per_chunk": float(np.median(res["shard_track"]) - np.median(res["band_call"])),
       "allreduce_bytes": 4 * (3 * NF + 2)}
print(json.dumps(out))
lib.klt_shard_destroy(s)
lib.KLTFreeTrackingContext(tc)
