"""Experiment: why bench.py's roofline_4k pass is slower than microbench's.
Variants of bench.pass_4k in one process, alternated."""
import ctypes as C, json, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import torch
import kltamd
from kltamd.device import PyrDesc, TrackDesc, Timing, check, use_torch_stream

def run(lib, dev, torch_stream, torch_frames, chunk=64, reps=2):
    W, H = 3840, 2160
    tc = lib.KLTCreateTrackingContext()
    ctx = lib.klt_amd_device_context(tc)
    if torch_stream:
        use_torch_stream(lib, ctx, dev)
    n = 1 + chunk * (1 + reps)
    if torch_frames:
        fr = torch.empty((n, H, W), dtype=torch.uint8, device=dev); base = fr.data_ptr()
    else:
        fr = None; base = lib.klt_hip_malloc(ctx, n * W * H)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, 2160, 0, n, W, H, C.c_void_p(base), W, W * H), "synth")
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    def go(t0, m):
        check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(base + t0 * W * H), W,
                                                 W * H, m, chunk, None, None, None, 0, None, None, None, 0), "4k")
    check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(base), W), "begin")
    go(1, chunk)
    lib.klt_hip_sync(ctx); torch.cuda.synchronize()
    lib.klt_hip_set_timing(ctx, 1)
    go(1 + chunk, chunk * reps)
    tm = Timing()
    check(lib, ctx, lib.klt_hip_get_timing(ctx, C.byref(tm)), "timing")
    if fr is None:
        lib.klt_hip_free(ctx, C.c_void_p(base))
    lib.KLTFreeTrackingContext(tc)
    del fr
    torch.cuda.empty_cache()
    return round(1000.0 * tm.ms_pyr_l0 / tm.frames_pyr_l0, 2), round(1000.0 * tm.ms_pyr_l1 / tm.frames_pyr_l1, 2)

lib = kltamd.load(); lib.KLTSetVerbosity(0)
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
order = [a for a in sys.argv[1:] if not a.startswith("--")] or ["lib", "torch", "tstream", "tframes"]
for r in range(2):
    for v in order:
        ts = v in ("torch", "tstream"); tf = v in ("torch", "tframes")
        print(v, run(lib, dev, ts, tf), flush=True)

def pre1080(lib, dev):
    """a 1080p tracking context like bench.py's main leg, then freed (its device context is cached)"""
    W, H, NF, T = 1920, 1080, 5000, 200
    tc = lib.KLTCreateTrackingContext(); tc.contents.sequentialMode = 1
    ctx = lib.klt_amd_device_context(tc)
    use_torch_stream(lib, ctx, dev)
    fr = torch.empty((T + 1, H, W), dtype=torch.uint8, device=dev)
    check(lib, ctx, lib.klt_hip_synth_frames(ctx, 1080, 0, T + 1, W, H, C.c_void_p(fr.data_ptr()), W, W * H), "synth")
    import numpy as np
    f0 = fr[0].cpu().numpy()
    fl = lib.KLTCreateFeatureList(NF)
    lib.KLTSelectGoodFeatures(tc, f0.ctypes.data_as(C.POINTER(C.c_ubyte)), W, H, fl)
    xs = torch.tensor([fl.contents.feature[k].contents.x for k in range(NF)], device=dev)
    ys = torch.tensor([fl.contents.feature[k].contents.y for k in range(NF)], device=dev)
    vs = torch.tensor([fl.contents.feature[k].contents.val for k in range(NF)], dtype=torch.int32, device=dev)
    lib.KLTFreeFeatureList(fl)
    pd, td = PyrDesc(), TrackDesc()
    lib.klt_amd_pyr_desc(tc, W, H, tc.contents.nPyramidLevels, 1, C.byref(pd))
    lib.klt_amd_track_desc(tc, C.byref(td))
    tab = [torch.empty((T, NF), dtype=dt, device=dev) for dt in (torch.float32, torch.float32, torch.int32)]
    check(lib, ctx, lib.klt_hip_frames_begin(ctx, C.byref(pd), C.c_void_p(fr.data_ptr()), W), "begin")
    check(lib, ctx, lib.klt_hip_track_frames(ctx, C.byref(pd), C.byref(td), C.c_void_p(fr.data_ptr() + W * H), W, W * H,
                                             T, 64, C.c_void_p(xs.data_ptr()), C.c_void_p(ys.data_ptr()),
                                             C.c_void_p(vs.data_ptr()), NF, *[C.c_void_p(a.data_ptr()) for a in tab], NF), "tf")
    torch.cuda.synchronize()
    lib.KLTFreeTrackingContext(tc)
    del fr, tab

if __name__ == "__main__" and "--pre1080" in sys.argv:
    pre1080(lib, dev)
    for r in range(3):
        print("after1080 torch", run(lib, dev, True, True), flush=True)
        print("after1080 lib", run(lib, dev, False, False), flush=True)
