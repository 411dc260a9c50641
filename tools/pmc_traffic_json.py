#!/usr/bin/env python3
"""profiles/pmc_latest.json from a tools/pmc_traffic.sh run: HBM-side bytes per
frame of the pyramid pass (k_pyr_l0 + k_pyr_l1), from the batched launches.

FETCH_SIZE / WRITE_SIZE are in KiB (WRITE_SIZE checked against k_synth's known
output).  gfx950 FETCH_SIZE counts half of the bytes of 16-byte-per-lane reads
(MI355X_MICROARCH.md, HBM): k_pyr_l1 reads hs that way, so its FETCH is
doubled.  k_pyr_l0's interior tiles read the u8 frame 16 bytes per lane
(since v14; before, 4 bytes per lane, where its raw FETCH came out at 0.56x
the frame's own bytes, below the least it can read); it is doubled too (raw
values kept in the JSON).
usage: python tools/pmc_traffic_json.py gpurun_out/<tag> WIDTH HEIGHT [out.json]
"""
import csv
import glob
import json
import sys

root, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
out = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_latest.json"
per = {}
fpl = set()
threads_l0 = ((W + 63) // 64) * ((H + 31) // 32) * 256
W1, H1 = W // 4, H // 4
threads_l1 = ((W1 + 31) // 32) * ((H1 + 31) // 32) * 256
for path in glob.glob(f"{root}/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        kern = "l0" if "k_pyr_l0" in name else "l1" if "k_pyr_l1" in name else None
        if not kern:
            continue
        frames = int(r["Grid_Size"]) // (threads_l0 if kern == "l0" else threads_l1)
        if frames < 2:
            continue  # single-frame launches (sequence starts) are not the batched pass
        per.setdefault((kern, r["Counter_Name"]), []).append(float(r["Counter_Value"]) * 1024 / frames)
        fpl.add(frames)
avg = {k: sum(v) / len(v) for k, v in per.items()}
px = W * H
alg_l0_read, alg_l0_write = px, px * 12 + W1 * H * 4
alg_l1_read, alg_l1_write = W1 * H * 4, W1 * H1 * 12
l0r, l0w = 2 * avg[("l0", "FETCH_SIZE")], avg[("l0", "WRITE_SIZE")]
l1r, l1w = 2 * avg[("l1", "FETCH_SIZE")], avg[("l1", "WRITE_SIZE")]
res = {
    "resolution": f"{W}x{H}",
    "frames_per_launch": sorted(fpl),
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tools/pmc_traffic.sh, batched launches",
    "per_frame_bytes": {"k_pyr_l0": {"read": l0r, "write": l0w, "alg_read": alg_l0_read, "alg_write": alg_l0_write},
                        "k_pyr_l1": {"read": l1r, "write": l1w, "alg_read": alg_l1_read, "alg_write": alg_l1_write}},
    "pass_hbm_bytes_per_frame": l0r + l0w + l1r + l1w,
    "pass_algorithmic_bytes_per_frame": px * 13 + W1 * H1 * 12,
    "raw_fetch_kib_per_frame": {"k_pyr_l0": avg[("l0", "FETCH_SIZE")] / 1024,
                                "k_pyr_l1": avg[("l1", "FETCH_SIZE")] / 1024},
    "note": "FETCH doubled for both kernels (gfx950 half-count; k_pyr_l0's interior tiles read 16 B/lane "
            "since v14, the guide's calibrated case, its edge tiles 4 B/lane); includes the sigma-3.6 row-pass round trip (hs written by "
            "k_pyr_l0, read by k_pyr_l1) that the pass-level algorithmic figure excludes; FETCH counts "
            "Infinity-Cache hits too",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
