#!/bin/bash
# band calls in sub-chunks (KLT_BAND_SUB: build/track pipeline inside one exchange chunk) with nontemporal or
# cache-allocating level-0 stores (variant plain): do MALL-resident band pyramids shorten the tracker's chain?
set -o pipefail
OUT=gpurun_out/exp12; mkdir -p $OUT
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for lib in default plain; do for sub in 0 8 16; do
  if [ $lib = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/$lib/libklt_amd.so; fi
  KLT_BAND_SUB=$sub timeout -k 10 400 python tools/shard_sim.py --worlds 1 8 --frames 257 --chunk 64 --margins 64 --lazy-flag > $OUT/s.log 2>&1 || { tail -5 $OUT/s.log; exit 1; }
  python3 - $OUT/s.log "$lib sub=$sub" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
out = []
for r in d["runs"]:
    q = max(r["per_rank_us_per_frame"], key=lambda q: q["wall"])
    k = q["replay_kernels"]
    out.append("w%d max %.2f (l0 %.2f l1 %.2f trk %.2f) x%.2f redo %d" % (r["world"], q["wall"], k["k_pyr_l0"], k["k_pyr_l1"],
               k["k_track"], r["projected_speedup"] or 1, r["chunks_redone_full_frame"]))
print(sys.argv[2], " | ".join(out))
PY
done; done
