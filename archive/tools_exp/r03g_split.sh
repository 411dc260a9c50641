#!/bin/bash
# CU split (klt_hip_set_cu_split) and chunk length at 8 simulated ranks, 4K/20k,
# build-ahead schedule; world 1 once as the base
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
export TMPDIR=/tmp
summ() {
python3 - $1 "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
out = []
for r in d["runs"]:
    q = max(r["per_rank_us_per_frame"], key=lambda q: q["wall"])
    k = q["replay_kernels"]
    walls = sorted(round(p["wall"], 2) for p in r["per_rank_us_per_frame"])
    out.append("w%d max %.2f (l0 %.2f l1 %.2f trk %.2f) redo %d digest %d walls %s" % (r["world"], q["wall"], k["k_pyr_l0"],
               k["k_pyr_l1"], k["k_track"], r["chunks_redone_full_frame"], r["state_digest"], walls))
print(sys.argv[2], " | ".join(out), flush=True)
PY
}
i=0
for c in "--worlds 1 8 --chunk 64 --margins 64" "--worlds 8 --chunk 64 --margins 64 --cu-split 8" \
         "--worlds 8 --chunk 64 --margins 64 --cu-split 12" "--worlds 8 --chunk 64 --margins 64 --cu-split 16" \
         "--worlds 8 --chunk 64 --margins 64 --cu-split 20" "--worlds 8 --chunk 128 --margins 96" \
         "--worlds 8 --chunk 64 --margins 64 --cu-split 12 --no-ahead"; do
  i=$((i+1))
  timeout -k 10 400 python tools/shard_sim.py --frames 257 $c --lazy-flag > $OUT/s$i.log 2>&1 || { tail -5 $OUT/s$i.log; exit 1; }
  summ $OUT/s$i.log "$c"
done
