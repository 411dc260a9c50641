#!/bin/bash
# interleaved levels: shard and pyramid tests, per-rank breakdown at 1/2/4/8 ranks (serial and build-ahead)
set -o pipefail
OUT=gpurun_out/r03e_shard; mkdir -p $OUT
true
true
for v in "--lazy-flag" "--lazy-flag --no-ahead"; do
  timeout -k 10 500 python tools/shard_sim.py --worlds 1 2 4 8 --frames 257 --chunk 64 --margins 64 $v > $OUT/s.log 2>&1 || { tail -5 $OUT/s.log; exit 1; }
  python3 - $OUT/s.log "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
out = []
for r in d["runs"]:
    q = max(r["per_rank_us_per_frame"], key=lambda q: q["wall"])
    k = q["replay_kernels"]
    out.append("w%d max %.2f (l0 %.2f l1 %.2f trk %.2f) x%.2f redo %d digest %d" % (r["world"], q["wall"], k["k_pyr_l0"],
               k["k_pyr_l1"], k["k_track"], r["projected_speedup"] or 1, r["chunks_redone_full_frame"], r["state_digest"]))
print(sys.argv[2], " | ".join(out))
PY
done
