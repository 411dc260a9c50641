#!/bin/bash
# config-4 rank simulation at 8 ranks: per-chunk host flag read vs lazy (speculative) read, build-ahead vs none
set -o pipefail
OUT=gpurun_out/exp4; mkdir -p $OUT
for v in "" "--lazy-flag" "--no-ahead" "--lazy-flag --no-ahead"; do
  timeout -k 10 500 python tools/shard_sim.py --worlds 1 8 --frames 257 --chunk 64 --margins 64 $v > $OUT/shard.log 2>&1 || { tail -5 $OUT/shard.log; exit 1; }
  echo "== $v"; grep '^{"world' $OUT/shard.log
  python3 - $OUT/shard.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
for r in d["runs"]:
    if r["world"] == 8:
        print("   walls", [round(q["wall"], 2) for q in r["per_rank_us_per_frame"]])
PY
done
