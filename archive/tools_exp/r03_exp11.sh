#!/bin/bash
# config-4 rank simulation, per-rank breakdown: build-ahead (overlapped) and serial, with per-kernel events
set -o pipefail
OUT=gpurun_out/exp11; mkdir -p $OUT
for v in "--lazy-flag" "--lazy-flag --no-ahead"; do
  tag=$(echo "$v" | tr -d ' -')
  timeout -k 10 500 python tools/shard_sim.py --worlds 1 2 4 8 --frames 257 --chunk 64 --margins 64 $v > $OUT/shard_$tag.log 2>&1 || { tail -5 $OUT/shard_$tag.log; exit 1; }
  echo "== $v"; grep '^{"world' $OUT/shard_$tag.log
  python3 - $OUT/shard_$tag.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
for r in d["runs"]:
    for q in r["per_rank_us_per_frame"]:
        k = q["replay_kernels"]
        print("  world", r["world"], "rank", q["rank"], q["band_rows"], "wall %.2f" % q["wall"],
              "l0 %.2f l1 %.2f trk %.2f" % (k["k_pyr_l0"], k["k_pyr_l1"], k["k_track"]))
PY
done
