#!/bin/bash
# How much of an all-gather's latency the config-4 schedule hides: the 8-rank
# projection with a device stall of S us in the all-gather's place on every
# rank's tracking stream (tools/shard_sim.py --exchange-in-stream-us S),
# S = 0 (the copy alone) .. 60, one box.
set -o pipefail
OUT=gpurun_out/${1:-r06es}; mkdir -p $OUT
export TMPDIR=/tmp
for S in ${STALLS:-0.001 20 40 60}; do
  timeout -k 10 600 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds 8 --margins 64 --pass1-shared \
    --exchange-in-stream-us $S > $OUT/exch_S$S.log 2>&1 || { tail -20 $OUT/exch_S$S.log; exit 1; }
  echo "stall $S us: $(grep '^{"world"' $OUT/exch_S$S.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["us_per_frame_synced"],3), "us/frame synced")')"
done
