#!/bin/bash
# config-4 rank simulation, 1000 frames: chunk/margin A/B, alternating, same box
set -o pipefail
OUT=gpurun_out/r03l; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for rep in 1 2; do
for c in "--worlds 1 8 --chunk 64 --margins 64" "--worlds 1 8 --chunk 128 --margins 80" "--worlds 8 --chunk 192 --margins 96"; do
  i=$((i+1))
  timeout -k 10 500 python tools/shard_sim.py --frames 1001 $c --lazy-flag --pass1-shared > $OUT/s$i.log 2>&1 || { tail -5 $OUT/s$i.log; exit 1; }
  echo "$c"; grep '^{"world' $OUT/s$i.log | cut -c1-200
done
done
