#!/bin/bash
# config-4 rank simulation, 1000 frames: 64-frame chunks against 128 (margins for 38 px of motion)
set -o pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for c in "--chunk 64 --margins 64" "--chunk 128 --margins 80 96"; do
  i=$((i+1))
  timeout -k 10 500 python tools/shard_sim.py --worlds 1 8 --frames 1001 $c --lazy-flag --pass1-shared > $OUT/s$i.log 2>&1 || { tail -5 $OUT/s$i.log; exit 1; }
  grep '^{"world' $OUT/s$i.log
done
