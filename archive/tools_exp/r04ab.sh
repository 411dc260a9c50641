#!/bin/bash
# Round 4: config-4 8-rank simulation by margin (48 / 56 / 64 rows), 1001 frames
set -o pipefail
OUT=gpurun_out/r04ab; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/shard_sim.py --worlds 8 --frames 1001 --chunk 64 --margins 48 56 64 --lazy-flag > $OUT/s.log 2>&1 || { tail -5 $OUT/s.log; exit 1; }
grep -E '^\{"world' $OUT/s.log | cut -c1-300
