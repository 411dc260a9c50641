#!/bin/bash
# Round 4: config-4 rank simulation (1 and 8 ranks, 1001 frames, 64-frame
# chunks, margin 64) with the round-4 build
set -o pipefail
OUT=gpurun_out/r04z; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/shard_sim.py --worlds 1 8 --frames 1001 --chunk 64 --margins 64 --lazy-flag > $OUT/s1000.log 2>&1 || { tail -5 $OUT/s1000.log; exit 1; }
grep -E '^\{"world|projected|speedup' $OUT/s1000.log | cut -c1-400
