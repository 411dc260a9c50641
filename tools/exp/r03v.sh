#!/bin/bash
# final round-3 cycle: GPU tests, bench (driver-shaped and default), rocprof, config-4 rank simulation at 1000 frames
set -o pipefail
bash tools/r03_cycle.sh r03v tests prof || exit 1
OUT=gpurun_out/r03v
timeout -k 10 600 python tools/shard_sim.py --worlds 1 8 --frames 1001 --chunk 64 --margins 64 --lazy-flag --pass1-shared > $OUT/s1000.log 2>&1 || { tail -5 $OUT/s1000.log; exit 1; }
grep '^{"world' $OUT/s1000.log
