#!/bin/bash
# Round 5: a band call's build-ahead running only level 0 on the pyramid
# stream, level 1 on the tracking stream in the next call after its exchange
# and order (KLT_AHEAD_L1=1, default) against both levels ahead (0): shard
# GPU tests, then the config-4 8-rank simulation, two alternating rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05al}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "shard or band" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for al in 1 0; do
    KLT_AHEAD_L1=$al timeout -k 10 600 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds 1 8 --margins 64 --pass1-shared \
      > $OUT/sim_$al.log 2>&1 || { tail -20 $OUT/sim_$al.log; exit 1; }
    grep '^{"world"' $OUT/sim_$al.log | cut -c1-230 | sed "s/^/round $round ahead_l1=$al /" | tee -a $OUT/ab.txt
  done
done
