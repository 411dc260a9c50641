#!/bin/bash
# REPLACE at host/device thresholds of 49 152 (default), 32 768 and 24 576
# map points (KLT_AMD_SELECT_THRESHOLD; any value gives the same list), with
# the round-6 walk (spine, lopsided rule); alternating, three rounds, one box.
set -o pipefail
OUT=gpurun_out/${1:-r06thr}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for T in 49152 32768 24576; do
    KLT_AMD_SELECT_THRESHOLD=$T timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT thr$T >> $OUT/threshold_ab.jsonl 2> $OUT/thr_$T.err || { tail -5 $OUT/thr_$T.err; exit 1; }
    tail -1 $OUT/threshold_ab.jsonl | cut -c1-200
  done
done
