#!/bin/bash
# REPLACE with the AVX2 stop collection of the host partition (default on
# x86 hosts that have it) against the scalar loops (KLT_SORT_SCALAR=1), same
# build, alternating, three rounds, one process per run; then the host-only
# sortbench both ways.
set -o pipefail
OUT=gpurun_out/${1:-r06avx}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for mode in avx2 scalar; do
    if [ $mode = scalar ]; then S=1; else S=; fi
    KLT_SORT_SCALAR=$S timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT $mode >> $OUT/avx2_ab.jsonl 2> $OUT/avx_$mode.err || { tail -5 $OUT/avx_$mode.err; exit 1; }
    tail -1 $OUT/avx2_ab.jsonl | cut -c1-200
  done
done
g++ -O3 -pthread -Iklt-feature-tracker-acceleration-gpus_amd/csrc tools/hostcheck/sortbench.cpp -o $OUT/sortbench || exit 1
for mode in avx2 scalar; do
  if [ $mode = scalar ]; then S=1; else S=; fi
  echo "sortbench $mode"; KLT_SORT_SCALAR=$S timeout -k 10 120 $OUT/sortbench > $OUT/sortbench_$mode.txt && cat $OUT/sortbench_$mode.txt
done
