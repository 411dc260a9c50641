#!/bin/bash
# REPLACE with and without the lopsided-split rule (a right part much longer
# than its left part stays unsorted and is split when reached, instead of
# sorted whole in the background): the default build against
# lib/var/nolop (make variant NAME=nolop DEFS=-DKLT_SEL_LOPSIDED=0),
# alternating, three rounds, one process per run.
set -o pipefail
OUT=gpurun_out/${1:-r06lop}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for lib in default nolop; do
    if [ $lib = default ]; then L=""; else L=klt-feature-tracker-acceleration-gpus_amd/lib/var/nolop/libklt_amd.so; fi
    KLT_AMD_LIB=$L timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT $lib >> $OUT/lopsided_ab.jsonl 2> $OUT/lop_$lib.err || { tail -5 $OUT/lop_$lib.err; exit 1; }
    tail -1 $OUT/lopsided_ab.jsonl | cut -c1-200
  done
done
