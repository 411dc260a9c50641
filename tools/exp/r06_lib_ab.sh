#!/bin/bash
# REPLACE with the default build against an experiment build
# (lib/var/<name>/libklt_amd.so: `make variant`, or the previous commit's
# sources built with `make OUT=<repo lib> variant NAME=prev`), alternating,
# three rounds, one process per run.  usage: r06_lib_ab.sh <tag> <name>
set -o pipefail
OUT=gpurun_out/${1:-r06lib}; V=${2:-prev}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for lib in default $V; do
    if [ $lib = default ]; then L=""; else L=klt-feature-tracker-acceleration-gpus_amd/lib/var/$V/libklt_amd.so; fi
    KLT_AMD_LIB=$L timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT $lib >> $OUT/lib_ab.jsonl 2> $OUT/lib_$lib.err || { tail -5 $OUT/lib_$lib.err; exit 1; }
    tail -1 $OUT/lib_ab.jsonl | cut -c1-200
  done
done
