#!/bin/bash
# HBM traffic of the pyramid pass (separate FETCH_SIZE / WRITE_SIZE passes,
# kernel-trace only), bench workload: 1080p, batched chunk 64, pyramids only.
# usage: bash tools/pmc_traffic.sh <tag> [microbench args]
set -o pipefail
TAG=${1:-traffic}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="frames --frames 129 --reps 1 --chunk 64 --pyr-only $*"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python tools/microbench.py $ARGS > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") | tee $OUT/summary.txt
