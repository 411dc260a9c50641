#!/bin/bash
# HBM traffic of the tracker (k_track7) at 1080p/5000 in 64-frame launches: FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
OUT=gpurun_out/exp14; mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python tools/microbench.py frames --frames 129 --reps 1 --chunk 64 --table > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") | tee $OUT/summary.txt
tail -1 $OUT/FETCH_SIZE.log
