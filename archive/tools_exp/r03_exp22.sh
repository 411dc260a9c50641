#!/bin/bash
# rocprof kernel durations: pyramids built between tracker launches vs back to back
set -o pipefail
OUT=gpurun_out/exp22; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in track pyr; do
  f=""; [ $m = pyr ] && f="--pyr-only"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/$m -o run --output-format csv -- python3 tools/microbench.py frames --frames 129 --reps 2 --chunk 64 $f > $OUT/$m.json 2> $OUT/$m.err || exit 1
done
for m in track pyr; do echo "== $m"; f=$(ls $OUT/$m/*/run_kernel_stats.csv 2>/dev/null || ls $OUT/$m/run_kernel_stats.csv); cut -d, -f1-8 $f | head -6; done
