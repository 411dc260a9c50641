#!/bin/bash
# rocprofv3 kernel trace of the 4K / 20 000-feature tracked workload (BASELINE config 4 on one GPU, 64-frame launches)
set -o pipefail
OUT=gpurun_out/r03e_prof4k; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/microbench.py frames --width 3840 --height 2160 --features 20000 --frames 193 --reps 2 --chunk 64 > $OUT/mb.json 2> $OUT/mb.err || { tail -5 $OUT/mb.err; exit 1; }
python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 64 > $OUT/kernel_stats_isolated.txt || exit 1
grep -E "pyr|track" $OUT/kernel_stats_isolated.txt
