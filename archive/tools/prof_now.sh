#!/bin/bash
# per-wave phase clocks of the tracker (instrumented build, make -C csrc prof)
OUT=gpurun_out/${1:-prof}; mkdir -p $OUT
export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/prof/libklt_amd.so
run() { timeout -k 10 300 python tools/microbench.py "$@" > $OUT/last.json || exit 1; echo "$*" | tee -a $OUT/sweep.txt; python3 -c "
import json; d=json.load(open('$OUT/last.json'))
for k in ('prof_cycles_per_wave_frame','prof_clock64_ghz','prof_wave_life_us','prof_start_us_pct','prof_end_us_pct','us_per_frame_wall'):
    print('  ', k, d.get(k))" | tee -a $OUT/sweep.txt; }
run frames --frames 129 --reps 2 --chunk 64 --prof
run frames --frames 129 --reps 2 --chunk 64 --prof --features 2500
run frames --frames 129 --reps 2 --chunk 64 --prof --features 1000
