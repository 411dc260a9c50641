#!/bin/bash
OUT=gpurun_out/${1:-misc}; mkdir -p $OUT
run() { timeout -k 10 300 python tools/microbench.py "$@" > $OUT/last.json || exit 1; echo "$*" $(cat $OUT/last.json) | tee -a $OUT/sweep.txt; }
run api --frames 60
run frames --frames 129 --reps 3 --chunk 16 --pyr-only
run frames --frames 129 --reps 3 --chunk 64 --pyr-only
run frames --frames 65 --reps 3 --chunk 16 --pyr-only --width 3840 --height 2160
run frames --frames 65 --reps 3 --chunk 16 --width 3840 --height 2160 --features 20000
run pyr --width 3840 --height 2160 --reps 100
