#!/bin/bash
# Round 4: host sort with team partition steps (csrc/host_sort.h) on the box's CPU
set -o pipefail
OUT=gpurun_out/r04s; mkdir -p $OUT
g++ -O3 -std=c++17 -pthread -Iklt-feature-tracker-acceleration-gpus_amd/csrc tools/hostcheck/sortbench.cpp -o $OUT/sortbench
timeout -k 10 300 $OUT/sortbench > $OUT/sortbench.txt && cat $OUT/sortbench.txt
