#!/bin/bash
set -o pipefail
OUT=gpurun_out/exp2; mkdir -p $OUT gpurun_out/pyrprof
timeout -k 10 120 tools/hipbench/pyrprof gpurun_out/pyrprof/rec.bin > $OUT/pyrprof.txt 2>&1 || { cat $OUT/pyrprof.txt; exit 1; }
cat $OUT/pyrprof.txt
python3 tools/exp/pyrprof_an.py gpurun_out/pyrprof/rec.bin | tee $OUT/pyrprof_an.txt
rm -f gpurun_out/pyrprof/rec.bin
