#!/bin/bash
# Same-box A/B of library builds on the bench workload (no CPU leg, no 4K line):
# usage (via gpurun): bash archive/tools/bench_ab.sh <tag> <var> [rounds]
set -o pipefail
OUT=gpurun_out/${1:-ab}; VAR=$2; R=${3:-2}; mkdir -p $OUT
for r in $(seq $R); do
  for v in default $VAR; do
    if [ "$v" = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
    timeout -k 10 300 python bench.py --no-cpu --no-4k > $OUT/last.json || exit 1
    echo "$v" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); k=d['kernels_us_per_frame']; print(round(d['value']), 'frames/s', 'l0', round(k['k_pyr_l0'],2), 'l1', round(k['k_pyr_l1'],2), 'track', round(k['k_track'],2))") | tee -a $OUT/sweep.txt
  done
done
