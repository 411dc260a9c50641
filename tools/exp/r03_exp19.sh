#!/bin/bash
# interleaved level 1: plain (default) vs nontemporal stores (variant l1nt)
set -o pipefail
OUT=gpurun_out/exp19; mkdir -p $OUT
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3; do for v in il l1nt; do
  if [ $v = il ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/$v/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --frames 129 --reps 2 --chunk 64 --pyr-only > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
  echo "$v | $a | $b"
done; done
