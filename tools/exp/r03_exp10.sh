#!/bin/bash
# k_track7 ordered-sum read batches: 7 (default) vs 13 (all in flight) vs 4
set -o pipefail
OUT=gpurun_out/exp10; mkdir -p $OUT
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2; do for v in default b13 b4; do
  if [ $v = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/$v/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print(round(d['track_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print(round(d['track_us_per_frame'],2))")
  echo "$v 1080p/5000 $a  4K/2500 $b"
done; done
