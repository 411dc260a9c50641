#!/bin/bash
# exp32 timing again with the order alternating (4K/20k and 1080p/5000, l0 / l1 per frame)
set -o pipefail
OUT=gpurun_out/exp33; mkdir -p $OUT
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="new h63"; else order="h63 new"; fi
  for m in $order; do
    if [ $m = new ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/h63/libklt_amd.so; fi
    timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 20000 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
    b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/20k l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
    timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
    a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
    echo "$m | $b | $a"
  done
done
