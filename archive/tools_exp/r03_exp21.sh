#!/bin/bash
# same box: pyramid kernel times with and without tracking in the same batched launches
set -o pipefail
OUT=gpurun_out/exp21; mkdir -p $OUT
for r in 1 2 3; do for m in track pyr; do
  f=""; [ $m = pyr ] && f="--pyr-only"
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 $f > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 $f > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
  echo "$m | $a | $b"
done; done
