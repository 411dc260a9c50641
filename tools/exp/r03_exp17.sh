#!/bin/bash
# interleaved levels: tracker speed by bank allocation (one arena / a block per level / contiguous arena)
set -o pipefail
OUT=gpurun_out/exp17; mkdir -p $OUT
for r in 1 2; do for v in "X=0" "KLT_BANK_ARENA=0" "KLT_BANK_CONTIG=1"; do
  env $v timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))")
  env $v timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/2500 l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))")
  echo "$v | $a | $b"
done; done
