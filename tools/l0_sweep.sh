#!/bin/bash
# level-0 kernel comparison (pyramid-only batched frames): bash tools/l0_sweep.sh tag "opts1" "opts2" ...
OUT=gpurun_out/${1:-l0s}; shift; mkdir -p $OUT
for v in "$@"; do
  for args in "--frames 65 --chunk 32" "--width 3840 --height 2160 --frames 65 --chunk 32"; do
    timeout -k 10 300 python tools/microbench.py frames --reps 3 --pyr-only --features 8 $args $v > $OUT/last.json || exit 1
    echo "[$v] $args" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['us_per_frame_wall'],2), 'l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))") | tee -a $OUT/sweep.txt
  done
done
