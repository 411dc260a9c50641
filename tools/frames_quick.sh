#!/bin/bash
OUT=gpurun_out/${1:-fq}; mkdir -p $OUT; shift
for args in "$@"; do
  timeout -k 10 300 python tools/microbench.py frames --reps 3 $args > $OUT/last.json || exit 1
  echo "$args" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['us_per_frame_wall'],2), 'l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))") | tee -a $OUT/sweep.txt
done
