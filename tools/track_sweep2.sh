#!/bin/bash
OUT=gpurun_out/${1:-trks}; mkdir -p $OUT
for args in "--features 64 --lost" "--features 5000 --lost" "--features 64" "--features 64 --max-it 1" "--features 1" "--features 1 --max-it 1"; do
  timeout -k 10 300 python tools/microbench.py track $args > $OUT/last.json || exit 1
  python3 -c "import json; d=json.load(open('$OUT/last.json')); print('$args', round(d['k_track_us'],2), d['status_hist'])" | tee -a $OUT/sweep.txt
done
