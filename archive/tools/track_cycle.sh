#!/bin/bash
# tracker microbenchmark sweep: bash archive/tools/track_cycle.sh [tag] [extra microbench args]
OUT=gpurun_out/${1:-trk}; mkdir -p $OUT
shift || true
for args in "--features 5000" "--features 5000 --reduction fast" "--features 500" \
            "--width 3840 --height 2160 --features 20000"; do
  timeout -k 10 300 python tools/microbench.py track $args "$@" > $OUT/last.json || exit 1
  python3 -c "import json; d=json.load(open('$OUT/last.json')); print('$args', round(d['k_track_us'],2))" | tee -a $OUT/sweep.txt
done
