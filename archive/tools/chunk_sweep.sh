#!/bin/bash
# tracker/pipeline time per frame against the launch length (frames per chunk)
set -o pipefail
mkdir -p gpurun_out
for cfg in "--width 1920 --height 1080 --features 5000" "--width 3840 --height 2160 --features 2500"; do
  for c in 32 64 128; do
    timeout -k 5 180 python tools/microbench.py frames --frames 257 --reps 2 --chunk $c --table $cfg > gpurun_out/chk.json || exit 1
    echo "$cfg chunk $c $(python3 -c "import json; d=json.load(open('gpurun_out/chk.json')); print('track', round(d['track_us_per_frame'],2), 'l0', round(d['l0_us_per_frame'],2), 'fps', round(d['fps_wall']))")"
  done
done
