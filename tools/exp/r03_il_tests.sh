#!/bin/bash
# interleaved levels: the whole GPU suite, then the tracker / pyramid microbenchmarks
set -o pipefail
OUT=gpurun_out/il; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for r in 1 2; do
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2), 'wall', round(d['us_per_frame_wall'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/2500 l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))")
  echo "$a | $b"
done
