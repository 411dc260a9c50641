#!/bin/bash
# k_track7 next-frame prefetch wave: parity, then tracker time with / without it
set -o pipefail
OUT=gpurun_out/exp23; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do for m in pf nopf; do
  f=""; [ $m = nopf ] && f="--no-pf"
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 $f > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p/5000 trk', round(d['track_us_per_frame'],2), 'l0', round(d['l0_us_per_frame'],2), 'wall', round(d['us_per_frame_wall'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 $f > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/2500 trk', round(d['track_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 20000 --frames 129 --reps 2 --chunk 64 $f > $OUT/t.json || exit 1
  c=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/20000 trk', round(d['track_us_per_frame'],2))")
  echo "$m | $a | $b | $c"
done; done
