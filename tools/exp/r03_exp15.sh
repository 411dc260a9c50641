#!/bin/bash
# experiment: tracker gathers from {img, gx, gy}-interleaved levels (KLT_AOS=1, copies made before each launch)
set -o pipefail
OUT=gpurun_out/exp15; mkdir -p $OUT
KLT_AOS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "(batched or tuning or overlap or sequence or long) and not generic and not fast and not nondefault" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do for v in 0 1; do
  KLT_AOS=$v timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print(round(d['track_us_per_frame'],2))")
  KLT_AOS=$v timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print(round(d['track_us_per_frame'],2))")
  echo "aos=$v 1080p/5000 $a  4K/2500 $b"
done; done
