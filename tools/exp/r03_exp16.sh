#!/bin/bash
# experiment: pyramid kernels writing {img, gx, gy}-interleaved banks (KLT_IL=1) that k_track7 reads directly
set -o pipefail
OUT=gpurun_out/exp16; mkdir -p $OUT
KLT_IL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "batched_frames and not generic" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do for v in 0 1; do
  KLT_IL=$v timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --frames 129 --reps 2 --chunk 64 --pyr-only > $OUT/p.json || exit 1
  p=$(python3 -c "import json; d=json.load(open('$OUT/p.json')); print('4K l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
  KLT_IL=$v timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2), 'wall', round(d['us_per_frame_wall'],2))")
  KLT_IL=$v timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 --overlap --table > $OUT/t.json || exit 1
  o=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('overlap wall', round(d['us_per_frame_wall'],2))")
  echo "il=$v | $p | $a | $o"
done; done
