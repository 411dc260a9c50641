#!/bin/bash
# interleaved level 1 written through an LDS-staged tile (this build) vs direct triple-strided stores (variant l1nt)
set -o pipefail
OUT=gpurun_out/exp20; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3; do for v in staged l1nt; do
  if [ $v = staged ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/$v/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 --pyr-only > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --frames 129 --reps 2 --chunk 64 --pyr-only > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
  echo "$v | $a | $b"
done; done
