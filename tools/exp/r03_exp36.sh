#!/bin/bash
# level-1 hs loads: one column group per thread, constant row stride, unclamped interior tiles (this build) vs ad0e0ab (variant ad0)
set -o pipefail
OUT=gpurun_out/exp36; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_pyramid.py tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="new ad0"; else order="ad0 new"; fi
  for m in $order; do
    if [ $m = new ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/ad0/libklt_amd.so; fi
    timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 20000 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
    b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/20k l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
    timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
    a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
    echo "$m | $b | $a"
  done
done
