#!/bin/bash
# persistent level-0 kernel (KLT_PYR_L0P=<workgroups per CU>) vs k_pyr_l0: parity, 4K pass, 1080p bench
set -o pipefail
OUT=gpurun_out/exp3; mkdir -p $OUT
KLT_PYR_L0P=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/l0p_tests.log 2>&1 || { tail -20 $OUT/l0p_tests.log; exit 1; }
tail -1 $OUT/l0p_tests.log
for r in 1 2; do for v in 0 4 3 2; do
  KLT_PYR_L0P=$v timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --frames 129 --reps 2 --chunk 64 --pyr-only > $OUT/pyr_$v.json || exit 1
  echo l0p=$v $(python3 -c "import json; d=json.load(open('$OUT/pyr_$v.json')); print('l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
done; done
for v in 0 4; do
  KLT_PYR_L0P=$v timeout -k 10 300 python bench.py --no-cpu --api-frames 0 --no-fast --replace-frames 0 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -5 $OUT/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('l0p=$v', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, 'roof', round(d['roofline']['frac'],3), '4k', round(d['roofline_4k']['frac'],3), d['roofline_4k']['kernels_us_per_frame'])"
done
