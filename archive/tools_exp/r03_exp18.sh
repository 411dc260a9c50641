#!/bin/bash
# same-box A/B: interleaved levels (this build) against the planar build of the previous commit (lib/var/head)
set -o pipefail
OUT=gpurun_out/exp18; mkdir -p $OUT
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3; do for v in head il; do
  if [ $v = il ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/$v/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/2500 l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))")
  echo "$v | $a | $b"
done; done
for v in head il; do
  if [ $v = il ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/$v/libklt_amd.so; fi
  timeout -k 10 300 python bench.py --no-cpu --api-frames 0 --no-fast --replace-frames 0 > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v bench', round(d['value']), {k: round(x,2) for k,x in d['kernels_us_per_frame'].items() if x}, 'roof', round(d['roofline']['frac'],3), '4k', round(d['roofline_4k']['frac'],3), {k: round(x,2) for k,x in d['roofline_4k']['kernels_us_per_frame'].items()})"
done
