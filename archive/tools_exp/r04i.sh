#!/bin/bash
# Round 4: {gx, gy, img} records -- the GPU suite, then the bench
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
Q="--no-cpu --api-frames 0 --no-fast"
timeout -k 10 300 python3 bench.py $Q > $OUT/full.json 2> $OUT/full.err || { tail -5 $OUT/full.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/full.json')); print(round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), d['roofline_4k']['kernels_us_per_frame'], round(d['roofline_4k']['frac'],3), round(d['roofline_4k']['pyramids_only']['frac'],3))"
