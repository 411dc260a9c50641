#!/bin/bash
# Round 4: 64-row level-0 tiles for whole frames (KLT_L0_WIDE=1, default) vs
# 32-row tiles: pyramid/tracker parity, then the bench (1080p and 4K legs) A/B
set -o pipefail
OUT=gpurun_out/r04x; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for w in 1 0 1 0; do
  KLT_L0_WIDE=$w timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/b$w.json 2> $OUT/b$w.err || { tail -5 $OUT/b$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$w.json')); r=d['roofline_4k']; print('wide=$w', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), '4k', {k: round(v,2) for k,v in r['kernels_us_per_frame'].items() if v}, round(r['frac'],3), round(r['pyramids_only']['frac'],3))"
done
