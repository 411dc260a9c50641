#!/bin/bash
# Round 4: 48-row level-0 tiles for whole frames (KLT_L0_WIDE_ROWS=48: 384
# threads, 47.5 KB LDS, three workgroups per CU) against 64-row (default,
# 61.6 KB, two per CU) at 4K, and at 1080p against the 32-row default
# (KLT_L0_WIDE_MIN=1000): pyramid/tracker parity with every whole frame on
# 48-row tiles (KLT_L0_WIDE_MIN=0), then the bench A/B alternating
set -o pipefail
OUT=gpurun_out/r04av; mkdir -p $OUT
export TMPDIR=/tmp
KLT_L0_WIDE_ROWS=48 KLT_L0_WIDE_MIN=0 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_track.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests48.log 2>&1 || { tail -30 $OUT/tests48.log; exit 1; }
tail -1 $OUT/tests48.log
for cfg in def r48 r48all def r48 r48all; do
  case $cfg in def) E="";; r48) E="KLT_L0_WIDE_ROWS=48";; r48all) E="KLT_L0_WIDE_ROWS=48 KLT_L0_WIDE_MIN=1000";; esac
  env $E timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); r=d['roofline_4k']; print('$cfg', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), '4k', {k: round(v,2) for k,v in r['kernels_us_per_frame'].items() if v}, round(r['frac'],3), round(r['pyramids_only']['frac'],3))"
done
