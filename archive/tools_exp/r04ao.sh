#!/bin/bash
# Round 4: k_pyr_l0's sigma-3.6 rows pass (D3) as lagged output pairs (the
# second output of a pair three taps behind, so even steps read aligned
# register pairs; default build) vs output pairs four apart assembled by moves
# (variant d3old, KLT_L0_D3_LAG=0): pyramid/selection/tracker parity on the new
# build, then the bench A/B alternating processes (1080p and 4K legs)
set -o pipefail
OUT=gpurun_out/r04ao; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_select.py tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
V=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/d3old/libklt_amd.so
for w in new old new old new old; do
  L=""; [ $w = old ] && L="KLT_AMD_LIB=$V"
  env $L timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/b$w.json 2> $OUT/b$w.err || { tail -5 $OUT/b$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$w.json')); r=d['roofline_4k']; print('$w', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), '4k', {k: round(v,2) for k,v in r['kernels_us_per_frame'].items() if v}, round(r['frac'],3), round(r['pyramids_only']['frac'],3))"
done
