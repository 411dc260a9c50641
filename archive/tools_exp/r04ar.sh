#!/bin/bash
# Round 4: k_pyr_l0 edge tiles with the interior's 16-byte chunk loads (rows
# and crossing dwords clamped) and whole-record / whole-slab-row stores
# (default build) vs per-dword loads and per-plane stores (variant edge0,
# KLT_L0_EDGE=0): pyramid/selection/tracker parity on the new build, the
# workgroup phase profile of both (1080p), then the bench A/B alternating
set -o pipefail
OUT=gpurun_out/r04ar; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_select.py tests/test_gpu_track.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in pyrprof pyrprof_edge0; do
  echo "== $v"
  timeout -k 10 120 tools/hipbench/$v $OUT/rec_$v.bin 1920 1080 1 || exit 1
  python3 tools/exp/pyrprof_an.py $OUT/rec_$v.bin || exit 1
done
V=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/edge0/libklt_amd.so
for w in new old new old new old; do
  L=""; [ $w = old ] && L="KLT_AMD_LIB=$V"
  env $L timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/b$w.json 2> $OUT/b$w.err || { tail -5 $OUT/b$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$w.json')); r=d['roofline_4k']; print('$w', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), '4k', {k: round(v,2) for k,v in r['kernels_us_per_frame'].items() if v}, round(r['frac'],3), round(r['pyramids_only']['frac'],3))"
done
