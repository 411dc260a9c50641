#!/bin/bash
# Round 4: k_pyr_l0's sigma-3.6 rows pass (D3) reading its tap pairs with
# ds_read2_b32 (variant d3on) vs 16-byte reads + moves (default build):
# pyramid parity, then the full bench A/B (1080p and 4K legs)
set -o pipefail
OUT=gpurun_out/r04ad; mkdir -p $OUT
export TMPDIR=/tmp
KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/d3on/libklt_amd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_select.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
V=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/d3on/libklt_amd.so
for w in new old new old; do
  L=""; [ $w = new ] && L="KLT_AMD_LIB=$V"
  env $L timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/b$w.json 2> $OUT/b$w.err || { tail -5 $OUT/b$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$w.json')); r=d['roofline_4k']; print('$w', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), '4k', {k: round(v,2) for k,v in r['kernels_us_per_frame'].items() if v}, round(r['frac'],3), round(r['pyramids_only']['frac'],3))"
done
