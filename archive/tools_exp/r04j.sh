#!/bin/bash
# Round 4: k_pyr_l0_rp (pairs across each stencil, {gx, gy, img} records by
# 12-byte stores) -- pyramid/tracker parity, then A/B against k_pyr_l0's
# interleaved path (KLT_L0_RP=0) on the pyramid pass and the bench, and the
# level-0 HBM writes of both
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_track.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do for v in 1 0; do
  KLT_L0_RP=$v timeout -k 10 120 python3 tools/microbench.py frames --pyr-only --width 3840 --height 2160 --chunk 64 --frames 129 --reps 3 > $OUT/p4k_$v_$r.json 2>&1 || { tail -5 $OUT/p4k_$v_$r.json; exit 1; }
  echo "rp=$v 4k $(python3 -c "import json; d=json.loads(open('$OUT/p4k_$v_$r.json').read().splitlines()[-1]); print(round(d['l0_us_per_frame'],2), round(d['l1_us_per_frame'],2))")"
  KLT_L0_RP=$v timeout -k 10 120 python3 tools/microbench.py frames --pyr-only --chunk 64 --frames 129 --reps 3 > $OUT/p1080_$v_$r.json 2>&1 || { tail -5 $OUT/p1080_$v_$r.json; exit 1; }
  echo "rp=$v 1080 $(python3 -c "import json; d=json.loads(open('$OUT/p1080_$v_$r.json').read().splitlines()[-1]); print(round(d['l0_us_per_frame'],2), round(d['l1_us_per_frame'],2))")"
done; done
for v in 1 0; do
  KLT_L0_RP=$v timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -5 $OUT/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('rp=$v', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), {k: round(v,2) for k,v in d['roofline_4k']['kernels_us_per_frame'].items()}, round(d['roofline_4k']['frac'],3), round(d['roofline_4k']['pyramids_only']['frac'],3))"
done
for v in 1 0; do
  KLT_L0_RP=$v timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/wr$v -o run -- python3 tools/microbench.py frames --frames 129 --reps 1 --chunk 64 --pyr-only --width 3840 --height 2160 > $OUT/wr$v.log 2>&1 || { tail -5 $OUT/wr$v.log; exit 1; }
  python3 tools/pmc_summary.py $(find $OUT/wr$v -name "*counter_collection.csv") | grep -i "k_pyr_l0" | head -3
done
