#!/bin/bash
# Round 4: k_pyr_l0's interleaved path with (tx, ty) / (gx, gy) pairs and
# 12-byte record stores (this build) against HEAD (lib/var/head): parity,
# pyramid-pass A/B alternating, bench, level-0 writes, PMC
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
export TMPDIR=/tmp
HEADLIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/head/libklt_amd.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_track.py tests/test_gpu_long.py tests/test_gpu_select.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() { # tag lib args...
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = head ]; then export KLT_AMD_LIB=$HEADLIB; else unset KLT_AMD_LIB; fi
  timeout -k 10 120 python3 tools/microbench.py frames --pyr-only --chunk 64 --frames 129 --reps 3 "$@" > $OUT/$tag.json 2>&1 || { tail -5 $OUT/$tag.json; exit 1; }
  echo "$tag $(python3 -c "import json; d=json.loads(open('$OUT/$tag.json').read().splitlines()[-1]); print(round(d['l0_us_per_frame'],2), round(d['l1_us_per_frame'],2))")"
}
for r in 1 2; do for v in new head; do
  run p4k_${v}_$r $v --width 3840 --height 2160
  run p1080_${v}_$r $v
done; done
for v in new head; do
  if [ "$v" = head ]; then export KLT_AMD_LIB=$HEADLIB; else unset KLT_AMD_LIB; fi
  timeout -k 10 300 python3 bench.py --no-cpu --api-frames 0 --no-fast > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -5 $OUT/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), {k: round(v,2) for k,v in d['roofline_4k']['kernels_us_per_frame'].items()}, round(d['roofline_4k']['frac'],3), round(d['roofline_4k']['pyramids_only']['frac'],3))"
done
unset KLT_AMD_LIB
bash tools/pmc_traffic.sh r04l/traffic4k --width 3840 --height 2160 > $OUT/traffic4k.log 2>&1 || { tail -5 $OUT/traffic4k.log; exit 1; }
grep -A3 "k_pyr_l0\|k_pyr_l1" $OUT/traffic4k.log | head -12
bash tools/pmc_pyr.sh r04l/pmcpyr > $OUT/pmcpyr.log 2>&1 || { tail -5 $OUT/pmcpyr.log; exit 1; }
grep -A22 "k_pyr_l0" gpurun_out/r04l/pmcpyr/summary.txt | grep -E "k_pyr|VALU|LDS|WAVE_CYCLES|GRBM|WAIT_ANY" | head -12
