#!/bin/bash
# Round 5: k_pyr_l0's phase E on interior tiles storing each pair of rows as
# soon as it is summed (KLT_L0_ESTREAM=1, default build; es2: =2, with a
# scheduling barrier after each pair) against all eight rows summed first
# and stored at the end (lib/var/es0, =0): pyramid and tracker parity first,
# then l0 / l1 per frame (tools/microbench.py frames, 64-frame chunks:
# 1080p/5000 tracked, 4K/20 000 tracked, 4K pyramids only), three
# alternating rounds, then the light 1080p bench with each build.
set -o pipefail
OUT=gpurun_out/${1:-r05es}; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "pyramid or track or long or shard or select" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $OUT/tests.log
for round in 1 2 3; do
  for lib in default es0 es2; do
    for shape in "--width 1920 --height 1080 --features 5000" "--width 3840 --height 2160 --features 20000" \
                 "--width 3840 --height 2160 --features 20000 --pyr-only"; do
      if [ $lib = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$lib/libklt_amd.so; fi
      timeout -k 10 300 python3 tools/microbench.py frames $shape --chunk 64 --frames 129 --reps 3 --table > $OUT/mb.json 2>> $OUT/mb.err || { tail -5 $OUT/mb.err; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open('$OUT/mb.json').read().strip().splitlines()[-1])
k={kk:round(v,3) for kk,v in d.items() if kk in ('l0_us_per_frame', 'l1_us_per_frame', 'track_us_per_frame')}
print('round $round', '$lib', '$shape', k)" | tee -a $OUT/ab.txt
    done
  done
done
unset KLT_AMD_LIB
BENCH_ROUNDS=${BENCH_ROUNDS-1 2}
LIGHT="--no-cpu --no-4k --api-frames 0 --replace-frames 0 --no-fast"
for round in $BENCH_ROUNDS; do
  for lib in default es0 es2; do
    if [ $lib = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$lib/libklt_amd.so; fi
    timeout -k 10 300 python3 bench.py $LIGHT > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('bench round $round $lib', round(d['value']), 'us/frame', round(1e3*d['ms_per_step'],2), 'roof', round(d['roofline']['frac'],4),
      'kernels/frame', {k: round(x, 3) for k, x in d['kernels_us_per_frame'].items()})" | tee -a $OUT/ab.txt
  done
done
