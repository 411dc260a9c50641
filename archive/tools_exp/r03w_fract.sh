#!/bin/bash
# k_track7 v_fract corners, packed products A/B: tracker us/frame at three loads, bench value, tracker tests
set -o pipefail
OUT=gpurun_out/r03w; mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for rep in 1 2; do
for lib in libklt_amd.so var/old/libklt_amd.so; do
  for cfg in "--features 5000" "--width 3840 --height 2160 --features 2500" "--width 3840 --height 2160 --features 20000"; do
    KLT_AMD_LIB=$L/$lib timeout -k 5 200 python tools/microbench.py frames $cfg --frames 193 --reps 3 --chunk 64 > $OUT/m.json 2> $OUT/m.err || { tail -5 $OUT/m.err; exit 1; }
    echo "$lib $cfg" $(python3 -c "import json; d=json.load(open('$OUT/m.json')); print('track', round(d['track_us_per_frame'], 2), 'fps', round(d['fps_wall']))")
  done
  KLT_AMD_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu --no-4k --api-frames 0 --no-fast --replace-frames 0 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  echo "$lib bench" $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v})")
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_long.py tests/test_shard.py tests/test_gpu_pyramid.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
