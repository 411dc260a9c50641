#!/bin/bash
# the processing-order sort queued ahead of the pyramid wait (this build) vs ee9628f (variant ee9):
# tracker / shard / API tests, then the driver-shaped bench (--steps 20) and the default bench
set -o pipefail
OUT=gpurun_out/exp30; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_track.py tests/test_shard.py tests/test_gpu_memory.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3; do for m in new ee9; do
  if [ $m = new ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/ee9/libklt_amd.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --api-frames 0 --no-4k > $OUT/s20.json 2> $OUT/s20.err || { tail -5 $OUT/s20.err; exit 1; }
  a=$(python3 -c "import json; d=json.load(open('$OUT/s20.json')); print('s20', round(d['value']))")
  timeout -k 10 300 python bench.py --no-cpu --api-frames 0 --no-4k > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  b=$(python3 -c "import json; d=json.load(open('$OUT/b.json')); print('default', round(d['value']), 'trk', round(d['kernels_us_per_frame']['k_track'],2))")
  echo "$m | $a | $b"
done; done
