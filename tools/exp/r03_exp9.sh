#!/bin/bash
# REPLACE leg at device/host thresholds (leaves <= 4096 sorted on the device, longer ones on the host)
set -o pipefail
OUT=gpurun_out/exp9; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_select_engine.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/select_tests.log 2>&1 || { tail -30 $OUT/select_tests.log; exit 1; }
tail -1 $OUT/select_tests.log
for r in 1 2; do for t in 32768 4096 8192 2048; do
  KLT_SEL_THRESHOLD=$t timeout -k 10 300 python bench.py --no-cpu --no-fast --no-4k --steps 64 --replay-frames 64 --api-frames 60 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json'))['api']['replace']; print('T=$t', round(d['value']), round(d['us_per_replace_median']), {k: round(v) for k,v in d['select_median'].items()}, d['parity']['columns_mismatched'])"
done; done
