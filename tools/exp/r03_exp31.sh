#!/bin/bash
# driver-shaped bench (--steps 20): timed-region schedules
set -o pipefail
OUT=gpurun_out/exp31; mkdir -p $OUT
for r in 1 2 3; do for m in "--min-chunks 2" "--min-chunks 1 --serial" "--min-chunks 2 --serial" "--min-chunks 4"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --api-frames 0 --no-4k --no-fast --replay-frames 64 $m > $OUT/s20.json 2> $OUT/s20.err || { tail -5 $OUT/s20.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s20.json')); print('$m', round(d['value']), d['config']['chunk'])"
done; done
