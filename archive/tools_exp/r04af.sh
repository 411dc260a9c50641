#!/bin/bash
# Round 4: the driver-shaped region (--steps 20) with the warm-up adjacent:
# one chunk on one stream (default) vs 2 or 4 overlapped chunks (--min-chunks)
set -o pipefail
OUT=gpurun_out/r04af; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5"
for m in 1 2 4 1 2 4; do
  timeout -k 10 300 python3 bench.py $Q --min-chunks $m > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('min_chunks=$m', round(d['value']), round(d['ms_per_step']*1e3,2), round(d['timed_region_host']['enqueue_us'],1))"
done
