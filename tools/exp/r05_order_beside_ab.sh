#!/bin/bash
# Round 5: a one-stream klt_hip_track_frames call's processing-order sort on
# the pyramid stream beside the build (KLT_ORDER_BESIDE=1, default) against
# ahead of the build on the tracking stream (KLT_ORDER_BESIDE=0): tracker
# parity, then the driver-shaped bench (--steps 20 --warmup 5, where the
# timed call sorts) and the default bench, three alternating rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05ob}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "track or long or sequence or api" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LIGHT="--no-cpu --no-4k --api-frames 0 --replace-frames 0 --no-fast"
for round in 1 2 3; do
  for ob in 1 0; do
    for shape in "--steps 20 --warmup 5" ""; do
      KLT_ORDER_BESIDE=$ob timeout -k 10 300 python3 bench.py $LIGHT $shape > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('round $round beside=$ob', repr('$shape'), round(d['value']), 'us/frame', round(1e3*d['ms_per_step'],2),
      'enqueue_us', round(d['timed_region_host']['enqueue_us'],1))" | tee -a $OUT/ab.txt
    done
  done
done
