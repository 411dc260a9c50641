#!/bin/bash
# Round 5: bench.py drops the library's cached processing order after its
# device warm-up (klt_hip_set_track_order), so that the timed region starts
# from the order state it would have with no device warm-up (default) --
# against keeping the order the warm-up runs left (--keep-order-cache): the
# driver-shaped and the default bench, three alternating rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05or}; mkdir -p $OUT
export TMPDIR=/tmp
LIGHT="--no-cpu --no-4k --api-frames 0 --replace-frames 0 --no-fast"
for round in 1 2 3; do
  for v in "" "--keep-order-cache" "--no-device-warmup"; do
    for shape in "--steps 20 --warmup 5" ""; do
      timeout -k 10 300 python3 bench.py $LIGHT $shape $v > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('round $round', repr('$v'), repr('$shape'), round(d['value']), 'us/frame', round(1e3*d['ms_per_step'],2), 'live', d['live_features'])" | tee -a $OUT/ab.txt
    done
  done
done
