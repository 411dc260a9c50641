#!/bin/bash
# Round 5: the 1080p timed region (16.0 us/frame in r05f3) against its own
# replay's kernel sum (13.7 us/frame).  The rocprof trace of r05f3 shows the
# overlapped pyramids and tracker each running 1.6-2x their solo time while
# co-resident, and the timed region starting after ~8 ms of host-only work.
# Round 1 (r05ow): overlapped (default) vs --serial, each with the 10-frame
# warm-up and a 489-frame one (the latter also tracks fewer live features, so
# it only bounds the clock effect).  Round 2 (r05ow2, after bench.py's device
# warm-up): with and without it, overlapped and serial.
set -o pipefail
OUT=gpurun_out/${1:-r05ow}; mkdir -p $OUT
export TMPDIR=/tmp
LIGHT="--no-cpu --no-4k --api-frames 0 --replace-frames 0 --no-fast"
VARIANTS=${VARIANTS:-"default|--serial|--no-device-warmup|--no-device-warmup --serial"}
for round in 1 2 3; do
  IFS='|' read -ra VS <<< "$VARIANTS"
  for v in "${VS[@]}"; do
    [ "$v" = default ] && a="" || a="$v"
    timeout -k 10 300 python3 bench.py $LIGHT $a > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('round $round', repr('$v'), round(d['value']), 'us/frame', round(1e3*d['ms_per_step'],2),
      'kernels/frame', {k: round(x, 2) for k, x in d['kernels_us_per_frame'].items()},
      'live', d['live_features'], 'devwarm', {k: d.get('device_warmup', {}).get(k) for k in ('runs', 'ms')})" | tee -a $OUT/ab.txt
  done
done
