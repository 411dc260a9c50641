#!/bin/bash
# Round 5: the 1080p bench at short chunks, whose pyramids (8 frames ~ 213 MB)
# could still sit in the 256 MB MALL when the tracker gathers from them,
# against the default 64 (with the device warm-up; light legs only).
set -o pipefail
OUT=gpurun_out/${1:-r05cs}; mkdir -p $OUT
export TMPDIR=/tmp
LIGHT="--no-cpu --no-4k --api-frames 0 --replace-frames 0 --no-fast"
for round in 1 2; do
  for ch in ${CHUNKS:-64 8 16 32}; do
    timeout -k 10 300 python3 bench.py $LIGHT --chunk $ch $EXTRA > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('round $round chunk $ch $EXTRA', round(d['value']), 'us/frame', round(1e3*d['ms_per_step'],2),
      'kernels/frame', {k: round(x, 2) for k, x in d['kernels_us_per_frame'].items()},
      'per launch', {k: round(x, 1) for k, x in d['kernels_us_per_launch'].items() if x})" | tee -a $OUT/ab.txt
  done
done
