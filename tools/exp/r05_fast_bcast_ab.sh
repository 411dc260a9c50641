#!/bin/bash
# Round 5: the fast (wave-shuffle) window sums combining their four row
# totals by DPP row_bcast:15 / row_bcast:31 and one readlane (KLT_T7_BCAST=1,
# default build) against four readlanes and three adds (lib/var/bc0): the
# fast-mode GPU tests (same floats: a + b == b + a), then the bench's fast
# leg, three alternating rounds.
set -o pipefail
OUT=gpurun_out/${1:-r05bc}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  -k "fast" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ARGS="--no-cpu --no-4k --api-frames 0 --replace-frames 0"
for round in 1 2 3; do
  for lib in default bc0; do
    if [ $lib = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$lib/libklt_amd.so; fi
    timeout -k 10 300 python3 bench.py $ARGS > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); f=d['fast']
print('round $round $lib exact', round(d['value']), 'fast', round(f['value']), 'fast k_track us/frame', round(f['k_track_us_per_frame'], 3),
      'exact k_track', round(d['kernels_us_per_frame']['k_track'], 3), 'vs_exact', {k: f['vs_exact'][k] for k in ('val_mismatches', 'max_dx', 'max_dy')})" | tee -a $OUT/ab.txt
  done
done
