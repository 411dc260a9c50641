#!/bin/bash
# Round 5: the host copy pool's workers spinning up to 300 us after a
# generation before they sleep (KLT_AMD_POOL_SPIN_US, default 300) against
# sleeping at once (0): the per-call API (pageable frames: four pool
# generations per upload) and KLTTrackSequence, three alternating rounds;
# API and sequence GPU tests first.
set -o pipefail
OUT=gpurun_out/${1:-r05ps}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "api or sequence or host or per_call or memory" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ARGS="--steps 64 --no-cpu --no-4k --no-fast --replace-frames 0"
for round in 1 2 3; do
  for sp in 300 0; do
    KLT_AMD_POOL_SPIN_US=$sp timeout -k 10 300 python3 bench.py $ARGS > $OUT/b.json 2>> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); a=d['api']
print('round $round spin=$sp', {k: round(v['value']) for k, v in a.items() if isinstance(v, dict) and 'value' in v},
      'seq calls', [round(x) for x in a['sequence'].get('calls_fps', [])])" | tee -a $OUT/ab.txt
  done
done
