#!/bin/bash
# Round 4: the bench's API legs (per call, registered, REPLACE, sequence) after
# the host-sort / selection-engine changes; registered frames read in place by
# k_pyr_l0 (KLT_MAPPED_FRAMES=1) as an A/B
set -o pipefail
OUT=gpurun_out/r04q; mkdir -p $OUT
export TMPDIR=/tmp
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for v in 0 1 0 1; do
  KLT_MAPPED_FRAMES=$v timeout -k 10 300 python3 bench.py $Q > $OUT/b$v.json 2> $OUT/b$v.err || { tail -5 $OUT/b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$v.json'))['api']; print('mapped=$v', {k: (round(v['value']), round(v.get('us_per_call_median', v.get('us_per_replace_median', 0)))) for k,v in d.items() if isinstance(v, dict) and 'value' in v}, d['replace']['parity'], {k: round(v) for k, v in d['replace']['select_median'].items()})"
done
