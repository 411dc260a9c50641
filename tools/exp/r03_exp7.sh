#!/bin/bash
# per-call API variants: feature list via copy kernels (KLT_FEAT_MODE=2), level-0 reading registered frames in place
# (KLT_MAPPED_FRAMES=1); parity of each variant against the default is in the bench's equals_* keys
set -o pipefail
OUT=gpurun_out/exp7; mkdir -p $OUT
for r in 1 2; do for v in "X=0" "KLT_FEAT_MODE=2" "KLT_MAPPED_FRAMES=1" "KLT_FEAT_MODE=2 KLT_MAPPED_FRAMES=1"; do
  env $v timeout -k 10 300 python bench.py --no-cpu --no-fast --no-4k --replace-frames 0 --api-frames 120 --steps 64 --replay-frames 64 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json'))['api']
print('$v', {k: (round(d[k]['value']), round(d[k]['us_per_call_median'],1)) for k in ('per_call','per_call_harness','per_call_registered')}, d['per_call_registered']['equals_per_call'], d['per_call_equals_sequence'])"
done; done
