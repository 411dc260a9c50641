#!/bin/bash
# Same-box A/B of the round-1 build (ab/r01: the f04005e tree, built in place)
# against HEAD: the batched pyramid pass only, 64-frame launches, alternated.
# usage (via gpurun): bash archive/tools/ab_r01.sh [W H]
set -o pipefail
W=${1:-3840}; H=${2:-2160}
mkdir -p gpurun_out
for r in 1 2 3; do for v in r01 head; do
  if [ $v = r01 ]; then D=ab/r01; else D=.; fi
  timeout -k 5 120 python $D/tools/microbench.py frames --width $W --height $H --frames 129 --reps 2 --chunk 64 --pyr-only > gpurun_out/ab.json || exit 1
  echo $v $(python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
done; done
