#!/bin/bash
# Round 4: KLTTrackSequence call-to-call variance (12 calls per process, 200
# frames each), three processes; the last with the sort pool off (KLT_AMD_SORT_DEPTH=0)
set -o pipefail
OUT=gpurun_out/r04aj2; mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 3 2 4; do
  E=""; [ $k -ge 3 ] && E="KLT_AMD_SORT_DEPTH=0"
  env $E timeout -k 10 300 python3 tools/microbench.py apiseq --frames 201 --reps 12 > $OUT/s$k.json 2> $OUT/s$k.err || { tail -5 $OUT/s$k.err; exit 1; }
  echo "process $k $E: $(grep -o 'rep [0-9]*: [0-9]* fps' $OUT/s$k.err | awk '{print $3}' | tr '\n' ' ')"
done
