#!/bin/bash
# Timing sweep of the microbenchmarks.  usage: bash tools/micro_cycle.sh <tag>
set -o pipefail
TAG=${1:-micro}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for args in "pyr --width 1920 --height 1080" "pyr --width 3840 --height 2160" "pyr --width 3840 --height 2160 --generic" \
            "track --width 1920 --height 1080 --features 5000" "track --width 1920 --height 1080 --features 5000 --reduction fast" \
            "track --width 3840 --height 2160 --features 20000" "track --width 3840 --height 2160 --features 20000 --reduction fast"; do
  timeout -k 10 300 python tools/microbench.py $args >> $OUT/micro.jsonl 2>> $OUT/micro.err || { echo "failed: $args"; exit 1; }
done
cat $OUT/micro.jsonl
