#!/bin/bash
# KLTTrackSequence (host frames, uploads overlapped with the batched device
# path): pinned staging filled by N copy threads (KLT_AMD_COPY_THREADS; 0 =
# the runtime's own staging of pageable frames), 1080p and 4K.
# usage (via gpurun): bash tools/apiseq_cycle.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-apiseq}; mkdir -p $OUT
for th in 4 0 8 2; do
  for args in "--frames 300 --features 5000" "--width 3840 --height 2160 --frames 100 --features 20000"; do
    KLT_AMD_COPY_THREADS=$th timeout -k 10 300 python tools/microbench.py apiseq $args > $OUT/last.json || exit 1
    echo "copy_threads=$th $args" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['fps'],1), 'fps', round(d['us_per_frame'],1), 'us/frame', d['live_at_end'], 'live')") | tee -a $OUT/sweep.txt
  done
done
