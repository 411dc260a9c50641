#!/bin/bash
# Batched sequence A/B (1080p, 5000 features, feature table, chunk c+1's
# pyramids overlapped with chunk c's tracking) over chunk sizes and library
# variants (VARS -> lib/var/<name>/libklt_amd.so): wall frames/s and the
# kernels' own us per frame.  usage (via gpurun): VARS="a" CHUNKS="8 16 64" bash archive/tools/chunk_ab.sh
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for c in ${CHUNKS:-8 16 32 64}; do for v in default $VARS; do
  if [ $v = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --frames 257 --reps 2 --chunk $c --table --overlap "$@" > gpurun_out/chunkab.json || exit 1
  echo "chunk $c $v $(python3 -c "import json; d=json.load(open('gpurun_out/chunkab.json')); print('fps', round(d['fps_wall']), 'l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'track', round(d['track_us_per_frame'],2))")"
done; done; done
