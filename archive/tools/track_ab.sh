#!/bin/bash
# Tracker A/B on one box: the default library against variant builds
# (VARS -> lib/var/<name>/libklt_amd.so), batched 1080p/5000 features (64-frame
# launches, table on, tracker events) and 4K/2500 features (a sharded rank's
# load); two rounds.  usage (via gpurun): VARS="a" bash archive/tools/track_ab.sh
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for cfg in "--width 1920 --height 1080 --features 5000" "--width 3840 --height 2160 --features 2500"; do
  for v in default $VARS; do
    if [ $v = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
    timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 --table $cfg > gpurun_out/trkab.json || exit 1
    echo "$cfg $v $(python3 -c "import json; d=json.load(open('gpurun_out/trkab.json')); print('track', round(d['track_us_per_frame'],2), 'fps', round(d['fps_wall']))")"
  done
done; done
