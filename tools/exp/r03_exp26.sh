#!/bin/bash
# k_track7 per-wave phase cycles (instrumented build) at 4K/2500 (one rank's load at 8 ranks) and 1080p/5000
set -o pipefail
OUT=gpurun_out/exp26; mkdir -p $OUT
export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/prof/libklt_amd.so
for args in "--width 3840 --height 2160 --features 2500" "--features 5000" "--width 3840 --height 2160 --features 20000"; do
  timeout -k 10 200 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 --prof $args > $OUT/last.json || exit 1
  echo "== $args"
  python3 -c "
import json; d=json.load(open('$OUT/last.json'))
for k in ('prof_cycles_per_wave_frame','prof_clock64_ghz','prof_wave_life_us','track_us_per_frame'):
    print('  ', k, d.get(k))"
done
