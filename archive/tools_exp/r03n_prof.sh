#!/bin/bash
# k_track7 per-wave phase cycles and wave end-time spread (instrumented build), 1080p and 4K
set -o pipefail
mkdir -p gpurun_out/r03n
export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/prof/libklt_amd.so
for cfg in "--features 1000" "--features 5000" "--width 3840 --height 2160 --features 2500" "--width 3840 --height 2160 --features 20000"; do
  timeout -k 5 120 python tools/microbench.py frames $cfg --frames 129 --reps 1 --chunk 64 --impl 0 --prof > gpurun_out/r03n/p.json || exit 1
  echo "$cfg" $(python3 -c "
import json; d=json.load(open('gpurun_out/r03n/p.json')); p=d['prof_cycles_per_wave_frame']
print({k: round(v) if v > 10 else round(v, 2) for k, v in p.items()}, 'track', round(d['track_us_per_frame'], 2), 'life_us', round(d['prof_wave_life_us'],1), 'start%', [round(x,1) for x in d['prof_start_us_pct']], 'end%', [round(x,1) for x in d['prof_end_us_pct']], 'ghz', round(d['prof_clock64_ghz'],2))")
done
