# per-wave phase cycles of the two tracker kernels (instrumented build)
set -o pipefail
export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/prof/libklt_amd.so
for impl in 0 1; do for cfg in "--features 1000" "--features 5000"; do
  timeout -k 5 120 python tools/microbench.py frames $cfg --frames 129 --reps 1 --chunk 64 --impl $impl --prof > gpurun_out/t7p.json || exit 1
  echo "impl=$impl $cfg" $(python3 -c "
import json; d=json.load(open('gpurun_out/t7p.json')); p=d['prof_cycles_per_wave_frame']
print({k: round(v) if v > 10 else round(v, 2) for k, v in p.items()}, 'track', round(d['track_us_per_frame'], 2))")
done; done
