VARS=${VARS:-nohs}
set -o pipefail
for r in 1 2; do for v in default $VARS; do
  if [ $v = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --frames 129 --reps 2 --chunk 64 --pyr-only > gpurun_out/pyrab.json || exit 1
  echo $v $(python3 -c "import json; d=json.load(open('gpurun_out/pyrab.json')); print('l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
done; done
