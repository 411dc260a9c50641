#!/bin/bash
# Pyramid-kernel A/B on one box: the k_pyr_l0 + k_pyr_l1 tiles (mode 1) and
# k_pyr_strip (mode 2) of the default library and of variant builds
# (VARS="name ..." -> lib/var/<name>/libklt_amd.so), batched 64 frames per
# launch, pyramids only, at 1080p and 4K; two rounds.
# usage (via gpurun): VARS="a b" bash tools/strip_ab.sh [extra microbench args]
set -o pipefail
mkdir -p gpurun_out
run() {  # lib mode W H
  if [ $1 = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$1/libklt_amd.so; fi
  timeout -k 5 120 python tools/microbench.py frames --width $3 --height $4 --frames 129 --reps 2 --chunk 64 \
    --pyr-only --strips $2 "${EXTRA[@]}" > gpurun_out/stripab.json || exit 1
  echo "$3x$4 $1 mode $2 $(python3 -c "import json; d=json.load(open('gpurun_out/stripab.json')); print('pass', round(d['pass_us_per_frame'],2), 'l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'strip', round(d['strip_us_per_frame'],2))")"
}
EXTRA=("$@")
for r in 1 2; do for res in "1920 1080" "3840 2160"; do
  run default 1 $res
  for v in default $VARS; do run $v 2 $res; done
done; done
