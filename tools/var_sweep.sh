#!/bin/bash
# compare library variants (make -C csrc variant NAME=... DEFS=...) on the frames microbench
OUT=gpurun_out/${1:-var}; shift; mkdir -p $OUT
for v in default "$@"; do
  if [ "$v" = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
  for args in "--chunk 16 --no-patch" "--chunk 16" "--chunk 16 --no-patch --features 4000" "--chunk 16 --no-patch --width 3840 --height 2160 --features 20000 --frames 65"; do
    timeout -k 10 300 python tools/microbench.py frames --frames 129 --reps 3 $args > $OUT/last.json || exit 1
    echo "$v $args" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['us_per_frame_wall'],2), round(d['l0_us_per_frame'],2), round(d['track_us_per_frame'],2))") | tee -a $OUT/sweep.txt
  done
done
