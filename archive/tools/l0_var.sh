#!/bin/bash
# level-0 kernel: library variants (lib/var/NAME) x options: bash tools/l0_var.sh tag var1 var2 ...
OUT=gpurun_out/${1:-l0v}; shift; mkdir -p $OUT
for v in default "$@"; do
  if [ "$v" = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
  for args in "--frames 65 --chunk 32" "--width 3840 --height 2160 --frames 65 --chunk 32"; do
    timeout -k 10 300 python tools/microbench.py frames --reps 3 --pyr-only --features 8 $args $L0OPT > $OUT/last.json || exit 1
    echo "$v $args" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['us_per_frame_wall'],2), 'l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))") | tee -a $OUT/sweep.txt
  done
done
