#!/bin/bash
# klt.h per-call path (host frames, PCIe inclusive): A/B of library builds and
# of the per-call switches (KLT_AMD_UPLOAD_PIECE_KB, KLT_AMD_FEAT_ZERO_COPY,
# KLT_AMD_TRACK_ORDER).  usage (via gpurun): bash tools/api_cycle.sh <tag> [var ...]
set -o pipefail
OUT=gpurun_out/${1:-api}; shift; mkdir -p $OUT
for v in default "$@"; do
  if [ "$v" = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
  for cfg in "0 0 0" "0 1 0" "512 1 0" "512 1 1" "256 1 1" "1024 1 1" "512 0 0"; do
    set -- $cfg
    KLT_AMD_UPLOAD_PIECE_KB=$1 KLT_AMD_FEAT_ZERO_COPY=$2 KLT_AMD_TRACK_ORDER=$3 \
      timeout -k 10 200 python tools/microbench.py api --frames 120 --features 5000 > $OUT/last.json || exit 1
    echo "$v piece_kb=$1 zero_copy=$2 input_order=$3" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['us_per_call_median'],1), 'us/call', round(d['fps'],1), 'fps', d['live_at_end'], 'live')") | tee -a $OUT/sweep.txt
  done
done
