#!/bin/bash
# Round 4: the 4K pass (bench roofline_4k) A/B, this build vs HEAD, alternating processes
set -o pipefail
OUT=gpurun_out/r04m; mkdir -p $OUT
export TMPDIR=/tmp
HEADLIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/head/libklt_amd.so
for r in 1 2 3; do for v in new head; do
  if [ "$v" = head ]; then export KLT_AMD_LIB=$HEADLIB; else unset KLT_AMD_LIB; fi
  echo "$v $(timeout -k 10 120 python3 archive/tools_exp/pass4k_once.py 2>/dev/null | tail -1)" || exit 1
done; done
