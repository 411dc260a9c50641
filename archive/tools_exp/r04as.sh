#!/bin/bash
# Round 4: k_pyr_l0 workgroup phase cycles after the edge-tile change, interior
# against edge tiles (tools/hipbench/pyrprof), 1080p and 4K, interleaved levels
set -o pipefail
OUT=gpurun_out/r04as; mkdir -p $OUT
for sz in "1920 1080" "3840 2160"; do
  set -- $sz
  timeout -k 10 120 tools/hipbench/pyrprof $OUT/rec_$1.bin $1 $2 1 || exit 1
  python3 tools/exp/pyrprof_an.py $OUT/rec_$1.bin || exit 1
done
