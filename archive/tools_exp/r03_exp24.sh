#!/bin/bash
# effective clock of the pyramid kernels (GRBM_GUI_ACTIVE / 8 / duration), back to back vs between tracker launches
set -o pipefail
OUT=gpurun_out/exp24; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in track pyr; do
  f=""; [ $m = pyr ] && f="--pyr-only"
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $OUT/$m -o run --output-format csv -- python3 tools/microbench.py frames --width 3840 --height 2160 --features 20000 --frames 129 --reps 2 --chunk 64 $f > $OUT/$m.json 2> $OUT/$m.err || { tail -5 $OUT/$m.err; exit 1; }
done
ls -R $OUT | head -30
