#!/bin/bash
# Per-call KLTTrackFeatures timelines (tools/api_timeline.py under rocprofv3
# --kernel-trace --memory-copy-trace; torch-free process), registered and
# pageable frames, 60 calls each.
set -o pipefail
OUT=gpurun_out/${1:-r06tl}; mkdir -p $OUT
export TMPDIR=/tmp
for mode in register pageable; do
  F=; [ $mode = register ] && F=--register
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/$mode -o run --output-format csv -- \
    python3 tools/api_timeline.py run $F --frames 60 > $OUT/$mode.log 2>&1 || { tail -20 $OUT/$mode.log; exit 1; }
  python3 tools/api_timeline.py summary $OUT/$mode > $OUT/${mode}_summary.txt 2>&1 || { tail -5 $OUT/${mode}_summary.txt; exit 1; }
  echo "$mode: $(grep median $OUT/$mode.log) | $(tail -1 $OUT/${mode}_summary.txt)"
done
