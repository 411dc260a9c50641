#!/bin/bash
# per-call KLTTrackFeatures timelines (pageable and registered frame buffers)
set -o pipefail
OUT=gpurun_out/exp6; mkdir -p $OUT
export TMPDIR=/tmp
for v in "" "--register"; do
  tag=plain; [ -n "$v" ] && tag=registered
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl_$tag -o run -- python tools/api_timeline.py run $v --frames 100 > $OUT/tl_$tag.log 2>&1 || { tail -5 $OUT/tl_$tag.log; exit 1; }
  python3 tools/api_timeline.py summary $OUT/tl_$tag > $OUT/timeline_$tag.txt || exit 1
  echo "== $tag"; cat $OUT/timeline_$tag.txt
done
