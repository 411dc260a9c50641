#!/bin/bash
# the round-5 reproduction (tools/seq_variance.py, 12
# KLTTrackSequence calls, under rocprofv3 --kernel-trace --memory-copy-trace)
# with the exit hook's host release off (KLT_EXIT_RELEASE=0, the round-5 hook)
# and on (default); each run: exit code, wall time, profiler timeout lines.
set -o pipefail
OUT=gpurun_out/${1:-r06es}; mkdir -p $OUT
export TMPDIR=/tmp
for rel in ${RELS:-0 1}; do
  mkdir -p $OUT/es_rel$rel
  a=$(date +%s.%N)
  KLT_EXIT_RELEASE=$rel timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/es_rel$rel -o run \
    --output-format csv -- python3 -u tools/seq_variance.py $OUT/es_rel$rel > $OUT/es_rel$rel.log 2>&1
  rc=$?
  b=$(date +%s.%N)
  echo "KLT_EXIT_RELEASE=$rel rc=$rc wall_s=$(python3 -c "print(round($b-$a,1))") profiler_timeouts=$(grep -c 'timed out after' $OUT/es_rel$rel.log) $(grep -o 'waiting for [0-9]* completion' $OUT/es_rel$rel.log | head -1)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
