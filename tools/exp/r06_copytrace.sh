#!/bin/bash
# each probe mode under rocprofv3 --kernel-trace
# --memory-copy-trace; reports the exit code, the wall time and whether the
# profiler timed out waiting for async-copy completions.
set -o pipefail
OUT=gpurun_out/${1:-r06ct}; mkdir -p $OUT
export TMPDIR=/tmp
for m in ${MODES:-torch hip seq_live seq_freed}; do
  a=$(date +%s.%N)
  timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/ct_$m -o run --output-format csv -- \
    python3 tools/exp/r06_copytrace_probe.py $m > $OUT/ct_$m.log 2>&1
  rc=$?
  b=$(date +%s.%N)
  to=$(grep -c "timed out after" $OUT/ct_$m.log)
  echo "$m rc=$rc wall_s=$(python3 -c "print(round($b-$a,1))") profiler_timeouts=$to $(grep -o 'waiting for [0-9]* completion' $OUT/ct_$m.log | head -1)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
done
exit 0
