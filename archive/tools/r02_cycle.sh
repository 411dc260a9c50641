#!/bin/bash
# One GPU-box cycle of round 2: the GPU tests (optionally a -k subset), then
# the default bench line.  Every GPU step has its own time limit; the script
# stops at the first failure.
# usage (via gpurun): bash archive/tools/r02_cycle.sh <tag> [pytest -k expr] [bench args...]
set -o pipefail
TAG=${1:-dev}; K=${2:-}; shift 2 2>/dev/null
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" != "none" ]; then
  if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -s "${KARG[@]}" > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log; grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
  [ $rc -ne 0 ] && { tail -40 $OUT/gpu_tests.log; exit $rc; }
fi
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
