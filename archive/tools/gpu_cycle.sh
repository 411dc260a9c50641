#!/bin/bash
# One GPU-box cycle: parity tests, the default bench line, a kernel-trace profile.
# usage (via gpurun): bash archive/tools/gpu_cycle.sh <tag> [pytest -k expr | none] [bench args...]
set -o pipefail
TAG=${1:-dev}
K=${2:-}
shift $(( $# < 2 ? $# : 2 ))
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" != "none" ]; then
  if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider "${KARG[@]}" > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log; tail -3 $OUT/gpu_tests.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
fi
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu "$@" > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec python3 archive/tools/kstats.py {} \;
python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 5 > $OUT/kernel_stats_isolated.txt && cat $OUT/kernel_stats_isolated.txt
