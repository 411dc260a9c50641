#!/bin/bash
# One GPU-box cycle: parity tests, the default bench line, a kernel-trace profile.
# usage (via gpurun): bash tools/gpu_cycle.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-dev}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider "${KARG[@]}" > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/gpu_tests.log; tail -3 $OUT/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
find $OUT/prof -name "*kernel_stats.csv" -exec cut -c1-60,200- {} \; | cut -c1-200
python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 5 > $OUT/kernel_stats_isolated.txt && cat $OUT/kernel_stats_isolated.txt
