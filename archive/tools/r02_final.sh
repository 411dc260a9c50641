#!/bin/bash
# Round-2 GPU cycle: full GPU tests, the default bench line, a kernel-trace
# profile of it, tracker PMC (profiles/pmc_tracker.json), pyramid traffic PMC
# at 1080p and 4K, and the config-4 rank simulation.  Every GPU step has its
# own time limit; the script stops at the first failure.
# usage (via gpurun): bash archive/tools/r02_final.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r02}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu --api-frames 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 5 > $OUT/kernel_stats_isolated.txt || exit 1
bash tools/pmc_track.sh $TAG/pmctrk > $OUT/pmctrk.log 2>&1 || { tail -20 $OUT/pmctrk.log; exit 1; }
bash tools/pmc_traffic.sh $TAG/traffic1080 --chunk 64 > $OUT/traffic1080.log 2>&1 || { tail -5 $OUT/traffic1080.log; exit 1; }
bash tools/pmc_traffic.sh $TAG/traffic4k --chunk 64 --width 3840 --height 2160 > $OUT/traffic4k.log 2>&1 || { tail -5 $OUT/traffic4k.log; exit 1; }
timeout -k 10 600 python tools/shard_sim.py --worlds 1 2 4 8 --frames 257 --chunk 64 --margins 64 > $OUT/shard_sim.log 2>&1 || { tail -5 $OUT/shard_sim.log; exit 1; }
cat $OUT/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('value', d['value'], 'kern', d['kernels_us_per_frame'], 'roof', d['roofline']['frac'], d['roofline_4k']['frac'], 'api', d['api']['per_call']['value'], d['api']['sequence']['value'])"
grep '^{"world' $OUT/shard_sim.log
