#!/bin/bash
# Round-3 GPU cycle.  usage (via gpurun): bash archive/tools/r03_cycle.sh <tag> [tests] [prof] [pmc] [shard]
# Steps: optional GPU tests, the driver-shaped bench (--steps 20) and the
# default bench, optional rocprofv3 kernel-trace of the bench, pyramid traffic
# PMC at 1080p / 4K, the config-4 rank simulation.  Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r03}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
has() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err || { tail -20 $OUT/bench_s20.err; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu --api-frames 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
  python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 5 > $OUT/kernel_stats_isolated.txt || exit 1
fi
if has pmc; then
  bash tools/pmc_traffic.sh $TAG/traffic1080 > $OUT/traffic1080.log 2>&1 || { tail -5 $OUT/traffic1080.log; exit 1; }
  python3 tools/pmc_traffic_json.py $OUT/traffic1080 1920 1080 $OUT/pmc_1080.json > /dev/null || exit 1
  bash tools/pmc_traffic.sh $TAG/traffic4k --width 3840 --height 2160 > $OUT/traffic4k.log 2>&1 || { tail -5 $OUT/traffic4k.log; exit 1; }
  python3 tools/pmc_traffic_json.py $OUT/traffic4k 3840 2160 $OUT/pmc_4k.json > /dev/null || exit 1
fi
if has shard; then
  timeout -k 10 600 python tools/shard_sim.py --worlds 1 2 4 8 --frames 257 --chunk 64 --margins 64 > $OUT/shard_sim.log 2>&1 || { tail -5 $OUT/shard_sim.log; exit 1; }
  grep '^{"world' $OUT/shard_sim.log
fi
for b in bench_s20 bench; do
python3 - $OUT/$b.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r, r4 = d["roofline"], d.get("roofline_4k", {})
print(sys.argv[1], "value", round(d["value"]), "kern/frame", {k: round(v, 2) for k, v in d["kernels_us_per_frame"].items() if v},
      "roof", round(r["frac"], 3), "fpl", r["frames_per_launch"], "4k", round(r4.get("frac", 0), 3),
      {k: round(v, 2) for k, v in r4.get("kernels_us_per_frame", {}).items()},
      "api", {k: round(v["value"]) for k, v in d.get("api", {}).items() if isinstance(v, dict) and "value" in v})
PY
done
