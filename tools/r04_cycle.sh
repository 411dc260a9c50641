#!/bin/bash
# Round-4 GPU cycle.  usage (via gpurun): bash tools/r04_cycle.sh <tag> [tests] [prof] [pmc] [trk]
# Steps: optional GPU tests; the driver-shaped bench (--steps 20) and the
# default bench; optional rocprofv3 kernel traces (the bench, then the 4K
# config-4 shape in two separate processes: 20 000 features tracked between
# the pyramid launches, and the same frames' pyramids built back to back);
# pyramid traffic PMC at 1080p / 4K; tracker PMC.  Each GPU step has its own
# time limit; the script stops at the first failure.  Every summary starts
# with the commit it measured (COMMIT, set by the caller, else "unknown").
set -o pipefail
TAG=${1:-r04}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C=${COMMIT:-unknown}
has() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
if has tests; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err || { tail -20 $OUT/bench_s20.err; exit 1; }
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --api-frames 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
  { echo "# commit $C: rocprofv3 --kernel-trace of bench.py --no-cpu --api-frames 0 (1080p legs and the 4K legs together), isolated launches"; \
    python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 5; } > $OUT/kernel_stats_isolated.txt || exit 1
  # the 4K config-4 shape, one leg per process: tracked (20 000 features between the launches) and pyramids only
  M="frames --width 3840 --height 2160 --features 20000 --chunk 64 --frames 128 --reps 3 --table"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof4k_tracked -o run --output-format csv -- python3 tools/microbench.py $M > $OUT/prof4k_tracked.log 2>&1 || { tail -20 $OUT/prof4k_tracked.log; exit 1; }
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof4k_pyr -o run --output-format csv -- python3 tools/microbench.py $M --pyr-only > $OUT/prof4k_pyr.log 2>&1 || { tail -20 $OUT/prof4k_pyr.log; exit 1; }
  for leg in tracked pyr; do
    { echo "# commit $C: rocprofv3 --kernel-trace of tools/microbench.py $M$([ $leg = pyr ] && echo ' --pyr-only') (4K, 64-frame launches; $leg leg alone in its process), isolated launches"; \
      python3 tools/kstats_isolated.py $(find $OUT/prof4k_$leg -name "*kernel_trace.csv") 5; } > $OUT/kernel_stats_4k_$leg.txt || exit 1
  done
fi
if has pmc; then
  bash tools/pmc_traffic.sh $TAG/traffic1080 > $OUT/traffic1080.log 2>&1 || { tail -5 $OUT/traffic1080.log; exit 1; }
  python3 tools/pmc_traffic_json.py $OUT/traffic1080 1920 1080 $OUT/pmc_1080.json > /dev/null || exit 1
  bash tools/pmc_traffic.sh $TAG/traffic4k --width 3840 --height 2160 > $OUT/traffic4k.log 2>&1 || { tail -5 $OUT/traffic4k.log; exit 1; }
  python3 tools/pmc_traffic_json.py $OUT/traffic4k 3840 2160 $OUT/pmc_4k.json > /dev/null || exit 1
fi
if has trk; then
  bash tools/pmc_track.sh $TAG/trk > $OUT/trk.log 2>&1 || { tail -5 $OUT/trk.log; exit 1; }
fi
for b in bench_s20 bench; do
python3 - $OUT/$b.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r, r4 = d["roofline"], d.get("roofline_4k", {})
print(sys.argv[1], "value", round(d["value"]), "kern/frame", {k: round(v, 2) for k, v in d["kernels_us_per_frame"].items() if v},
      "roof", round(r["frac"], 3), "fpl", r["frames_per_launch"], "4k", round(r4.get("frac", 0), 3),
      {k: round(v, 2) for k, v in r4.get("kernels_us_per_frame", {}).items()},
      "po", round(r4.get("pyramids_only", {}).get("frac", 0), 3),
      "api", {k: round(v["value"]) for k, v in d.get("api", {}).items() if isinstance(v, dict) and "value" in v})
PY
done
