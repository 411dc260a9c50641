#!/bin/bash
# Round-6 profile step: rocprofv3 --kernel-trace --stats of bench.py (1080p and
# the 4K legs) and of the 4K config-4 shape in two separate processes
# (tracked / pyramids only), each summarised by tools/kstats_isolated.py;
# tools/r04_cycle.sh's prof step without its two bench runs.
set -o pipefail
TAG=${1:-r06}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C=${COMMIT:-unknown}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu --api-frames 0 --no-sharded-4k > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
{ echo "# commit $C: rocprofv3 --kernel-trace of bench.py --no-cpu --api-frames 0 --no-sharded-4k (1080p legs and the 4K legs together), isolated launches"; \
  python3 tools/kstats_isolated.py $(find $OUT/prof -name "*kernel_trace.csv") 5; } > $OUT/kernel_stats_isolated.txt || exit 1
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv 2>/dev/null
M="frames --width 3840 --height 2160 --features 20000 --chunk 64 --frames 128 --reps 3 --table"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof4k_tracked -o run --output-format csv -- python3 tools/microbench.py $M > $OUT/prof4k_tracked.log 2>&1 || { tail -20 $OUT/prof4k_tracked.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof4k_pyr -o run --output-format csv -- python3 tools/microbench.py $M --pyr-only > $OUT/prof4k_pyr.log 2>&1 || { tail -20 $OUT/prof4k_pyr.log; exit 1; }
for leg in tracked pyr; do
  { echo "# commit $C: rocprofv3 --kernel-trace of tools/microbench.py $M$([ $leg = pyr ] && echo ' --pyr-only') (4K, 64-frame launches; $leg leg alone in its process), isolated launches"; \
    python3 tools/kstats_isolated.py $(find $OUT/prof4k_$leg -name "*kernel_trace.csv") 5; } > $OUT/kernel_stats_4k_$leg.txt || exit 1
done
head -12 $OUT/kernel_stats_isolated.txt
