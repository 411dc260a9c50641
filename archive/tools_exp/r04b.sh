#!/bin/bash
# Round 4: where the driver-shaped timed region's non-kernel time goes --
# CLOCK_MONOTONIC marks around the region (bench timed_region_host) against
# the kernel trace, for the overlapped two-chunk and the one-chunk serial
# schedules.  usage (via gpurun): bash archive/tools_exp/r04b.sh
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5"
i=0
for v in "" "--min-chunks 1 --serial" "" "--min-chunks 1 --serial"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt$i -o run --output-format csv -- python3 bench.py $Q $v > $OUT/kt$i.json 2> $OUT/kt$i.err || { tail -5 $OUT/kt$i.err; exit 1; }
done
for i in 1 2 3 4; do python3 tools/region_marks.py $OUT/kt$i.json $(find $OUT/kt$i -name "*kernel_trace.csv"); done
