#!/bin/bash
# Round 4: kernel timeline of the driver-shaped timed region (--steps 20),
# warm-up adjacent: the launches of the timed call (l0/l1 with grid.z 20, then k_track7)
set -o pipefail
OUT=gpurun_out/r04al; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$OUT/b.json 2> $GRAFT_REPO_ROOT/$OUT/b.err || { tail -5 $GRAFT_REPO_ROOT/$OUT/b.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/region_marks.py $OUT/b.json $(find $OUT/p -name "*kernel_trace.csv") 2>&1 | tail -12
