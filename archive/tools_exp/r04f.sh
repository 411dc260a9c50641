#!/bin/bash
# Round 4: first-launch host cost -- launch microbench after device sync, and
# the batched call's enqueue by sync kind / stream (archive/tools_exp/enqueue_probe.py)
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 tools/hipbench/launch 2000 > $OUT/launch.txt || exit 1
cat $OUT/launch.txt
timeout -k 10 300 python3 archive/tools_exp/enqueue_probe.py 20 30 || exit 1
timeout -k 10 300 python3 archive/tools_exp/enqueue_probe.py 64 20 || exit 1
