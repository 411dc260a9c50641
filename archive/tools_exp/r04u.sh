#!/bin/bash
# Round 4: host enqueue of the driver-shaped call by how the caller waits before it
set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 archive/tools_exp/enqueue_probe.py 20 40 > $OUT/enqueue.txt 2> $OUT/enqueue.err || { tail -5 $OUT/enqueue.err; exit 1; }
cat $OUT/enqueue.txt
