#!/bin/bash
# Round 4: launch cost on this stack (tools/hipbench/launch) and the
# driver-shaped bench's enqueue time, with the kernel-argument placement
# switched (HIP_FORCE_DEV_KERNARG) both ways.
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5 --min-chunks 1 --serial"
timeout -k 10 120 tools/hipbench/launch 2000 > $OUT/launch.txt || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 tools/hipbench/launch 2000 > $OUT/launch_k0.txt || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 tools/hipbench/launch 2000 > $OUT/launch_k1.txt || exit 1
for k in "" 0 1 "" 0 1; do
  if [ -n "$k" ]; then export HIP_FORCE_DEV_KERNARG=$k; else unset HIP_FORCE_DEV_KERNARG; fi
  timeout -k 10 300 python3 bench.py $Q > $OUT/b$k.json 2> $OUT/b$k.err || { tail -5 $OUT/b$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$k.json')); print('kernarg=$k', round(d['value']), d['timed_region_host'])"
done
cat $OUT/launch*.txt
