#!/bin/bash
# timeline of the driver-shaped bench (--steps 20): kernels + HIP API calls
set -o pipefail
OUT=gpurun_out/exp29; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT/tr -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --api-frames 0 --no-4k > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
ls $OUT/tr/*
