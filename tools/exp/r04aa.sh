#!/bin/bash
# Round 4: the driver-shaped timed region -- warm-up steps right before it
# (new order) vs the harness's bookkeeping between them (KLT_BENCH_OLD_ORDER=1);
# host marks of the timed call (KLT_HOST_PROF build)
set -o pipefail
OUT=gpurun_out/r04aa; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5"
for o in 0 1 0 1 0 1; do
  KLT_BENCH_OLD_ORDER=$o timeout -k 10 300 python3 bench.py $Q > $OUT/s$o.json 2> $OUT/s$o.err || { tail -5 $OUT/s$o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s$o.json')); print('old_order=$o', round(d['value']), round(d['timed_region_host']['enqueue_us'],1), round(d['ms_per_step']*1e3,2), round(d['roofline']['frac'],3))"
done
for o in 0 1; do
  KLT_BENCH_OLD_ORDER=$o KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/hp/libklt_amd.so timeout -k 10 300 python3 bench.py $Q > $OUT/hp$o.json 2> $OUT/hp$o.err || { tail -5 $OUT/hp$o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/hp$o.json')); print('hp old_order=$o', round(d['value']), d['timed_region_host'])"
  awk '/enter_ns/{n++} n==1' $OUT/hp$o.err | grep hostmark | head -20
done
