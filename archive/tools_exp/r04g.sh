#!/bin/bash
# Round 4 checkpoint: GPU suite, then the driver-shaped and default benches
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
Q="--no-cpu --api-frames 0 --no-4k --no-fast"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $Q --steps 20 --warmup 5 > $OUT/s20_$i.json 2> $OUT/s20_$i.err || { tail -5 $OUT/s20_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py $Q > $OUT/full_$i.json 2> $OUT/full_$i.err || { tail -5 $OUT/full_$i.err; exit 1; }
done
for f in $OUT/s20_*.json $OUT/full_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), round(d['timed_region_host']['enqueue_us'],1), 'pmc' in d['tracker'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run --output-format csv -- python3 bench.py $Q --steps 20 --warmup 5 > $OUT/kt.json 2> $OUT/kt.err || { tail -5 $OUT/kt.err; exit 1; }
python3 tools/region_marks.py $OUT/kt.json $(find $OUT/kt -name "*kernel_trace.csv")
