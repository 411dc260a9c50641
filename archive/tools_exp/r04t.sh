#!/bin/bash
# Round 4: host sort with lock-free claiming and a spinning caller (and team
# steps, sortbench only); REPLACE parity and the bench's API legs
set -o pipefail
OUT=gpurun_out/r04t; mkdir -p $OUT
export TMPDIR=/tmp
g++ -O3 -std=c++17 -pthread -Iklt-feature-tracker-acceleration-gpus_amd/csrc tools/hostcheck/sortbench.cpp -o $OUT/sortbench
timeout -k 10 300 $OUT/sortbench > $OUT/sortbench.txt && grep -E 'partition_n|"depth": (0|3|4)' $OUT/sortbench.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_select_engine.py tests/test_gpu_select.py "tests/test_gpu_long.py::test_replace_harness_config3r" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
KLT_SEL_TRACE=1 timeout -k 10 120 python3 tools/exp/replace_probe.py 12 > $OUT/probe.txt 2> $OUT/probe_trace.txt; tail -3 $OUT/probe.txt
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $Q > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$i.json'))['api']; print({k: (round(v['value']), round(v.get('us_per_call_median', v.get('us_per_replace_median', 0)))) for k,v in d.items() if isinstance(v, dict) and 'value' in v}, d['replace']['parity']['columns_mismatched'], {k: round(v) for k, v in d['replace']['select_median'].items()})"
done
# host time inside the driver-shaped timed call (KLT_HOST_PROF build)
Q="--no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5"
KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/hp/libklt_amd.so timeout -k 10 300 python3 bench.py $Q > $OUT/hp.json 2> $OUT/hp.err || { tail -5 $OUT/hp.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/hp.json')); print(round(d['value']), d['timed_region_host'])"
grep -n hostmark $OUT/hp.err | head -60
# registered frames fetched by a kernel on the tracking stream (KLT_FETCH_KERNEL=1) vs one DMA
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for v in 0 1 0 1; do
  KLT_FETCH_KERNEL=$v timeout -k 10 300 python3 bench.py $Q > $OUT/f$v.json 2> $OUT/f$v.err || { tail -5 $OUT/f$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/f$v.json'))['api']; print('fetch=$v', {k: (round(x['value']), round(x.get('us_per_call_median', 0))) for k,x in d.items() if isinstance(x, dict) and 'value' in x and 'per_call' in k})"
done
