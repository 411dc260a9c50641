#!/bin/bash
# round-3 experiments: tile write patterns, E-phase 16-byte stores (variant e4), tracker wave priority
set -o pipefail
OUT=gpurun_out/exp1; mkdir -p $OUT
timeout -k 10 120 tools/hipbench/tilewrite > $OUT/tilewrite.txt 2>&1 || exit 1
cat $OUT/tilewrite.txt
VARS=e4 timeout -k 10 600 bash tools/pyr_ab.sh > $OUT/pyr_ab.txt 2>&1 || { cat $OUT/pyr_ab.txt; exit 1; }
cat $OUT/pyr_ab.txt
KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/e4/libklt_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/e4_tests.log 2>&1 || { tail -20 $OUT/e4_tests.log; exit 1; }
tail -1 $OUT/e4_tests.log
bash tools/exp/prio_ab.sh exp1/prio
timeout -k 10 600 python -u -m pytest tests/test_gpu_select_engine.py tests/test_gpu_select.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/select_tests.log 2>&1 || { tail -20 $OUT/select_tests.log; exit 1; }
tail -1 $OUT/select_tests.log
timeout -k 10 300 python bench.py --no-cpu --no-fast --no-4k > $OUT/bench_api.json 2> $OUT/bench_api.err || { tail -5 $OUT/bench_api.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_api.json')); print(json.dumps(d['api']['replace']))"
