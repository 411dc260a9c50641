#!/bin/bash
# device segment sort (k_sel_segsort / _g): selection tests, REPLACE bench leg
set -o pipefail
OUT=gpurun_out/exp8; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_select_engine.py tests/test_gpu_select.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/select_tests.log 2>&1 || { tail -30 $OUT/select_tests.log; exit 1; }
tail -1 $OUT/select_tests.log
timeout -k 10 300 python bench.py --no-cpu --no-fast --no-4k --steps 64 --replay-frames 64 --api-frames 60 > $OUT/bench_api.json 2> $OUT/bench_api.err || { tail -5 $OUT/bench_api.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_api.json')); print(json.dumps(d['api']['replace']))"
