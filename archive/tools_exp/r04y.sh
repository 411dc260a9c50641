#!/bin/bash
# Round 4: refinement steps as cached graph launches (KLT_SEL_GRAPH=1, default)
# vs one launch per kernel; 4K-only 64-row l0 tiles: parity and REPLACE
set -o pipefail
OUT=gpurun_out/r04y; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_select.py tests/test_gpu_select_engine.py "tests/test_gpu_long.py::test_replace_harness_config3r" "tests/test_shard.py::test_c_shard_replace_equals_single_gpu" tests/test_gpu_pyramid.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for g in 1 0 1 0; do
  KLT_SEL_GRAPH=$g timeout -k 10 300 python3 bench.py $Q > $OUT/b$g.json 2> $OUT/b$g.err || { tail -5 $OUT/b$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$g.json'))['api']; r=d['replace']; print('graph=$g', round(r['value']), round(r['us_per_replace_median']), r['parity']['columns_mismatched'], {k: round(v) for k, v in r['select_median'].items()})"
done
KLT_SEL_TRACE=1 timeout -k 10 120 python3 tools/exp/replace_probe.py 12 > $OUT/probe.txt 2> $OUT/probe_trace.txt; tail -1 $OUT/probe.txt
