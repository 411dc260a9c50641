#!/bin/bash
# Round 4: tiled 7x7 trackability map (k_min_eigen7), segment downloads on
# their own stream: selection parity, REPLACE timing, kernel times; then the
# 64-row level-0 tiles A/B (r04x.sh)
set -o pipefail
OUT=gpurun_out/r04w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_select.py tests/test_gpu_select_engine.py "tests/test_gpu_long.py::test_replace_harness_config3r" "tests/test_shard.py::test_eigen_rows_of_band_pyramid" "tests/test_shard.py::test_c_shard_replace_equals_single_gpu" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $Q > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$i.json'))['api']; r=d['replace']; print(round(r['value']), round(r['us_per_replace_median']), r['parity']['columns_mismatched'], {k: round(v) for k, v in r['select_median'].items()}, 'registered', round(d['per_call_registered']['value']))"
done
KLT_SEL_TRACE=1 timeout -k 10 120 python3 tools/exp/replace_probe.py 12 > $OUT/probe.txt 2> $OUT/probe_trace.txt; tail -1 $OUT/probe.txt
bash archive/tools_exp/r04x.sh
