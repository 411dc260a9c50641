#!/bin/bash
# Round 4: KLTTrackSequence leg after the selection engine stopped creating
# streams (graphs built node by node; downloads on the selection stream)
set -o pipefail
OUT=gpurun_out/r04ac3; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_select.py tests/test_gpu_select_engine.py "tests/test_gpu_long.py::test_replace_harness_config3r" "tests/test_gpu_track.py::test_track_sequence_api_vs_loop" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for cfg in a b c; do
  timeout -k 10 300 python3 bench.py $Q > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json'))['api']; print('dl=$cfg', {k: round(v['value']) for k,v in d.items() if isinstance(v, dict) and 'value' in v}, round(d['replace']['us_per_replace_median']), d['replace']['parity']['columns_mismatched'])"
done
