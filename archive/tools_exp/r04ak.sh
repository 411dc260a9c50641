#!/bin/bash
# Round 4: per-call frames uploaded in row bands on the copy stream, each
# band's level-0 tiles launched once it has landed (KLT_UPLOAD_BANDS, default
# 4; 1 = one DMA on the tracking stream): parity, then the API legs A/B
set -o pipefail
OUT=gpurun_out/r04ak; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_track.py tests/test_gpu_select.py tests/test_abi.py tests/test_io.py "tests/test_gpu_long.py::test_replace_harness_config3r" "tests/test_gpu_long.py::test_track_features_per_call_config2" tests/test_affine.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for nb in 4 1 2 4 1 2; do
  KLT_UPLOAD_BANDS=$nb timeout -k 10 300 python3 bench.py $Q > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json'))['api']; print('bands=$nb', {k: (round(v['value']), round(v.get('us_per_call_median', 0))) for k,v in d.items() if isinstance(v, dict) and 'value' in v}, d['replace']['parity']['columns_mismatched'])"
done
