#!/bin/bash
# Round 4: pooled host sort with spinning workers: sortbench on the box, REPLACE at depth 3 / 4, parity
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
export TMPDIR=/tmp
g++ -O3 -pthread -Iklt-feature-tracker-acceleration-gpus_amd/csrc tools/hostcheck/sortbench.cpp -o $OUT/sortbench || exit 1
timeout -k 10 120 $OUT/sortbench | tee $OUT/sortbench.txt || exit 1
for d in 4 3 4 3; do
  KLT_AMD_SORT_DEPTH=$d KLT_SEL_TRACE=1 timeout -k 10 120 python3 tools/exp/replace_probe.py 12 > $OUT/replace_$d.log 2>&1 || { tail -5 $OUT/replace_$d.log; exit 1; }
  echo "depth $d: $(tail -1 $OUT/replace_$d.log)"; grep "sort len" $OUT/replace_$d.log | tail -4
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_select.py tests/test_gpu_select_engine.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
