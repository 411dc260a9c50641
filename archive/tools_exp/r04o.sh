#!/bin/bash
# Round 4: host sort on the box's CPU (branch-free exact partition), REPLACE
# engine timeline with pivots returned by the device state
set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
export TMPDIR=/tmp
g++ -O3 -pthread -Iklt-feature-tracker-acceleration-gpus_amd/csrc tools/hostcheck/sortbench.cpp -o $OUT/sortbench || exit 1
timeout -k 10 120 $OUT/sortbench | tee $OUT/sortbench.txt || exit 1
KLT_SEL_TRACE=1 timeout -k 10 120 python3 tools/exp/replace_probe.py 12 > $OUT/replace.log 2>&1 || { tail -5 $OUT/replace.log; exit 1; }
tail -22 $OUT/replace.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_select.py tests/test_gpu_select_engine.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
