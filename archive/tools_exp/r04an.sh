#!/bin/bash
# Round 4: k_track7 packed (gx, gy) pairs (KLT_T7_PK) and all 13 ordered-sum
# reads in flight (KLT_T7_BATCH=13): tracker parity on the pk build, then the
# tracker A/B (archive/tools/track_ab.sh) against the default build
set -o pipefail
mkdir -p gpurun_out/r04an
KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/pkb13/libklt_amd.so timeout -k 10 400 python3 -u -m pytest \
  tests/test_gpu_track.py tests/test_gpu_long.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04an/tests.log 2>&1 || { tail -20 gpurun_out/r04an/tests.log; exit 1; }
tail -1 gpurun_out/r04an/tests.log
VARS="pk b13 pkb13" bash archive/tools/track_ab.sh
