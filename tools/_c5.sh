set -o pipefail
mkdir -p gpurun_out/c5
KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib//libklt_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c5/t.log 2>&1; rc=$?; tail -3 gpurun_out/c5/t.log; [ $rc -ne 0 ] && exit $rc
bash tools/l0_var.sh l0v5 stg32 stg127
