set -o pipefail
mkdir -p gpurun_out/c6
timeout -k 10 300 python -u -m pytest tests/test_affine.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c6/t.log 2>&1; rc=$?; tail -25 gpurun_out/c6/t.log; exit $rc
