#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer over the host C layer
# (klt_api.c, klt_io.c, klt_select.c, klt_synth.c) and the oracle
# (oracle/klt_oracle.c), driven by the whole CPU test suite.  No GPU: every
# device call fails and the klt.h layer reports it through KLTError, which the
# suite's no-GPU test expects.  The HIP object is linked unsanitized.
# usage: bash tools/hostcheck/asan_ubsan.sh   (CPU only; writes a log under /tmp)
set -eo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
make -s -C "$R/klt-feature-tracker-acceleration-gpus_amd/csrc" all asan
make -s -C "$R/oracle" all asan
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export KLT_AMD_LIB="$R/klt-feature-tracker-acceleration-gpus_amd/lib/asan/libklt_amd.so"
export KLT_ORACLE_LIB="$R/oracle/build/asan/libklt_oracle.so"
cd "$R"
python -m pytest tests -m "not gpu" -q -p no:cacheprovider -x "$@"
