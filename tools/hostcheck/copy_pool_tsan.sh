#!/bin/bash
# ThreadSanitizer run of the copy pool (host code only; no GPU needed):
# runtime.hip compiled with -Xarch_host -fsanitize=thread, linked with the
# kernel and host objects of the library and a driver calling klt_hip_selftest_copy_pool.
# usage: bash tools/hostcheck/copy_pool_tsan.sh   (after make -C .../csrc)
set -eo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/klt-feature-tracker-acceleration-gpus_amd/csrc
O=$R/klt-feature-tracker-acceleration-gpus_amd/lib/obj
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O1 -g --offload-arch=gfx950 -ffp-contract=off -std=c++17 -w -I$R/include -I$C \
  -Xarch_host -fsanitize=thread -c $C/runtime.hip -o $T/k.o
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -fsanitize=thread -c $R/tools/hostcheck/copy_pool_tsan.cpp -o $T/main.o
/opt/rocm/lib/llvm/bin/clang++ -fsanitize=thread -o $T/t $T/main.o $T/k.o $O/pyramid.o $O/track.o $O/affine.o $O/klt_api.o $O/klt_io.o \
  $O/klt_select.o $O/klt_synth.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lm -lpthread
TSAN_OPTIONS=halt_on_error=1 $T/t
rm -rf $T
