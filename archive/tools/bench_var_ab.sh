#!/bin/bash
# bench value (1080p/5000, overlapped schedule) of the default library against
# variant builds (VARS -> lib/var/<name>/libklt_amd.so), three rounds
set -o pipefail
mkdir -p gpurun_out/bv
python3 -c "import ctypes; l=ctypes.CDLL('/opt/rocm/lib/libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); l.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)); print('stream priority range least', a.value, 'greatest', b.value)"
for r in 1 2 3; do for v in default $VARS; do
  if [ $v = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/$v/libklt_amd.so; fi
  timeout -k 10 300 python bench.py --no-cpu --no-4k --no-fast --api-frames 0 > gpurun_out/bv/$v.json 2>gpurun_out/bv/err.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bv/$v.json')); print('$v', round(d['value']), d['kernels_us_per_frame'])"
done; done
