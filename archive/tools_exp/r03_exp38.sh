#!/bin/bash
# level-0 interleaved tile staged in LDS, whole-row nontemporal stores (this build) vs direct 8-byte nontemporal stores (variant ad0)
set -o pipefail
OUT=gpurun_out/exp38; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_shard.py tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for r in 1 2 3 4; do
  if [ $((r % 2)) = 1 ]; then order="new ad0"; else order="ad0 new"; fi
  for m in $order; do
    if [ $m = new ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/ad0/libklt_amd.so; fi
    timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 20000 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
    b=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/20k l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
    timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
    a=$(python3 -c "import json; d=json.load(open('$OUT/t.json')); print('1080p l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2))")
    echo "$m | $b | $a"
  done
done
for m in new ad0; do
  if [ $m = new ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$L/var/ad0/libklt_amd.so; fi
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$m -o run -- python tools/microbench.py frames --width 3840 --height 2160 --frames 129 --reps 1 --chunk 64 --pyr-only > $OUT/w_$m.log 2>&1 || { tail -5 $OUT/w_$m.log; exit 1; }
  python3 - $OUT/w_$m/run_counter_collection.csv $m <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "k_pyr_l0" in r["Kernel_Name"] and int(r["Grid_Size"]) > 40000000]
print(sys.argv[2], "l0 WRITE_SIZE per 64-frame 4K launch", [round(x) for x in v])
PY
done
