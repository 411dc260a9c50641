#!/bin/bash
# k_track7 band test as integer compares: 8-rank config-4 simulation A/B, shard/long tests
set -o pipefail
OUT=gpurun_out/r03x; mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib
for rep in 1 2; do
for lib in libklt_amd.so var/old/libklt_amd.so; do
  KLT_AMD_LIB=$L/$lib timeout -k 10 400 python tools/shard_sim.py --worlds 8 --frames 257 --chunk 64 --margins 64 --lazy-flag --pass1-shared > $OUT/s.log 2>&1 || { tail -5 $OUT/s.log; exit 1; }
  echo "$lib" $(python3 - $OUT/s.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
r = d["runs"][0]
q = max(r["per_rank_us_per_frame"], key=lambda q: q["wall"])
print("max %.2f trk %.2f l0 %.2f digest %d redo %d" % (q["wall"], q["replay_kernels"]["k_track"], q["replay_kernels"]["k_pyr_l0"], r["state_digest"], r["chunks_redone_full_frame"]))
PY
)
done
done
timeout -k 10 600 python -u -m pytest tests/test_shard.py tests/test_gpu_long.py tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
