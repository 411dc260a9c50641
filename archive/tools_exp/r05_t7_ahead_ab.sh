#!/bin/bash
# Round 5: k_track7 fetching the finest level.s first corners ahead (KLT_T7_AHEAD=1, default
# build: image 1 carried from the previous frame, image 2 at the predicted position) against
# none (lib/var/ah0, make variant NAME=ah0
# DEFS=-DKLT_T7_AHEAD=0): tracker parity first, then tracker time per frame
# (tools/microbench.py frames, 1080p/5000 and 4K/2500, 64-frame chunks, two
# alternating rounds), then the config-4 8-rank simulation with each build.
set -o pipefail
OUT=gpurun_out/${1:-r05t7}; mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/ah0/libklt_amd.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "track or long or sequence or shard" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for lib in default ah0; do
    for shape in "--width 1920 --height 1080 --features 5000" "--width 3840 --height 2160 --features 2500"; do
      if [ $lib = default ]; then unset KLT_AMD_LIB; else export KLT_AMD_LIB=$V; fi
      timeout -k 10 300 python3 tools/microbench.py frames $shape --chunk 64 --frames 129 --reps 3 --table > $OUT/mb.json 2>> $OUT/mb.err || { tail -5 $OUT/mb.err; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open('$OUT/mb.json').read().strip().splitlines()[-1])
k={kk:round(v,3) for kk,v in d.items() if 'track' in kk and isinstance(v,(int,float))}
print('round $round', '$lib', '$shape', k)" | tee -a $OUT/ab.txt
    done
  done
done
unset KLT_AMD_LIB
for lib in default ah0; do
  if [ $lib = ah0 ]; then export KLT_AMD_LIB=$V; fi
  timeout -k 10 600 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds 1 8 --margins 64 --pass1-shared \
    > $OUT/shard8_$lib.log 2>&1 || { tail -20 $OUT/shard8_$lib.log; exit 1; }
  grep '"world": 8' $OUT/shard8_$lib.log | cut -c1-260 | sed "s/^/$lib /" | tee -a $OUT/ab.txt
done
