#!/bin/bash
# Config 4 projection at other chunk lengths (frames per exchange), margins
# grown with the chunk's motion (0.3 px/frame down: 64 frames ~ 19 rows):
# tools/shard_sim.py over the 1 001-frame sequence, worlds 1 and 8.
set -o pipefail
OUT=gpurun_out/${1:-r06ch}; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in ${CFGS:-"96:72" "128:80" "64:64"}; do
  ch=${cfg%%:*}; m=${cfg#*:}
  timeout -k 10 900 python3 -u tools/shard_sim.py --frames 1001 --chunk $ch --worlds 1 8 --margins $m --pass1-shared \
    > $OUT/chunk${ch}_m$m.log 2>&1 || { tail -20 $OUT/chunk${ch}_m$m.log; exit 1; }
  echo "chunk $ch margin $m:"; grep '^{"world"' $OUT/chunk${ch}_m$m.log | cut -c1-330
done
