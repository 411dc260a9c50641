#!/bin/bash
# Level 1 after every S frames' level 0 (KLT_PYR_SUB) in the 8-rank config-4
# schedule, where the chunk's level 1 otherwise runs alone after the tracker
# has finished (round-5 rank timeline): tools/shard_sim.py at 8 ranks with the
# all-gather as a 40 us in-stream stall, S = 0 (production) / 32 / 16,
# alternating, two rounds, one box.
set -o pipefail
OUT=gpurun_out/${1:-r06sub8}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for S in ${SUBS:-0 32 16}; do
    KLT_PYR_SUB=$S timeout -k 10 600 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds 8 --margins 64 --pass1-shared \
      --exchange-in-stream-us 40 > $OUT/sub${S}_r$round.log 2>&1 || { tail -20 $OUT/sub${S}_r$round.log; exit 1; }
    echo "round $round KLT_PYR_SUB=$S: $(grep '^{"world"' $OUT/sub${S}_r$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["us_per_frame_synced"],3), "us/frame synced, redone", d["chunks_redone_full_frame"], "digest", d["state_digest"])')"
  done
done
