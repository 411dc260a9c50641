#!/bin/bash
# the built-ahead bank handed to the next tracker by
# hipStreamWriteValue32 / hipStreamWaitValue32 on signal memory
# (KLT_WAIT_VALUE=1) instead of ev_bbuilt + hipStreamWaitEvent: config 4 at 8
# ranks, tools/shard_sim.py, alternating, two rounds on one box.
set -o pipefail
OUT=gpurun_out/${1:-r06wv}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for wv in 0 1; do
    KLT_WAIT_VALUE=$wv timeout -k 10 600 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds ${WORLDS:-8} \
      --margins 64 --pass1-shared > $OUT/wv${wv}_r$round.log 2>&1 || { tail -20 $OUT/wv${wv}_r$round.log; exit 1; }
    echo "round $round KLT_WAIT_VALUE=$wv: $(grep "^{\"world\"" $OUT/wv${wv}_r$round.log | cut -c1-330)"
  done
done
