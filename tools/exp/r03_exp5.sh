#!/bin/bash
# world-1 exchange cost of klt_shard_track; tracker PMC (k_track7) for profiles/pmc_tracker.json
set -o pipefail
OUT=gpurun_out/exp5; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/exp/exchange_w1.py > $OUT/exchange_w1.json 2> $OUT/exchange_w1.err || { tail -5 $OUT/exchange_w1.err; exit 1; }
cat $OUT/exchange_w1.json
bash tools/pmc_track.sh exp5/pmctrk > $OUT/pmc_track.log 2>&1 || { tail -20 $OUT/pmc_track.log; exit 1; }
tail -40 $OUT/pmc_track.log
