#!/bin/bash
# kernel timeline of the slowest 8-rank replay (4K/20k, 64-frame chunks, build-ahead)
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python tools/shard_sim.py --worlds 8 --frames 257 --chunk 64 --margins 64 --lazy-flag \
  --keep-states $OUT/st > $OUT/s.log 2>&1 || { tail -5 $OUT/s.log; exit 1; }
grep '^{"world' $OUT/s.log
R=$(python3 -c "
import json
d=json.loads([l for l in open('$OUT/s.log') if l.startswith('{\"workload')][0])
r=d['runs'][0]; print(max(r['per_rank_us_per_frame'], key=lambda q: q['wall'])['rank'])")
echo slowest rank $R
for mode in "" "--no-ahead"; do
  tag=p${mode:+_serial}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$tag -o run -- python tools/shard_sim.py \
    --replay $OUT/st/states_w8.npz --rank $R --worlds 8 --frames 257 --chunk 64 --lazy-flag $mode > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  tail -1 $OUT/$tag.log
  python3 tools/exp/timeline.py $(find $OUT/$tag -name "*kernel_trace.csv") > $OUT/${tag}_timeline.txt || exit 1
  tail -12 $OUT/${tag}_timeline.txt
done
rm -rf $OUT/st
