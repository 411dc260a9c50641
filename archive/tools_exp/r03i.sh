#!/bin/bash
# faster k_band_order: tracker/shard tests, config-4 rank simulation at config 4's 1000 frames, and the 8-rank timeline
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python tools/shard_sim.py --worlds 1 8 --frames 1001 --chunk 64 --margins 64 --lazy-flag --keep-states $OUT/st > $OUT/s1000.log 2>&1 || { tail -5 $OUT/s1000.log; exit 1; }
grep '^{"world' $OUT/s1000.log
R=$(python3 -c "
import json
d=json.loads([l for l in open('$OUT/s1000.log') if l.startswith('{\"workload')][0])
r=d['runs'][1]; print(max(r['per_rank_us_per_frame'], key=lambda q: q['wall'])['rank'])")
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o run -- python tools/shard_sim.py \
    --replay $OUT/st/states_w8.npz --rank $R --worlds 8 --frames 1001 --chunk 64 --lazy-flag > $OUT/p.log 2>&1 || { tail -5 $OUT/p.log; exit 1; }
python3 tools/exp/timeline.py $(find $OUT/p -name "*kernel_trace.csv") > $OUT/p_timeline.txt || exit 1
grep order $OUT/p_timeline.txt | tail -5
rm -rf $OUT/st
