#!/bin/bash
# A/B of the tracker's wave priority (KLT_TRACK_PRIO, an env switch of the
# experiment build; now klt_hip_set_track_prio, default on): the 1080p bench
# (next chunk's pyramids overlapped with tracking) and the config-4 rank
# simulation (band pyramids built ahead while a rank tracks).
set -o pipefail
OUT=gpurun_out/${1:-prio}; mkdir -p $OUT
for p in 0 1 0 1; do
  KLT_TRACK_PRIO=$p timeout -k 10 300 python bench.py --no-cpu --api-frames 0 --no-fast --no-4k --replace-frames 0 \
    > $OUT/bench_p$p.json 2> $OUT/bench_p$p.err || { tail -5 $OUT/bench_p$p.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_p$p.json')); print('prio $p', round(d['value']), d['kernels_us_per_frame'])"
done
for p in 0 1; do
  KLT_TRACK_PRIO=$p timeout -k 10 500 python tools/shard_sim.py --worlds 1 8 --frames 257 --chunk 64 --margins 64 32 \
    > $OUT/shard_p$p.log 2>&1 || { tail -5 $OUT/shard_p$p.log; exit 1; }
  echo "prio $p"; grep '^{"world' $OUT/shard_p$p.log
done
