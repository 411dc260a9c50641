#!/bin/bash
# Round 4: the multi-rank bench paths after the round-4 harness changes,
# rehearsed on one GPU (KLT_BENCH_SHARE_GPU=1: both ranks on GPU 0, gloo):
# config 5 (independent sequences) at N=2, and config 4 sharded at N=1 and N=2
# (state digests must agree)
set -o pipefail
OUT=gpurun_out/r04ag; mkdir -p $OUT
export TMPDIR=/tmp
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
KLT_BENCH_SHARE_GPU=1 timeout -k 10 400 $R --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-4k --no-fast --api-frames 0 > $OUT/c5_n2.json 2> $OUT/c5_n2.err || { tail -20 $OUT/c5_n2.err; exit 1; }
tail -1 $OUT/c5_n2.json | cut -c1-300
timeout -k 10 400 python3 bench.py --mode sharded --steps 128 --warmup 5 > $OUT/c4_n1.json 2> $OUT/c4_n1.err || { tail -20 $OUT/c4_n1.err; exit 1; }
tail -1 $OUT/c4_n1.json | cut -c1-400
KLT_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --master-port 29532 bench.py --mode sharded --gpus 2 --steps 128 --warmup 5 > $OUT/c4_n2.json 2> $OUT/c4_n2.err || { tail -20 $OUT/c4_n2.err; exit 1; }
tail -1 $OUT/c4_n2.json | cut -c1-400
