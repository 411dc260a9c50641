#!/bin/bash
# Round 5: the multi-rank bench paths rehearsed on one GPU (KLT_BENCH_SHARE_GPU=1:
# every rank on GPU 0, gloo): config 5 (independent sequences) at N=2, and
# config 4 sharded (all-gather exchange, bands of equal built rows) at N=1, 2
# and 4 -- the state digests must agree.
set -o pipefail
OUT=gpurun_out/${1:-r05reh}; mkdir -p $OUT
export TMPDIR=/tmp
R="python3 -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
KLT_BENCH_SHARE_GPU=1 timeout -k 10 400 $R --nproc-per-node 2 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-4k --no-fast --api-frames 0 > $OUT/c5_n2.json 2> $OUT/c5_n2.err || { tail -20 $OUT/c5_n2.err; exit 1; }
tail -1 $OUT/c5_n2.json | cut -c1-300
timeout -k 10 400 python3 bench.py --mode sharded --steps 128 --warmup 5 > $OUT/c4_n1.json 2> $OUT/c4_n1.err || { tail -20 $OUT/c4_n1.err; exit 1; }
tail -1 $OUT/c4_n1.json | cut -c1-600
for n in 2 4; do
  KLT_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --nproc-per-node $n --master-port 2953$n bench.py --mode sharded --gpus $n --steps 128 --warmup 5 > $OUT/c4_n$n.json 2> $OUT/c4_n$n.err || { tail -20 $OUT/c4_n$n.err; exit 1; }
  tail -1 $OUT/c4_n$n.json | cut -c1-600
done
