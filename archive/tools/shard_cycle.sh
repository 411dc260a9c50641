#!/bin/bash
# sharded mode: GPU tests, N=1 bench at config 4, and a 2-rank rehearsal on one GPU (gloo)
OUT=gpurun_out/${1:-shard}; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_shard.py -q -x --timeout 300 -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --mode sharded --steps 128 --warmup 32 > $OUT/n1.json 2> $OUT/n1.err || exit $?
cat $OUT/n1.json
KLT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode sharded --gpus 2 --steps 128 --warmup 32 > $OUT/n2.json 2> $OUT/n2.err || exit $?
cat $OUT/n2.json
