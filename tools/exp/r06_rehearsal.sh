#!/bin/bash
# the driver's own multi-GPU command shape, rehearsed on
# one GPU (KLT_BENCH_SHARE_GPU=1: every rank on GPU 0, gloo): bench.py --gpus N
# at N = 1, 2 and 4 must print sharded_4k (config 4 sharded over the N ranks)
# with parity.columns_mismatched 0 and the same state digest at every N.
set -o pipefail
OUT=gpurun_out/${1:-r06reh}; mkdir -p $OUT
export TMPDIR=/tmp
R="python3 -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
FAST="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast --api-frames 0 --replace-frames 0"
a=$(date +%s)
timeout -k 10 300 python3 bench.py $FAST > $OUT/n1.json 2> $OUT/n1.err || { tail -20 $OUT/n1.err; exit 1; }
echo "n1 wall_s=$(( $(date +%s) - a ))"
# one rank through torch.distributed.run: the sharded_4k all-gather runs through RCCL
a=$(date +%s)
timeout -k 10 300 $R --nproc-per-node 1 --master-port 29540 bench.py --gpus 1 $FAST > $OUT/n1rccl.json 2> $OUT/n1rccl.err \
  || { tail -20 $OUT/n1rccl.err; exit 1; }
echo "n1rccl wall_s=$(( $(date +%s) - a ))"
for n in 2 4; do
  a=$(date +%s)
  KLT_BENCH_SHARE_GPU=1 timeout -k 10 600 $R --nproc-per-node $n --master-port 2954$n bench.py --gpus $n $FAST \
    > $OUT/n$n.json 2> $OUT/n$n.err || { tail -20 $OUT/n$n.err; exit 1; }
  echo "n$n wall_s=$(( $(date +%s) - a ))"
done
for n in 1 1rccl 2 4; do
python3 - $OUT/n$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["sharded_4k"]
print(sys.argv[1], "value", round(d["value"]), "sharded_4k", round(s["value"]), "us/frame", round(s["us_per_frame"], 2),
      "ranks", s["n_gpus"], "rank_us", [round(u, 2) for u in s["rank_us_per_frame"]],
      "allgather_us", round(s["exchange"]["allgather_us_per_chunk_median"], 1), s["exchange"]["allgather_op"],
      "parity", s["parity"]["columns_mismatched"], "redone", s["chunks_redone_full_frame"], "digest", s["state_digest"][:16],
      "agree", s["ranks_agree_on_state"])
PY
done
