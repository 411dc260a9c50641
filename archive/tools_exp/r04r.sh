#!/bin/bash
# Round 4: the shard failure agreement under fault injection (world-1 RCCL)
# and the shard tests, then the bench's API legs (archive/tools_exp/r04q.sh)
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_shard.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/shard.log 2>&1 || { tail -30 $OUT/shard.log; exit 1; }
tail -3 $OUT/shard.log
bash archive/tools_exp/r04q.sh
