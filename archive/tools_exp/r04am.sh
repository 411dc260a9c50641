#!/bin/bash
# Round 4: per-call pageable uploads by host copy workers / piece size
# (KLT_AMD_HOST_THREADS, KLT_AMD_COPY_PIECE): the bench's per-call legs
set -o pipefail
OUT=gpurun_out/r04am2; mkdir -p $OUT
export TMPDIR=/tmp
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for cfg in "3 32768" "5 32768" "7 32768" "5 65536" "3 65536" "7 65536" "5 32768"; do
  set -- $cfg
  KLT_AMD_HOST_THREADS=$1 KLT_AMD_COPY_PIECE=$2 timeout -k 10 300 python3 bench.py $Q > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json'))['api']; print('threads=$1 piece=$2', {k: (round(v['value']), round(v.get('us_per_call_median', 0))) for k,v in d.items() if isinstance(v, dict) and 'value' in v and k != 'replace'})"
done
