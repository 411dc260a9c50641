#!/bin/bash
# Round 4: the 489-frame default region by schedule: 64-frame chunks with the
# next chunk's pyramids overlapped (default) vs longer chunks on one stream
set -o pipefail
OUT=gpurun_out/r04ae; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast"
for cfg in "d" "128 s" "489 s" "d" "128 s" "489 s"; do
  set -- $cfg
  A=""; [ "$1" != d ] && A="--chunk $1 --serial"
  timeout -k 10 300 python3 bench.py $Q $A > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$cfg', round(d['value']), round(d['ms_per_step']*1e3,2), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, d['config'].get('schedule', d['config'])['chunk'] if isinstance(d['config'].get('schedule'), dict) else '')" 2>/dev/null || python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$cfg', round(d['value']), round(d['ms_per_step']*1e3,2))"
done
