#!/bin/bash
# A/B of bench.py's bank pre-touch for a capped timed region (--steps 20, the
# driver's shape) against the default run, on one box.
set -o pipefail
TAG=${1:-pretouch}; OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for opt in "" "--no-pretouch" "" "--no-pretouch" "FULL"; do
  i=$((i+1))
  if [ "$opt" = FULL ]; then a=""; else a="--steps 20 --warmup 5 $opt"; fi
  timeout -k 10 300 python bench.py $a --no-cpu --no-fast --api-frames 0 --replace-frames 0 > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  python3 - $OUT/b$i.json "$opt" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(repr(sys.argv[2]), "value", round(d["value"]), "roof", round(d["roofline"]["frac"], 3),
      {k: round(v, 2) for k, v in d["kernels_us_per_frame"].items() if v}, "4k", round(d["roofline_4k"]["frac"], 3))
PY
done
