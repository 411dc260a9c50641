#!/bin/bash
# Round 4: REPLACE by the device/host segment threshold now that refinements
# are graph launches (KLT_AMD_SELECT_THRESHOLD; default 32768)
set -o pipefail
OUT=gpurun_out/r04ah2; mkdir -p $OUT
export TMPDIR=/tmp
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for T in 49152 65536 32768 49152 65536 32768; do
  KLT_AMD_SELECT_THRESHOLD=$T timeout -k 10 300 python3 bench.py $Q > $OUT/t.json 2> $OUT/t.err || { tail -5 $OUT/t.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/t.json'))['api']['replace']; print('T=$T', round(d['value']), round(d['us_per_replace_median']), d['parity']['columns_mismatched'], {k: round(v) for k, v in d['select_median'].items()})"
done
