#!/bin/bash
# Round 4 close: the driver's exact command (bench.py --gpus 1 --steps 20
# --warmup 5) three times in a row on one box, for the spread of `value` and
# of the roofline fraction the driver will record
set -o pipefail
OUT=gpurun_out/r04ay; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$i.json')); print('run $i', round(d['value']), 'ms/step', round(d['ms_per_step'],5), 'roof', round(d['roofline']['frac'],3), '4k', round(d['roofline_4k']['frac'],3), 'po', round(d['roofline_4k']['pyramids_only']['frac'],3), 'k', {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, 'parity', d.get('parity',{}).get('mismatches', d.get('parity',{}).get('ok')))"
done
