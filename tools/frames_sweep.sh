#!/bin/bash
# batched-sequence sweep: bash tools/frames_sweep.sh [tag]
OUT=gpurun_out/${1:-frm}; mkdir -p $OUT
for args in "--chunk 1" "--chunk 4" "--chunk 16" "--chunk 32" "--chunk 64" \
            "--width 3840 --height 2160 --features 20000 --chunk 16 --frames 65"; do
  timeout -k 10 300 python tools/microbench.py frames --frames 129 --reps 3 $args > $OUT/last.json || exit 1
  python3 -c "import json; d=json.load(open('$OUT/last.json')); print('$args', {k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items() if k not in ('mode',)})" | tee -a $OUT/sweep.txt
done
