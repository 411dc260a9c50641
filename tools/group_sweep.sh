#!/bin/bash
OUT=gpurun_out/${1:-grp}; mkdir -p $OUT
run() { timeout -k 10 300 python tools/microbench.py "$@" > $OUT/last.json || exit 1; echo "$*" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print({k: (round(v, 2) if isinstance(v, float) else v) for k, v in d.items() if k not in ('mode','resolution','reps','status_hist')})") | tee -a $OUT/sweep.txt; }
run frames --frames 129 --reps 3 --chunk 16
run frames --frames 129 --reps 3 --chunk 16 --no-patch
run track --features 5000
run track --features 5000 --no-patch
run frames --frames 65 --reps 3 --chunk 16 --width 3840 --height 2160 --features 20000
run frames --frames 65 --reps 3 --chunk 16 --width 3840 --height 2160 --features 20000 --no-patch
