#!/bin/bash
OUT=gpurun_out/${1:-ser}; mkdir -p $OUT
for args in "--chunk 16 --no-patch --serial" "--chunk 16 --serial" "--chunk 16 --no-patch" "--chunk 4 --no-patch --serial" "--chunk 64 --no-patch --serial" "--chunk 16 --no-patch --serial --input-order"; do
  timeout -k 10 300 python tools/microbench.py frames --frames 129 --reps 3 $args > $OUT/last.json || exit 1
  echo "$args" $(python3 -c "import json; d=json.load(open('$OUT/last.json')); print(round(d['us_per_frame_wall'],2), round(d['l0_us_per_frame'],2), round(d['l1_us_per_frame'],2), round(d['track_us_per_frame'],2))") | tee -a $OUT/sweep.txt
done
export KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/prof/libklt_amd.so
timeout -k 10 300 python tools/microbench.py frames --frames 129 --reps 2 --chunk 16 --prof --no-patch --serial > $OUT/prof.json || exit 1
python3 -c "
import json; d=json.load(open('$OUT/prof.json'))
for k in ('prof_cycles_per_wave_frame','prof_wave_life_us','prof_end_us_pct','us_per_frame_wall','track_us_per_frame'):
    print('  ', k, d.get(k))"
