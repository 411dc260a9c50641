#!/bin/bash
# Round 4: host time inside klt_hip_track_frames (KLT_HOST_PROF variant build)
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast --steps 20 --warmup 5 --min-chunks 1 --serial"
for i in 1 2; do
  KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/hp/libklt_amd.so timeout -k 10 300 python3 bench.py $Q > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$i.json')); print(round(d['value']), d['timed_region_host'])"
  grep hostmark $OUT/b$i.err | head -24
done
for w in 1 2 4 8; do timeout -k 10 60 tools/hipbench/valu $w || exit 1; done
Q2="--no-cpu --api-frames 0 --no-4k --no-fast"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $Q2 --steps 20 --warmup 5 > $OUT/new_s20_$i.json 2> $OUT/new_s20_$i.err || { tail -5 $OUT/new_s20_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py $Q2 > $OUT/new_full_$i.json 2> $OUT/new_full_$i.err || { tail -5 $OUT/new_full_$i.err; exit 1; }
done
for f in $OUT/new_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), d['tracker']['kernel'], 'pmc' in d['tracker'], round(d['timed_region_host']['enqueue_us'],1))"; done
