#!/bin/bash
# Round 4: the driver-shaped timed region after the single-chunk schedule and
# the prebuilt call arguments (host marks, kernel trace), the replay warm-up's
# effect on the driver-vs-default roofline gap, and the tracker PMC refresh.
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast"
KLT_AMD_LIB=$PWD/klt-feature-tracker-acceleration-gpus_amd/lib/var/hp/libklt_amd.so timeout -k 10 300 python3 bench.py $Q --steps 20 --warmup 5 > $OUT/hp.json 2> $OUT/hp.err || { tail -5 $OUT/hp.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/hp.json')); print('hp', round(d['value']), d['timed_region_host'])"
grep hostmark $OUT/hp.err | head -40
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run --output-format csv -- python3 bench.py $Q --steps 20 --warmup 5 > $OUT/kt.json 2> $OUT/kt.err || { tail -5 $OUT/kt.err; exit 1; }
python3 tools/region_marks.py $OUT/kt.json $(find $OUT/kt -name "*kernel_trace.csv")
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $Q --steps 20 --warmup 5 > $OUT/s20_$i.json 2> $OUT/s20_$i.err || { tail -5 $OUT/s20_$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py $Q > $OUT/full_$i.json 2> $OUT/full_$i.err || { tail -5 $OUT/full_$i.err; exit 1; }
done
for f in $OUT/s20_*.json $OUT/full_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3), d['replay']['warmup']['runs'], round(d['timed_region_host']['enqueue_us'],1))"; done
bash tools/pmc_track.sh r04e/pmctrk > $OUT/pmctrk.log 2>&1 || { tail -20 $OUT/pmctrk.log; exit 1; }
tail -30 $OUT/pmctrk.log
