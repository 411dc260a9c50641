#!/bin/bash
# Round 4, first look: the driver-shaped bench (--steps 20 --warmup 5) under
# several timed-region schedules, its kernel timeline, and the shader clock of
# each replay launch (GRBM_GUI_ACTIVE / 8 / duration) in the --steps 20 and
# the 489-frame shapes.  usage (via gpurun): bash archive/tools_exp/r04a.sh
set -o pipefail
OUT=gpurun_out/r04a; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --api-frames 0 --no-4k --no-fast"
run() { local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$tag.json')); print('$tag', round(d['value']), d['config']['chunk'], d['config']['schedule'][:60], {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v}, round(d['roofline']['frac'],3))"
}
run s20_default --steps 20 --warmup 5 $Q
run s20_one --steps 20 --warmup 5 --min-chunks 1 $Q
run s20_one_serial --steps 20 --warmup 5 --min-chunks 1 --serial $Q
run s20_c5 --steps 20 --warmup 5 --chunk 5 $Q
run s20_c4 --steps 20 --warmup 5 --chunk 4 $Q
run s20_default_b --steps 20 --warmup 5 $Q
run full $Q
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $Q > $OUT/kt20.json 2> $OUT/kt20.err || { tail -5 $OUT/kt20.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $OUT/clk20 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $Q > $OUT/clk20.json 2> $OUT/clk20.err || { tail -5 $OUT/clk20.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $OUT/clkfull -o run --output-format csv -- python3 bench.py $Q > $OUT/clkfull.json 2> $OUT/clkfull.err || { tail -5 $OUT/clkfull.err; exit 1; }
find $OUT -name "*.csv" | head -20
