set -o pipefail
OUT=gpurun_out/v9b; mkdir -p $OUT
for c in 64 96 128 164; do
timeout -k 10 300 python bench.py --no-cpu --chunk $c > $OUT/b$c.json 2> $OUT/b$c.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/b$c.json')); print($c, round(d['value']), round(d['ms_per_step']*1000,2), d['kernels_us_per_frame'])"
done
