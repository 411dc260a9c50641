#!/bin/bash
# Round 4: per-call uploads with ROCclr's blit kernels instead of the SDMA
# engine (GPU_FORCE_BLIT_COPY_SIZE in KB: copies up to that size run as
# kernels on the stream's own queue), the bench's API legs, alternating
set -o pipefail
OUT=gpurun_out/r04au; mkdir -p $OUT
export TMPDIR=/tmp
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for b in 0 4096 0 4096 0 4096; do
  E=""; [ $b != 0 ] && E="GPU_FORCE_BLIT_COPY_SIZE=$b"
  env $E timeout -k 10 300 python3 bench.py $Q > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; D=json.load(open('$OUT/b.json')); d=D['api']; print('blit=$b', round(D['value']), {k: (round(v['value']), round(v.get('us_per_call_median', 0))) for k,v in d.items() if isinstance(v, dict) and 'value' in v})"
done
