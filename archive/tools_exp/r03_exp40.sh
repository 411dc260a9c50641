#!/bin/bash
# k_track7 fast-sum instance (DPP tree): tolerance and tracker tests, then the bench's exact and fast legs
set -o pipefail
OUT=gpurun_out/exp40; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_track.py tests/test_shard.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error|assert" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cat fast_tolerance_config2.json fast_tolerance_config3.json 2>/dev/null | head -c 600; echo
for r in 1 2; do
timeout -k 10 400 python bench.py --no-cpu --api-frames 0 --replace-frames 0 --no-4k > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b.json')); f=d['fast']; print('exact', round(d['value']), 'trk', round(d['kernels_us_per_frame']['k_track'],2), '| fast', round(f['value']), 'trk', round(f['k_track_us_per_frame'],2), f['vs_exact'])"
done
timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 --reduction fast > $OUT/t.json || exit 1
python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/2500 fast trk', round(d['track_us_per_frame'],2))"
timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 > $OUT/t.json || exit 1
python3 -c "import json; d=json.load(open('$OUT/t.json')); print('4K/2500 exact trk', round(d['track_us_per_frame'],2))"
