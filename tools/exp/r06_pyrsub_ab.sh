#!/bin/bash
# level 1 run per sub-batch of S frames right after their
# level 0 (KLT_PYR_SUB=S), so that it may read the sigma-3.6 row pass (hs)
# from the MALL; S = 0 is the production build (whole 64-frame batches).
# tools/microbench.py frames at 4K (pyramids only, and 20 000 features
# tracked) and 1080p (pyramids only), two alternating rounds on one box.
set -o pipefail
OUT=gpurun_out/${1:-r06ps}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for S in ${SUBS:-0 16 8}; do
    for shape in "4k_pyr:--width 3840 --height 2160 --features 20000 --pyr-only" \
                 "4k_trk:--width 3840 --height 2160 --features 20000 --table" \
                 "1080_pyr:--width 1920 --height 1080 --features 5000 --pyr-only"; do
      lab=${shape%%:*}; args=${shape#*:}
      KLT_PYR_SUB=$S timeout -k 10 200 python3 tools/microbench.py frames --chunk 64 --frames 193 --reps 3 $args \
        > $OUT/ps_${lab}_S$S.json 2> $OUT/ps_${lab}_S$S.err || { tail -10 $OUT/ps_${lab}_S$S.err; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open('$OUT/ps_${lab}_S$S.json').read().strip().splitlines()[-1])
print('round $round S=$S $lab', 'wall_us/frame', round(d['us_per_frame_wall'],2), 'l0', round(d['l0_us_per_frame'],2), 'l1', round(d['l1_us_per_frame'],2), 'trk', round(d['track_us_per_frame'],2))"
    done
  done
done
