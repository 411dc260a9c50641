# track7 (impl 0) vs generic tracker (impl 1): 1080p/5000 and 4K/2500, 64-frame launches
set -o pipefail
for r in 1 2; do for impl in 0 1; do
  timeout -k 5 120 python tools/microbench.py frames --frames 129 --reps 2 --chunk 64 --impl $impl > gpurun_out/t7.json || exit 1
  a=$(python3 -c "import json; d=json.load(open('gpurun_out/t7.json')); print(round(d['track_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --width 3840 --height 2160 --features 2500 --frames 129 --reps 2 --chunk 64 --impl $impl > gpurun_out/t7.json || exit 1
  b=$(python3 -c "import json; d=json.load(open('gpurun_out/t7.json')); print(round(d['track_us_per_frame'],2))")
  timeout -k 5 120 python tools/microbench.py frames --features 1000 --frames 129 --reps 2 --chunk 64 --impl $impl > gpurun_out/t7.json || exit 1
  c=$(python3 -c "import json; d=json.load(open('gpurun_out/t7.json')); print(round(d['track_us_per_frame'],2))")
  echo "impl=$impl 1080p/5000 $a  4K/2500 $b  1080p/1000 $c"
done; done
