#!/bin/bash
# Round 4: REPLACE engine timeline (KLT_SEL_TRACE), per-call KLTTrackFeatures
# timeline (registered buffers), pyramid-pass HBM traffic refresh (1080p, 4K)
set -o pipefail
OUT=gpurun_out/r04n; mkdir -p $OUT
export TMPDIR=/tmp
KLT_SEL_TRACE=1 timeout -k 10 120 python3 tools/exp/replace_probe.py 12 > $OUT/replace.log 2>&1 || { tail -5 $OUT/replace.log; exit 1; }
tail -40 $OUT/replace.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/api -o run -- python3 tools/api_timeline.py run --register --frames 60 > $OUT/api.log 2>&1 || { tail -5 $OUT/api.log; exit 1; }
python3 tools/api_timeline.py summary $OUT/api > $OUT/api_summary.txt 2>&1 || { tail -5 $OUT/api_summary.txt; exit 1; }
cat $OUT/api_summary.txt
bash tools/pmc_traffic.sh r04n/traffic1080 > $OUT/traffic1080.log 2>&1 || { tail -5 $OUT/traffic1080.log; exit 1; }
python3 tools/pmc_traffic_json.py gpurun_out/r04n/traffic1080 1920 1080 $OUT/pmc_1080.json > /dev/null || exit 1
bash tools/pmc_traffic.sh r04n/traffic4k --width 3840 --height 2160 > $OUT/traffic4k.log 2>&1 || { tail -5 $OUT/traffic4k.log; exit 1; }
python3 tools/pmc_traffic_json.py gpurun_out/r04n/traffic4k 3840 2160 $OUT/pmc_4k.json > /dev/null || exit 1
python3 -c "import json; [print(f, json.load(open(f))['pass_hbm_bytes_per_frame']/json.load(open(f))['pass_algorithmic_bytes_per_frame']) for f in ['$OUT/pmc_1080.json','$OUT/pmc_4k.json']]"
