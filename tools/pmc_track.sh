#!/bin/bash
# PMC passes over the batched tracker workload (1080p, 5000 features, 192
# frames in 64-frame launches, feature table on): SQ instruction / cycle
# counters in two passes (kernel-trace only), plus a counted replay for the
# Newton iterations.  usage: bash tools/pmc_track.sh <tag> [microbench args]
set -o pipefail
TAG=${1:-pmctrk}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="frames --frames 193 --reps 1 --chunk 64 --table $*"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python tools/microbench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
timeout -k 10 120 python tools/microbench.py $ARGS --count > $OUT/count.json || exit 1
python tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") > $OUT/summary.txt
cat $OUT/summary.txt; cat $OUT/count.json
python tools/pmc_track_json.py $OUT $OUT/pmc_tracker.json
