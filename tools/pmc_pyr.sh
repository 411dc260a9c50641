#!/bin/bash
# PMC passes over the batched pyramid kernels (4K, 64-frame launches,
# pyramids only): SQ instruction / wait / cycle counters in three passes
# (kernel-trace only).  usage: bash tools/pmc_pyr.sh <tag> [microbench args, e.g. --strips 2]
set -o pipefail
TAG=${1:-pmcpyr}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="frames --width 3840 --height 2160 --frames 129 --reps 1 --chunk 64 --pyr-only $*"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python tools/microbench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; }
done
python tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") > $OUT/summary.txt
cat $OUT/summary.txt
