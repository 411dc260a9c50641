#!/bin/bash
# one PMC pass per counter group over one microbench command.
# usage: bash archive/tools/pmc_one.sh <tag> "<counters>" <microbench args...>
set -o pipefail
TAG=$1; shift; CTRS=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/pmc -o run -- python tools/microbench.py "$@" > $OUT/pmc.log 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/pmc.log; exit 1; }
python tools/pmc_summary.py $(find $OUT/pmc -name "*counter_collection.csv") | grep -A12 "k_track\|k_pyr"
