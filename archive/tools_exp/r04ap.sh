#!/bin/bash
# Round 4: where the tracker's gathers are served (1080p/5000, 64-frame
# launches): vL1D accesses and misses to L2, L2 hits/misses, and the SQ's
# in-flight levels of vector-memory and LDS instructions (average latency =
# level / instructions), one --pmc pass each, kernel trace only
set -o pipefail
OUT=gpurun_out/r04ap; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="frames --frames 129 --reps 1 --chunk 64 --table"
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 tools/microbench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "k_track7" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[-3] if "/" in f else f, {k: f"{v:.4g}" for k, v in acc.items()}, "dispatch rows", dict(n))
PY
