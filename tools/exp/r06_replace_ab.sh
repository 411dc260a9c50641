#!/bin/bash
# the sort pool's spin bound and worker clamp, A/B on one
# box, three alternating rounds, one process per run.
#   spin=-1 (whole sort, the round-4 behaviour, now the default) vs spin=50 us (round 5)
#   clamp (usable_cpus()-1) vs no clamp (the round-4 count)
set -o pipefail
OUT=gpurun_out/${1:-r06rep}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for cfg in "whole_clamp:-1:0" "spin50_clamp:50:0" "whole_noclamp:-1:1"; do
    IFS=: read lab spin nc <<< "$cfg"
    KLT_SORT_SPIN_US=$spin KLT_SORT_NO_CLAMP=$nc timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT $lab \
      >> $OUT/replace_ab.jsonl 2> $OUT/replace_ab_$lab.err || { tail -20 $OUT/replace_ab_$lab.err; exit 1; }
    tail -1 $OUT/replace_ab.jsonl
  done
done
cat /sys/fs/cgroup/cpu.max 2>/dev/null | sed 's/^/cpu.max /'
