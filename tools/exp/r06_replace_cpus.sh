#!/bin/bash
# REPLACE (the bench's api.replace leg alone) with the whole process confined
# to one CCD's CPUs (one L3), to one NUMA node, or free (the default): how
# much of the host sort's time is cache traffic between far cores.  taskset
# starts python before anything touches the GPU.
set -o pipefail
OUT=gpurun_out/${1:-r06rc}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for cfg in "free:" "ccd0:0-7,128-135" "node0:0-63,128-191"; do
    lab=${cfg%%:*}; cpus=${cfg#*:}
    if [ -z "$cpus" ]; then
      timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT $lab >> $OUT/replace_cpus.jsonl 2> $OUT/rc_$lab.err || { tail -5 $OUT/rc_$lab.err; exit 1; }
    else
      timeout -k 10 120 taskset -c $cpus python3 tools/exp/r06_replace_ab.py $OUT $lab >> $OUT/replace_cpus.jsonl 2> $OUT/rc_$lab.err || { tail -5 $OUT/rc_$lab.err; exit 1; }
    fi
    tail -1 $OUT/replace_cpus.jsonl | cut -c1-250
  done
done
