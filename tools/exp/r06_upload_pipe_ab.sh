#!/bin/bash
# Per-call KLTTrackFeatures uploads: the round-5 schedule
# (one pool generation per DMA group, KLT_AMD_UPLOAD_PIPE=0, 4 groups) against
# one generation for the whole frame with each group's DMA queued as soon as
# its pieces are copied (default), at 4, 8 and 16 groups; and the feature
# list's completion polled (KLT_AMD_SYNC_SPIN_US) against a blocking wait
# (0), and the first group's share (KLT_AMD_UPLOAD_FIRST, 0: equal groups).
# Configurations PIPE:GROUPS:FIRST:SPIN; alternating, three
# rounds, one process per run (tools/exp/r06_upload_ab.py), then one traced
# run of each.
set -o pipefail
OUT=gpurun_out/${1:-r06pipe}; mkdir -p $OUT
export TMPDIR=/tmp
CONFS=${CONFS:-"0:4:0:0 0:2:0:0 1:2:0:0 1:2:0.33:0 1:2:0.25:0 1:3:0.2:0 1:2:0.33:2000"}
for round in ${ROUNDS:-1 2 3}; do
  for cf in $CONFS; do
    IFS=: read p g f sp <<< "$cf"; L=p${p}g${g}f${f}s$sp
    KLT_AMD_UPLOAD_FIRST=$f KLT_AMD_SYNC_SPIN_US=$sp KLT_AMD_UPLOAD_PIPE=$p KLT_AMD_UPLOAD_GROUPS=$g timeout -k 10 120 python3 tools/exp/r06_upload_ab.py $L >> $OUT/pipe_ab.jsonl 2> $OUT/$L.err || { tail -5 $OUT/$L.err; exit 1; }
    tail -1 $OUT/pipe_ab.jsonl | cut -c1-260
  done
done
for cf in $CONFS; do
  IFS=: read p g f sp <<< "$cf"; L=p${p}g${g}f${f}s$sp
  KLT_AMD_UPLOAD_FIRST=$f KLT_AMD_SYNC_SPIN_US=$sp KLT_UPLOAD_TRACE=1 KLT_AMD_UPLOAD_PIPE=$p KLT_AMD_UPLOAD_GROUPS=$g timeout -k 10 120 python3 tools/exp/r06_upload_ab.py trace > /dev/null 2> $OUT/trace_$L.err || { tail -5 $OUT/trace_$L.err; exit 1; }
  python3 - $OUT/trace_$L.err <<'PY'
import sys
import numpy as np
rows = [l.split() for l in open(sys.argv[1]) if l.startswith("uptrace")]
rows = rows[len(rows) // 3:]
cp = np.array([[float(t.split("=")[1]) for t in r if t.startswith("copy=")] for r in rows])
eq = np.array([[float(t.split("=")[1]) for t in r if t.startswith("enq=")] for r in rows])
print(sys.argv[1], "calls", len(rows), "until group ready (us, median)", np.round(np.median(cp, 0), 1).tolist(),
      "enqueue", np.round(np.median(eq, 0), 1).tolist(), "host total", round(float(np.median(cp.sum(1) + eq.sum(1))), 1))
PY
done
