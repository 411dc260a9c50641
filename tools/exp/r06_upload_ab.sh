#!/bin/bash
# Per-call KLTTrackFeatures uploads: the frame split into
# 2/4/8/16 DMA groups (KLT_AMD_UPLOAD_GROUPS), alternating, three rounds, one
# process per run, on one box; tools/exp/r06_upload_ab.py.
set -o pipefail
OUT=gpurun_out/${1:-r06up}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for g in ${GROUPS_LIST:-4 2 8 16}; do
    KLT_AMD_UPLOAD_GROUPS=$g timeout -k 10 120 python3 tools/exp/r06_upload_ab.py g$g >> $OUT/upload_ab.jsonl 2> $OUT/g$g.err || { tail -5 $OUT/g$g.err; exit 1; }
    tail -1 $OUT/upload_ab.jsonl
  done
done
# one traced run per group count: the host copy and the DMA enqueue of each group (KLT_UPLOAD_TRACE)
for g in ${GROUPS_LIST:-4 2 8 16}; do
  KLT_UPLOAD_TRACE=1 KLT_AMD_UPLOAD_GROUPS=$g timeout -k 10 120 python3 tools/exp/r06_upload_ab.py trace$g > /dev/null 2> $OUT/trace$g.err || { tail -5 $OUT/trace$g.err; exit 1; }
  python3 - $OUT/trace$g.err <<'PY'
import re, sys
import numpy as np
rows = [l.split() for l in open(sys.argv[1]) if l.startswith("uptrace")]
rows = rows[len(rows) // 3:]  # past the warm-up context
cp = np.array([[float(t.split("=")[1]) for t in r if t.startswith("copy=")] for r in rows])
eq = np.array([[float(t.split("=")[1]) for t in r if t.startswith("enq=")] for r in rows])
print(sys.argv[1], "calls", len(rows), "copy us per group (median)", np.round(np.median(cp, 0), 1).tolist(),
      "enqueue us", np.round(np.median(eq, 0), 1).tolist(), "host total", round(float(np.median(cp.sum(1) + eq.sum(1))), 1))
PY
done
