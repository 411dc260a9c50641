#!/bin/bash
# Registered per-call KLTTrackFeatures with and without the bounce buffer's
# event record after the DMA (KLT_AMD_REG_EVENT), alternating, four rounds,
# one process per run (tools/exp/r06_upload_ab.py).
set -o pipefail
OUT=gpurun_out/${1:-r06ev}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3 4; do
  for ev in 1 0; do
    KLT_AMD_REG_EVENT=$ev timeout -k 10 120 python3 tools/exp/r06_upload_ab.py ev$ev >> $OUT/regevent_ab.jsonl 2> $OUT/ev$ev.err || { tail -5 $OUT/ev$ev.err; exit 1; }
    tail -1 $OUT/regevent_ab.jsonl | cut -c1-100
  done
done
python3 - $OUT/regevent_ab.jsonl <<'PY'
import collections, json, sys
import numpy as np
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l)
    d[r["label"]].append((r["us_per_call_registered"], r["us_per_call_pageable"], r["digest"], r["lists_equal"]))
for k, v in d.items():
    print(k, "registered", [x[0] for x in v], "median", np.median([x[0] for x in v]), "pageable median",
          np.median([x[1] for x in v]), set(x[2] for x in v), set(x[3] for x in v))
PY
