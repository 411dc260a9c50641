#!/bin/bash
# REPLACE by the device refinement's slack levels (KLT_SEL_SLACK: partition
# steps queued past the expected log2(len / threshold); a level past the
# threshold runs its four launches as no-ops, a missing one costs a relaunch),
# alternating, three rounds, one process per run (tools/exp/r06_replace_ab.py).
set -o pipefail
OUT=gpurun_out/${1:-r06sl}; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2 3; do
  for sl in ${SLACKS:-2 1 0 -1}; do
    KLT_SEL_SLACK=$sl timeout -k 10 120 python3 tools/exp/r06_replace_ab.py $OUT slack$sl >> $OUT/slack_ab.jsonl 2> $OUT/slack$sl.err || { tail -5 $OUT/slack$sl.err; exit 1; }
  done
done
python3 - $OUT/slack_ab.jsonl <<'PY'
import collections, json, sys
import numpy as np
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l)
    d[r["label"]].append((r["us_per_replace_median"], r["us_device_splits"], r["us_downloads_and_host_sort"], r["parity_mismatched"]))
for k, v in d.items():
    print(k, "replace", [round(x[0]) for x in v], "median", round(float(np.median([x[0] for x in v]))), "device splits",
          [round(x[1]) for x in v], "host", [round(x[2]) for x in v], "mismatched", set(x[3] for x in v))
PY
