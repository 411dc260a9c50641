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
