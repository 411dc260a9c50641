#!/bin/bash
# The pyramid stream and the tracking stream confined to CU subsets
# (KLT_PYR_CUS / KLT_TRK_CUS, runtime.hip cu_masked_stream) against the
# shared chip: bench.py's 1080p value leg alone, alternating, two rounds.
# usage: r06_cumask_ab.sh <tag>   (CONFS="PYR:TRK ...", 0 = unmasked)
set -o pipefail
OUT=gpurun_out/${1:-r06cu}; mkdir -p $OUT
export TMPDIR=/tmp
B="--no-cpu --no-4k --no-fast --api-frames 0 --replace-frames 0 --no-sharded-4k"
CONFS=${CONFS:-"0:0 224:0 192:0 0:96 0:64 192:64 160:96"}
for round in ${ROUNDS:-1 2}; do
  for cf in $CONFS; do
    IFS=: read p t <<< "$cf"
    P=; T=
    [ "$p" != 0 ] && P=$p
    [ "$t" != 0 ] && T=$t
    KLT_PYR_CUS=$P KLT_TRK_CUS=$T timeout -k 10 300 python3 bench.py $B > $OUT/p${p}t$t.json 2> $OUT/p${p}t$t.err || { tail -5 $OUT/p${p}t$t.err; exit 1; }
    python3 - $OUT/p${p}t$t.json "$cf" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("pyr:trk", sys.argv[2], "value", round(d["value"]), "kern/frame", {k: round(v, 2) for k, v in d["kernels_us_per_frame"].items() if v},
      "parity", d.get("parity", {}).get("columns_mismatched", d.get("parity")), flush=True)
PY
  done
done
