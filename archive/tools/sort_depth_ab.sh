#!/bin/bash
# A/B of the REPLACE host-sort task depth (KLT_AMD_SORT_DEPTH) on one box.
# usage (via gpurun): bash archive/tools/sort_depth_ab.sh <tag> <depth>...
set -o pipefail
TAG=${1:-sortab}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for d in "$@"; do
  KLT_AMD_SORT_DEPTH=$d timeout -k 10 300 python bench.py --no-cpu --no-4k --no-fast > $OUT/bench_d$d.json 2> $OUT/bench_d$d.err || { tail -20 $OUT/bench_d$d.err; exit 1; }
  python3 - $OUT/bench_d$d.json $d <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))["api"]["replace"]
print("depth", sys.argv[2], "us/replace", round(r["us_per_replace_median"]), "host", round(r["select_median"]["us_downloads_and_host_sort"]),
      "fps", round(r["value"]), "mismatched", r["parity"]["columns_mismatched"])
PY
done
