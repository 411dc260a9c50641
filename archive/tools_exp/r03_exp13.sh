#!/bin/bash
# band builds whose outer margin rows build hs only: shard tests, pyramid tests, 8-rank simulation
set -o pipefail
OUT=gpurun_out/exp13; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_shard.py tests/test_gpu_pyramid.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in "--lazy-flag" "--lazy-flag --no-ahead"; do
  timeout -k 10 500 python tools/shard_sim.py --worlds 1 8 --frames 257 --chunk 64 --margins 64 $v > $OUT/s.log 2>&1 || { tail -5 $OUT/s.log; exit 1; }
  python3 - $OUT/s.log "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"workload')][0])
out = []
for r in d["runs"]:
    q = max(r["per_rank_us_per_frame"], key=lambda q: q["wall"])
    k = q["replay_kernels"]
    out.append("w%d max %.2f (l0 %.2f l1 %.2f trk %.2f) x%.2f redo %d digest %d" % (r["world"], q["wall"], k["k_pyr_l0"],
               k["k_pyr_l1"], k["k_track"], r["projected_speedup"] or 1, r["chunks_redone_full_frame"], r["state_digest"]))
print(sys.argv[2], " | ".join(out))
PY
done
