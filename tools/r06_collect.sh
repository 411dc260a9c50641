#!/bin/bash
# Copy a tools/r06_final.sh cycle's results from gpurun_out/<tag> into
# profiles/<tag>_* (and the PMC traffic into profiles/pmc_latest.json,
# pmc_4k_latest.json, which bench.py attaches).  CPU only.
set -eo pipefail
TAG=${1:?tag}; S=gpurun_out/$TAG; P=profiles; C=$(cat $S/commit.txt)
cp $S/bench.json $P/${TAG}_bench.json
cp $S/bench_s20.json $P/${TAG}_bench_s20.json
{ echo "$C"; tail -5 $S/gpu_tests.log; } > $P/${TAG}_gpu_tests_tail.txt
{ echo "$C"; cat $S/smoke.txt; } > $P/${TAG}_smoke.txt
for f in kernel_stats_isolated kernel_stats_4k_tracked kernel_stats_4k_pyr; do cp $S/$f.txt $P/${TAG}_$f.txt; done
cp $S/kernel_stats.csv $P/${TAG}_kernel_stats.csv
{ echo "$C: tools/exp/replace_probe.py 6 under rocprofv3 --kernel-trace --stats (the process exits cleanly after REPLACE)"; grep -v "^W20\|^E20" $S/exitprof.log | tail -15; } > $P/${TAG}_exit_after_replace_rocprof.txt
{ echo "$C: tools/shard_sim.py --frames 1001 --chunk 64 --worlds 1 8 --margins 64 --pass1-shared --exchange-in-stream-us 40 (config 4, 8-rank projection with the all-gather as a 40 us in-stream stall)"; grep '^{' $S/shard8_instream.log; } > $P/${TAG}_config4_shard_sim_instream.txt
{ echo "$C: tools/exp/r06_rehearsal.sh (bench.py at N=1, N=1 through torch.distributed.run/RCCL, N=2 and N=4 ranks sharing GPU 0 over gloo); the sharded_4k key of each line"
  for n in 1 1rccl 2 4; do python3 - $S/reh/n$n.json n$n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s = d["sharded_4k"]
print(json.dumps({"run": sys.argv[2], "value": d["value"], "sharded_4k": {k: s[k] for k in ("value", "us_per_frame", "n_gpus", "rank_us_per_frame", "chunks_redone_full_frame", "state_digest", "ranks_agree_on_state")}, "exchange": s["exchange"], "parity": s["parity"]}))
PY
  done; } > $P/${TAG}_rehearsal.txt
{ echo "$C: tools/pmc_traffic.sh at 1080p and 4K (separate FETCH_SIZE / WRITE_SIZE passes)"; echo "## 1080p"; cat $S/traffic1080/summary.txt; echo "## 4K"; cat $S/traffic4k/summary.txt; } > $P/${TAG}_pmc_traffic.txt
cp $S/pmc_1080.json $P/pmc_latest.json
cp $S/pmc_4k.json $P/pmc_4k_latest.json
echo "collected $TAG ($C)"
