#!/bin/bash
# Round-6 final cycle on one box: GPU tests, bench (default and the driver's
# --steps 20 shape), clean exit after REPLACE under rocprofv3, smoke(), the
# config-4 8-rank projection with the all-gather modelled in stream, the
# driver-shaped sharded_4k rehearsal at N = 1/2/4, kernel-trace summaries and
# the pyramid pass's PMC traffic at 1080p and 4K.  Each GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r06f}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp COMMIT=${COMMIT:-unknown}
bash tools/r05.sh $TAG tests bench s20 exitprof || exit 1
echo "== smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
SHARD_ARGS="--exchange-in-stream-us 40" LOGSFX=_instream bash tools/r05.sh $TAG shard8 || exit 1
echo "== rehearsal $(date +%T)"
bash tools/exp/r06_rehearsal.sh $TAG/reh || exit 1
echo "== prof $(date +%T)"
bash tools/r06_prof.sh $TAG || exit 1
echo "== pmc $(date +%T)"
bash tools/pmc_traffic.sh $TAG/traffic1080 > $OUT/traffic1080.log 2>&1 || { tail -5 $OUT/traffic1080.log; exit 1; }
python3 tools/pmc_traffic_json.py $OUT/traffic1080 1920 1080 $OUT/pmc_1080.json > /dev/null || exit 1
bash tools/pmc_traffic.sh $TAG/traffic4k --width 3840 --height 2160 > $OUT/traffic4k.log 2>&1 || { tail -5 $OUT/traffic4k.log; exit 1; }
python3 tools/pmc_traffic_json.py $OUT/traffic4k 3840 2160 $OUT/pmc_4k.json > /dev/null || exit 1
echo "== done $(date +%T)"
