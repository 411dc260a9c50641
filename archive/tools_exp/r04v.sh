#!/bin/bash
# Round 4: REPLACE by the device/host segment threshold (KLT_AMD_SELECT_THRESHOLD)
# and the host enqueue probe
set -o pipefail
OUT=gpurun_out/r04v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 archive/tools_exp/enqueue_probe.py 20 40 > $OUT/enqueue.txt 2> $OUT/enqueue.err || { tail -5 $OUT/enqueue.err; exit 1; }
cat $OUT/enqueue.txt
Q="--steps 20 --warmup 5 --no-cpu --no-4k --no-fast"
for T in 32768 16384 65536 24576 49152 32768; do
  KLT_AMD_SELECT_THRESHOLD=$T timeout -k 10 300 python3 bench.py $Q > $OUT/t$T.json 2> $OUT/t$T.err || { tail -5 $OUT/t$T.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/t$T.json'))['api']['replace']; print('T=$T', round(d['value']), round(d['us_per_replace_median']), d['parity']['columns_mismatched'], {k: round(v) for k, v in d['select_median'].items()})"
done
# device timeline of REPLACE (kernel trace of the probe, 6 frames)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o rp -- python3 $GRAFT_REPO_ROOT/tools/exp/replace_probe.py 6 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && find $OUT/prof -name "*kernel_trace.csv" | head -3
