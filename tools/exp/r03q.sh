#!/bin/bash
# smoke() and the config-4 sharded bench at N = 1 (whole job, exchange included)
set -o pipefail
OUT=gpurun_out/r03q; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -10 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --mode sharded > $OUT/sharded_n1.json 2> $OUT/sharded_n1.err || { tail -10 $OUT/sharded_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/sharded_n1.json')); print({k: d[k] for k in ('metric','value','unit','ms_per_step','steps','config') if k in d})"
