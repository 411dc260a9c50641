#!/bin/bash
# banks built planar when the generic tracker reads them (fast mode etc.): whole GPU suite, then the bench's fast leg
set -o pipefail
OUT=gpurun_out/exp39; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python bench.py --no-cpu --api-frames 0 --replace-frames 0 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b.json')); print('exact', round(d['value']), 'fast', d['fast'])"
