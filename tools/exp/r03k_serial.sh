#!/bin/bash
# overlapped (default) against one-stream (--serial) 1080p bench, alternating, same box; serial timeline
set -o pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu --no-4k --api-frames 0 --no-fast --replace-frames 0"
for i in 1 2 3; do
  for m in "" "--serial"; do
    timeout -k 10 300 python bench.py $Q $m > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b.json')); print('$m' or 'overlap', round(d['value']), {k: round(v,2) for k,v in d['kernels_us_per_frame'].items() if v})"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o run -- python bench.py $Q --serial > $OUT/p.json 2> $OUT/p.err || { tail -5 $OUT/p.err; exit 1; }
python3 - $(find $OUT/p -name "*kernel_trace.csv") <<'PY' > $OUT/serial_timeline.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_track7<false, true, 2, false>' in r['Kernel_Name']]
t0 = int(rows[idx[2]]['Start_Timestamp'])
for r in rows[idx[2] - 4: idx[5] + 2]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {r['Kernel_Name'][:70]}")
PY
cat $OUT/serial_timeline.txt
