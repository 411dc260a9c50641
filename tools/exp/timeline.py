#!/usr/bin/env python3
"""Timeline of one sharded rank's replay from a rocprofv3 kernel_trace.csv:
the last `--reps`-th of the launches (the timed replay), every kernel with its
start/end relative to the first, and the idle gaps of the device (no kernel
running) longer than 2 us.  usage: timeline.py kernel_trace.csv [--tail N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tail = int(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 0
ks = []
for r in rows:
    n = r["Kernel_Name"]
    short = ("track" if "k_track" in n else "l0" if "k_pyr_l0" in n else "l1" if "k_pyr_l1" in n else
             "order" if "k_band_order" in n else "copy" if "copyBuffer" in n or "fillBuffer" in n else
             "torch" if "at::native" in n else n.split("(")[0][-24:])
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r.get("Queue_Id", "")))
ks.sort()
if tail:
    ks = ks[-tail:]
t0 = ks[0][0]
busy_end = t0
gaps = []
for s, e, k, q in ks:
    if s > busy_end + 2000:
        gaps.append((busy_end - t0, s - busy_end))
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {k:8s} q{q}")
    busy_end = max(busy_end, e)
tot = (busy_end - t0) / 1e3
print(f"span {tot:.1f} us; idle gaps > 2 us: {len(gaps)}, total {sum(g for _, g in gaps) / 1e3:.1f} us")
for at, g in gaps:
    print(f"  gap at {at / 1e3:.1f} us: {g / 1e3:.1f} us")
