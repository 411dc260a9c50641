#!/usr/bin/env python3
"""Overlap of tracker and pyramid kernels in a rocprofv3 kernel_trace.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    name = r["Kernel_Name"]
    kind = "track" if "k_track" in name else "l0" if "k_pyr_l0" in name else "l1" if "k_pyr_l1" in name else None
    if kind:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
ks.sort()
t0 = ks[0][0]
busy = {"track": [], "l0": [], "l1": []}
for s, e, k in ks:
    busy[k].append((s, e))


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv)


tr = union(busy["track"])
py = union(busy["l0"] + busy["l1"])
allu = union(busy["track"] + busy["l0"] + busy["l1"])
# intersection
inter = 0
j = 0
for s, e in tr:
    for ps, pe in py:
        lo, hi = max(s, ps), min(e, pe)
        if hi > lo:
            inter += hi - lo
span = ks[-1][1] - t0
print(f"span {span/1e3:.1f} us, busy(any) {total(allu)/1e3:.1f}, track {total(tr)/1e3:.1f}, pyramid {total(py)/1e3:.1f}, "
      f"overlap {inter/1e3:.1f}")
for s, e, k in ks[:40]:
    print(f"{k:6s} {(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:8.1f}")

# gaps between consecutive kernels (any kind)
allk = sorted([(s, e, k) for s, e, k in ks])
gaps = [allk[i + 1][0] - allk[i][1] for i in range(len(allk) - 1)]
import statistics
if gaps:
    print("gap us: median", statistics.median(gaps) / 1e3, "mean", statistics.mean(gaps) / 1e3,
          "max", max(gaps) / 1e3)
