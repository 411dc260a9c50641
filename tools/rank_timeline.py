#!/usr/bin/env python3
"""One sharded rank's chunk timeline from a rocprofv3 kernel trace of its
replay (tools/shard_sim.py --replay ... under rocprofv3 --kernel-trace): for a
few steady-state chunks, every kernel between two tracker launches with its
queue, start (relative to the earlier tracker's end) and duration, and the
tracker-to-tracker gap.  usage: tools/rank_timeline.py kernel_trace.csv [chunks]"""
from __future__ import annotations

import csv
import re
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     m.group(1) if m else r["Kernel_Name"][:40], r["Queue_Id"], r.get("Grid_Size_Z", "")))
    rows.sort()
    trk = [i for i, r in enumerate(rows) if r[2].startswith("k_track")]
    # the timed replay is the last third of the tracker launches
    trk = trk[2 * len(trk) // 3:]
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    mid = len(trk) // 2
    gaps = []
    for a, b in zip(trk, trk[1:]):
        gaps.append((rows[b][0] - rows[a][1]) / 1e3)
    print(f"tracker launches in the timed replay: {len(trk)}; tracker-end to next tracker-start gap, us: "
          f"median {sorted(gaps)[len(gaps) // 2]:.1f}, all {[round(g) for g in gaps]}")
    print("tracker durations, us:", [round((rows[i][1] - rows[i][0]) / 1e3) for i in trk])
    for a, b in list(zip(trk, trk[1:]))[mid:mid + want]:
        t0 = rows[a][1]
        print(f"-- chunk: tracker {(rows[a][1] - rows[a][0]) / 1e3:.1f} us, then:")
        for s, e, k, q, z in rows[a + 1:b + 1]:
            print(f"   {k:22s} q{q:>3s} z{z:>3s} start {(s - t0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f}")


if __name__ == "__main__":
    main()
