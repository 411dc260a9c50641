#!/usr/bin/env python3
"""Align a bench.py line's timed-region marks (timed_region_host.monotonic_ns,
CLOCK_MONOTONIC) with a rocprofv3 kernel trace of the same run (the same
clock): how long after the region starts the first kernel starts, the
kernels inside it, the gaps between them, and how long after the last kernel
ends the host sees the region end.

usage: tools/region_marks.py bench.json run_kernel_trace.csv
"""
from __future__ import annotations

import csv
import json
import re
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    m0, m1 = d["timed_region_host"]["monotonic_ns"]
    ks = []
    for r in csv.DictReader(open(sys.argv[2])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= m0 and e <= m1:
            m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            ks.append((s, e, m.group(1) if m else r["Kernel_Name"][:24], r["Queue_Id"], r["Grid_Size_Z"]))
    ks.sort()
    print(f"{sys.argv[1]}: value {d['value']:.0f} frames/s, region {(m1 - m0) / 1e3:.1f} us, "
          f"enqueue {d['timed_region_host']['enqueue_us']:.1f} us, {len(ks)} kernels")
    if not ks:
        return
    busy_end = m0
    idle = 0.0
    for s, e, k, q, z in ks:
        gap = max(0, s - busy_end)
        idle += gap
        print(f"  {k:14s} q{q} z{z:>3s} start {(s - m0) / 1e3:8.1f} dur {(e - s) / 1e3:7.1f} idle-before {gap / 1e3:6.1f}")
        busy_end = max(busy_end, e)
    tail = m1 - busy_end
    print(f"  first kernel after {(ks[0][0] - m0) / 1e3:.1f} us; region ends {tail / 1e3:.1f} us after the last "
          f"kernel; GPU idle inside the region {(idle + tail) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
