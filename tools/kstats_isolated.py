#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, split into
launches that overlap another kernel in time (the overlapped schedule: a
pyramid build of chunk c+1 running beside the tracking of chunk c) and
isolated launches (nothing else on the GPU -- bench.py's one-stream replay,
whose HIP-event durations are the roofline's).

  python tools/kstats_isolated.py run_kernel_trace.csv [min_us]
"""
import csv
import sys
from collections import defaultdict


def main(path: str, min_us: float = 0.0) -> None:
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if int(r["Grid_Size_Z"]) > 1:  # batched pyramid launches: one row per frame size (grid.x)
            name = f"{name} [grid.x {r['Grid_Size_X']}]"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r["Grid_Size_Z"])))
    rows.sort()
    iso, ovl = defaultdict(list), defaultdict(list)
    for i, (s, e, n, z) in enumerate(rows):
        overlap = False
        for j in range(max(0, i - 64), min(len(rows), i + 64)):
            if j != i and rows[j][0] < e and rows[j][1] > s:
                overlap = True
                break
        (ovl if overlap else iso)[n].append(((e - s) / 1e3, z))
    # grid.z of the batched pyramid kernels is the frame count of the launch
    print(f"{'kernel':60s} {'isolated':>22s} {'us/frame':>9s} {'overlapped':>22s} {'us/frame':>9s}")
    for n in sorted(set(iso) | set(ovl)):
        a, b = iso.get(n, []), ovl.get(n, [])
        if max(d for d, _ in a + b) < min_us:
            continue
        cols = []
        for v in (a, b):
            if not v:
                cols += ["", ""]
                continue
            tot, fr = sum(d for d, _ in v), sum(z for _, z in v)
            cols += [f"{len(v):5d} x {tot / len(v):10.2f} us", f"{tot / fr:9.2f}" if fr > len(v) else ""]
        print(f"{n[:60]:60s} {cols[0]:>22s} {cols[1]:>9s} {cols[2]:>22s} {cols[3]:>9s}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
