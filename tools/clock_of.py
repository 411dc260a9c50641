#!/usr/bin/env python3
"""Effective shader clock per kernel dispatch from a rocprofv3 --pmc
GRBM_GUI_ACTIVE run (counter_collection.csv): GRBM_GUI_ACTIVE is summed over
the 8 XCDs, so clock = value / 8 / duration (MI355X_MICROARCH.md, "DVFS
give-back").  Prints one line per dispatch of the named kernels (or a summary
per kernel and per segment of consecutive launches with --summary).

usage: tools/clock_of.py run_counter_collection.csv [--kernels k_pyr_l0 k_track7] [--summary]
"""
from __future__ import annotations

import argparse
import csv
import re
import statistics


def short(name: str) -> str:
    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
    return m.group(1) if m else name.split("(")[0][-40:]


def rows(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            dur = (t1 - t0) * 1e-9
            out.append({"id": int(r["Dispatch_Id"]), "k": short(r["Kernel_Name"]), "t0": t0, "dur_us": dur * 1e6,
                        "ghz": float(r["Counter_Value"]) / 8 / dur / 1e9 if dur > 0 else 0.0})
    out.sort(key=lambda d: d["id"])
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--kernels", nargs="*", default=["k_pyr_l0", "k_pyr_l1", "k_track7"])
    p.add_argument("--summary", action="store_true")
    p.add_argument("--min-us", type=float, default=20.0, help="ignore shorter dispatches (clock is noisy)")
    a = p.parse_args()
    rs = [r for r in rows(a.csv) if r["k"] in a.kernels and r["dur_us"] >= a.min_us]
    if not a.summary:
        for r in rs:
            print(f"{r['id']:5d} {r['k']:12s} {r['dur_us']:9.1f} us {r['ghz']:.3f} GHz")
        return
    for k in a.kernels:
        g = [r["ghz"] for r in rs if r["k"] == k]
        if g:
            print(f"{k:12s} n={len(g):3d} clock median {statistics.median(g):.3f} GHz "
                  f"min {min(g):.3f} max {max(g):.3f}")


if __name__ == "__main__":
    main()
