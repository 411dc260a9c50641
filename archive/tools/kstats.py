#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: name, calls, avg/min us."""
import csv
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        name = r["Name"].replace("(anonymous namespace)::", "")[:48]
        print(f"  {name:48s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:10.2f} us avg "
              f"{float(r['MinNs'])/1e3:9.2f} min {float(r['Percentage']):6.2f}%")
