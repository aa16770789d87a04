#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv (name, calls, average and total us), largest total first.
usage: kstats.py DIR [N]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:n]:
        print(f"{r['Name'][:90]:90s} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:10.2f} us "
              f"{float(r['TotalDurationNs']) / 1e6:10.2f} ms")
