#!/usr/bin/env python3
"""Per-kernel durations and launch-to-launch spacing from a rocprofv3
--kernel-trace csv (kernel_trace.csv): for every kernel name the median
duration, and for the kernels matching REGEX the median start-to-start period
and end-to-next-start gap of consecutive launches, plus what else ran inside
those periods.  usage: kt_gaps.py DIR REGEX"""
import csv
import glob
import os
import re
import statistics
import sys

d, rx = sys.argv[1], re.compile(sys.argv[2])
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
dur = {}
for s, e, k in rows:
    dur.setdefault(k, []).append(e - s)
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(v):6d} x median {statistics.median(v) / 1000:8.2f} us  total {sum(v) / 1e6:8.3f} ms  {k[:90]}")
hot = [(s, e) for s, e, k in rows if rx.search(k)]
if len(hot) > 2:
    per = [b[0] - a[0] for a, b in zip(hot, hot[1:])]
    gap = [b[0] - a[1] for a, b in zip(hot, hot[1:])]
    print(f"matching launches {len(hot)}: start-to-start median {statistics.median(per) / 1000:.2f} us "
          f"(p10 {sorted(per)[len(per) // 10] / 1000:.2f}, p90 {sorted(per)[9 * len(per) // 10] / 1000:.2f}), "
          f"end-to-next-start median {statistics.median(gap) / 1000:.2f} us")
