#!/usr/bin/env python3
"""Kernel timeline of one steady-state period from a rocprofv3 --kernel-trace
csv: every dispatch from the ANCHOR-th launch of the kernel matching REGEX
(default: the middle one) to the next one, with start / end relative to the
anchor's start, duration and queue, so kernels on different streams (the
two-stage tail on its side stream beside the head's run) line up; then the
median per-kernel durations and gaps between consecutive anchors.
usage: kt_timeline.py DIR REGEX [ANCHOR] [PERIODS]"""
import csv
import glob
import os
import statistics
import sys

d, rx = sys.argv[1], sys.argv[2]
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fftconv::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?")))
rows.sort()
import re

hot = [i for i, r in enumerate(rows) if re.search(rx, r[2])]
if not hot:
    sys.exit(f"no dispatch matches {rx}")
a = int(sys.argv[3]) if len(sys.argv) > 3 else len(hot) // 2
np_ = int(sys.argv[4]) if len(sys.argv) > 4 else 1
i0 = hot[a]
i1 = hot[min(a + np_, len(hot) - 1)]
t0 = rows[i0][0]
print(f"{'start':>9} {'end':>9} {'dur':>8}  queue  kernel   (us, relative to {rows[i0][2]} #{a})")
for s, e, k, q in rows[i0 - 2 if i0 >= 2 else 0:i1 + 3]:
    print(f"{(s - t0) / 1000:9.2f} {(e - t0) / 1000:9.2f} {(e - s) / 1000:8.2f}  q{q:<4} {k}")
per = [rows[b][0] - rows[c][0] for c, b in zip(hot, hot[1:])]
if per:
    print(f"period (start to start of {rx}): median {statistics.median(per) / 1000:.2f} us over {len(per)}")
dur = {}
for s, e, k, q in rows[hot[0]:hot[-1]]:
    dur.setdefault(k, []).append(e - s)
for k, v in sorted(dur.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    print(f"  {len(v):6d} x median {statistics.median(v) / 1000:8.2f} us  {k}")
