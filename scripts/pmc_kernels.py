#!/usr/bin/env python3
"""Per-kernel medians of every counter in rocprofv3 --pmc output dirs.
usage: pmc_kernels.py DIR [DIR...]"""
import csv
import glob
import os
import statistics
import sys

vals = {}
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "at::native" in k or "rocclr" in k:
                continue
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items()):
    line = ", ".join(f"{c} {statistics.median(v):.0f} (n={len(v)})" for c, v in sorted(cs.items()))
    print(f"{k[:80]}: {line}")
    if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_LDS_IDX_ACTIVE" in cs:
        bc, act = statistics.median(cs["SQ_LDS_BANK_CONFLICT"]), statistics.median(cs["SQ_LDS_IDX_ACTIVE"])
        print(f"    -> bank conflicts {100 * bc / max(act, 1):.1f}% of LDS-active cycles")
