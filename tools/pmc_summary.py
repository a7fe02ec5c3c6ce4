#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per-kernel average duration and PMC counters per
dispatch (and per macroblock when --mbs is given)."""
import argparse
import collections
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--mbs", type=float, default=0, help="macroblocks per dispatch (for per-MB figures)")
a = ap.parse_args()

for f in glob.glob(os.path.join(a.dir, "stats", "**", "*kernel_stats.csv"), recursive=True):
    print(open(f).read())
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.dir, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(float)
    for row in csv.DictReader(open(f)):
        per[(row["Kernel_Name"], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, d, c), v in per.items():
        vals[k][c].append(v)
for k, cs in vals.items():
    if k.startswith("__amd") or "at::" in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        m = sum(v) / len(v)
        extra = f"   per MB {m / a.mbs:12.2f}" if a.mbs else ""
        print(f"  {c:24s} {m:16.1f}{extra}")
