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
ap.add_argument("--json", default=None, help="write per-kernel HBM traffic per MB (bytes) to this file")
ap.add_argument("--config", type=int, default=3, help="SURVEY config of the profiled bench run (bench.py matches it)")
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

if a.json and a.mbs:
    import json
    out = {"source": os.path.basename(os.path.normpath(a.dir)), "survey_config": a.config, "mbs_per_dispatch": a.mbs,
           "note": "FETCH_SIZE / WRITE_SIZE are KiB per dispatch (rocprofv3, separate --pmc passes). "
                   "gfx950 reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM): "
                   "read_bytes_per_mb doubles FETCH_SIZE (an upper bound for narrower access), "
                   "read_bytes_per_mb_raw does not.",
           "kernels": {}}
    for k, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs or k.startswith("__amd") or "at::" in k:
            continue
        f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 / a.mbs
        w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024 / a.mbs
        out["kernels"][k] = {"read_bytes_per_mb": 2 * f, "read_bytes_per_mb_raw": f, "write_bytes_per_mb": w,
                             "traffic_bytes_per_mb": 2 * f + w}
        # issue counts per MB (the second roof: bench.py turns VALU per MB into valu_frac)
        for c, key in (("SQ_INSTS_VALU", "valu_per_mb"), ("SQ_INSTS_SALU", "salu_per_mb"), ("SQ_INSTS_LDS", "lds_per_mb")):
            if c in cs:
                out["kernels"][k][key] = sum(cs[c]) / len(cs[c]) / a.mbs
        if "GRBM_GUI_ACTIVE" in cs:
            out["kernels"][k]["grbm_gui_active"] = sum(cs["GRBM_GUI_ACTIVE"]) / len(cs["GRBM_GUI_ACTIVE"])
    json.dump(out, open(a.json, "w"), indent=1)
