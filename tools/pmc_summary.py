#!/usr/bin/env python3
"""Sum rocprofv3 counter CSVs (gpurun_out/pmc*/) per kernel; per-op figures use --ops."""
import collections
import csv
import glob
import sys

n_ops = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if not any(x in k for x in ("pair", "big", "replay", "compile")):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:24s} {v:16.4g}   per-op {v / n_ops:10.2f}")
