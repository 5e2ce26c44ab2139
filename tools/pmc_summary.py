#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection CSVs: per kernel, median over
dispatches of each counter (summed over dimensions)."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        c = row.get("Counter_Name", "?")
        d = row.get("Dispatch_Id", row.get("Correlation_Id", "0"))
        vals[k][c][d] = vals[k][c].get(d, 0.0) + float(row.get("Counter_Value", 0))
for k, cs in vals.items():
    if not any(s in k for s in ("stencil", "face", "chol", "mass3")):
        continue
    print(k[:90])
    for c in sorted(cs):
        v = statistics.median(cs[c].values())
        print("   %-26s %16.0f" % (c, v))
