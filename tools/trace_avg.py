#!/usr/bin/env python3
"""Mean duration of the last K launches of each kernel matching a substring in a
rocprofv3 kernel-trace CSV (the timed steps of bench.py, after its settle and
warm-up launches):  tools/trace_avg.py TRACE.csv K [substring ...]"""
import csv
import sys

path, k = sys.argv[1], int(sys.argv[2])
subs = sys.argv[3:] or ["stencil8_kernel", "face_step2_add_kernel"]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
for s in subs:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if s in r["Kernel_Name"]]
    if d:
        last = d[-k:]
        print("%-24s launches %4d  mean of last %d: %.1f us  (all: %.1f us)"
              % (s, len(d), len(last), sum(last) / len(last), sum(d) / len(d)))
