#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc counter CSV (one row per dispatch and
counter): kernel family, dispatches, and the mean of every counter a dispatch."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kb2e::", "").split("<")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
names = sorted({c for v in agg.values() for c in v})
print("kernel".ljust(34), "n".rjust(6), *[c.rjust(22) for c in names])
for k in sorted(agg, key=lambda k: -agg[k].get("SQ_BUSY_CYCLES", 0)):
    n = max(1, len(disp[k]))
    print(k[:34].ljust(34), str(n).rjust(6), *[f"{agg[k][c] / n:22.1f}" for c in names])
