#!/usr/bin/env python3
"""Per-kernel PMC totals of a rocprofv3 --pmc csv directory (first dispatch of each kernel)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[(r["Kernel_Name"][:70], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
seen = set()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for (k, d), v in sorted(agg.items(), key=lambda kv: kv[0][1]):
    if k in seen or pat not in k:
        continue
    seen.add(k)
    print(k, d, {a: int(b) for a, b in sorted(v.items())})
