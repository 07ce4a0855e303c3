#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 counter_collection.csv files."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(path)
    for k, d in agg.items():
        if "amod" not in k and "k_" not in k:
            continue
        print("  ", k, "dispatches", len(next(iter(d.values()))))
        for c, v in sorted(d.items()):
            print("      %-24s %16.1f" % (c, sum(v) / len(v)))
