#!/usr/bin/env python3
"""Per-stage PMC deltas from a `run_gpu.sh pmcstages` run (stage_profile.py under rocprofv3 --pmc):
fast-kernel dispatches come in groups of 6 per AMOD_STOP_AFTER level (1 warm-up + 5 timed)."""
import collections
import csv
import os
import sys


def main(d, stages):
    agg = collections.defaultdict(float)
    disp = []
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "k_decode_fast" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        if k not in disp:
            disp.append(k)
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    disp.sort()
    names = sorted({c for (_, c) in agg})
    rows = []
    for i, st in enumerate(stages):
        grp = disp[6 * i + 1: 6 * i + 6]
        rows.append((st, {c: sum(agg[(k, c)] for k in grp) / len(grp) for c in names}))
    prev = {c: 0.0 for c in names}
    F = 10000
    print("per frame: " + " ".join(f"{c:>18s}" for c in names))
    for st, v in rows:
        print(f"stage<={st:3d} " + " ".join(f"{(v[c] - prev[c]) / F:18.1f}" for c in names))
        prev = v


if __name__ == "__main__":
    main(sys.argv[1], [int(s) for s in os.environ.get("STAGES", "0,1,2,3,99").split(",")])
