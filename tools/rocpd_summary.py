#!/usr/bin/env python3
"""Kernel-stats summary (name, calls, total/avg us, %) from a rocprofv3 rocpd database."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow(r)
    for r in rows:
        print(f"{r[3]:10.3f} us avg  {r[1]:5d} calls  {r[4]:6.2f}%  {r[0][:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
