#!/usr/bin/env python3
"""profiles/<round>/traffic.json: the per-workload traffic.json files of
tools/profile_summary.py as one list (bench.py's traffic_for picks the entry whose
frames and samples_per_frame match its workload).
usage: python tools/profile_merge.py profiles/r03 c2 c4 c5_10db"""
import json
import os
import sys


def main(root, subs):
    out = []
    for s in subs:
        p = os.path.join(root, s, "traffic.json")
        if os.path.exists(p):
            e = json.load(open(p))
            e["profile_dir"] = s
            out.append(e)
    json.dump(out, open(os.path.join(root, "traffic.json"), "w"), indent=1)
    print(json.dumps([(e["profile_dir"], e["frames"], e["samples_per_frame"]) for e in out]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
