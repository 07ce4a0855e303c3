#!/usr/bin/env python3
"""Experiments only: bench.py's host_api leg (amod_decode_host from Python, decodeBatch from
Node) on C2 and C4 alone, without the rest of the default run.
  python tools/probes/host_api.py [c2,c4]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import bench
    env = bench.Env()
    for conf in (sys.argv[1] if len(sys.argv) > 1 else "c2,c4").split(","):
        wl = bench.Workload(env, conf)
        r = bench.host_api_leg(env, wl)
        print(conf, json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "what"} for k, v in r.items()}), flush=True)
        wl.dm.close()


if __name__ == "__main__":
    main()
