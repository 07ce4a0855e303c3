#!/usr/bin/env python3
"""Diagnostics: the streaming receiver's host sub-phases (AMOD_STREAM_DIAG=1 prints them on
stderr) over a C4-shaped stream of N chunks, host samples and device-resident.
  python tools/stream_diag.py [nchunks]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32000
    env = bench.Env()
    bench.stream_leg(env, 2000)  # warm-up run (tables, kernels, pinned buffers)
    os.environ["AMOD_STREAM_DIAG"] = "1"
    r = bench.stream_leg(env, n)
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
