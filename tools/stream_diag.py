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
    # warm-up run (tables, kernels, pinned buffers): 2000 chunks, or `same` = n chunks (the
    # bench's own warm-up: every buffer and the assembler arena at their final size)
    bench.stream_leg(env, n if len(sys.argv) > 2 and sys.argv[2] == "same" else 2000)
    os.environ["AMOD_STREAM_DIAG"] = "1"
    r = bench.stream_leg(env, n)
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main()
