#!/usr/bin/env python3
"""Diagnostics: bench.py's soft_chunk_leg alone (C5 acoustic BPSK rep3 256 B chunk
windows at 1.76 dB, soft vs hard vote, oracle agreement of the hard vote)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench

    class A:
        steps, warmup, frames = 10, 5, 0
    env = bench.Env()
    out = bench.soft_chunk_leg(env, A())
    for k in ("hard", "soft"):
        print(k, json.dumps(out[k]))
    print("oracle", out.get("oracle_agree"))


if __name__ == "__main__":
    main()
