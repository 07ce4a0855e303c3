#!/usr/bin/env python3
"""Diagnostics: the bench's streaming-receiver leg alone (C4-shaped stream), for
rocprofv3 --kernel-trace --stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))

import bench  # noqa: E402
import amodem  # noqa: E402
from amodem import _lib as L  # noqa: E402

print(bench.stream_leg(amodem, L, 0, int(sys.argv[1]) if len(sys.argv) > 1 else 2000))
