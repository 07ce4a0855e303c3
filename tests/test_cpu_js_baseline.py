"""Pin the JavaScript CPU baseline (oracle/rx_cpu.js, the reference RX restated in JS and
timed on the GPU box's host cores by bench.py) to the reference's own outputs: every
golden frame (tests/golden/frames.json, produced by the unmodified modem.js) must decode
to the identical result object, and its worker-thread bench driver must report the
outcomes of the frames it timed."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import ROOT, frames
from oracle import oracle as O

NODE = shutil.which("node")
JS = os.path.join(ROOT, "oracle", "rx_cpu.js")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")


def _write(tmp_path, sigs, **spec):
    lens = [len(s) for s in sigs]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64).tolist() if sigs else []
    x = np.concatenate(sigs).astype(np.float32) if sigs else np.zeros(1, np.float32)
    p = tmp_path / "x.f32"
    x.tofile(p)
    spec.update(samples=str(p), offsets=offs, lengths=lens)
    sp = tmp_path / "spec.json"
    sp.write_text(json.dumps(spec))
    return str(sp)


def test_golden_frames_bit_exact(tmp_path):
    cases = frames()
    sigs = [O.build_case(c) for c in cases]
    sp = _write(tmp_path, sigs, presets=[c["config"] for c in cases], mods=[c["mod"] for c in cases],
                reps=[c["rep"] for c in cases], chunks=[c["rx"] == "chunk" for c in cases])
    out = json.loads(subprocess.run([NODE, JS, "decode", sp], capture_output=True, text=True, check=True).stdout)
    assert len(out) == len(cases)
    for c, r in zip(cases, out):
        assert r == c["result"], c["name"]


def test_bench_driver_reports_outcomes(tmp_path):
    """Two worker threads over a few noisy and clean C2-shaped frames: the per-frame
    status and CRC the driver reports equal the C oracle's."""
    c = O.cfg("standard")
    sigs = []
    for i in range(6):
        x = O.build_tx(c, {"kind": "legacy", "seed": 0x9E3779B9 ^ i, "len": 1024, "name": "f.bin", "mod": "QPSK",
                           "rep": 1})
        sigs.append(O.add_noise(x, 12, 100 + i) if i % 2 else x)
    sp = _write(tmp_path, sigs, preset="standard", mod="QPSK", rep=1, chunk=False, threads=2, seconds=0,
                single_frames=2, single_seconds=0)
    r = json.loads(subprocess.run([NODE, JS, "bench", sp], capture_output=True, text=True, check=True).stdout)
    assert r["threads"] == 2 and r["all_cores"] > 0 and r["single_core"] > 0
    for i, x in enumerate(sigs):
        rec, _ = O.decode(c, x, "QPSK", 1, chunk=False)
        assert r["status"][i] == rec.status, i
        if rec.status == 0:
            assert r["crc"][i] == rec.actual_crc, i
