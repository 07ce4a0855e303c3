"""bench.py's printed line: the driver parses ONE stdout line, and round 5's 20.9 KB line
was not parsed (BENCH_r05.json `parsed: null`). `compact_line` keeps the contract keys,
the whole roofline and cpu_baseline objects and one-number summaries of every leg, under
LINE_MAX bytes; the full object goes to a side file (no GPU needed: recorded objects)."""
import json
import os

import bench
from helpers import ROOT

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic")
CPU = ("value", "unit", "cores", "kind", "sample")


def recorded():
    """Full objects the default run printed in earlier rounds (r05: the unparsed 20.9 KB one)."""
    out = []
    with open(os.path.join(ROOT, "profiles", "r05", "final", "bench_default_last.json")) as f:
        out.append(json.load(f))
    with open(os.path.join(ROOT, "profiles", "r04", "final", "bench_default.log")) as f:
        lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
    out.append(json.loads(lines[-1]))
    return out


def test_line_bounded_and_complete():
    for full in recorded():
        line = json.dumps(bench.compact_line(full, "gpurun_out/bench_full.json"), separators=(",", ":"))
        assert len(line) <= bench.LINE_MAX, len(line)
        obj = json.loads(line)
        for k in REQUIRED:
            assert k in obj, k
        assert obj["value"] == full["value"] and obj["ms_per_step"] == full["ms_per_step"]
        assert obj["config"] == full["config"]
        for k in ROOF:
            assert obj["roofline"][k] == full["roofline"][k], k
        for k in CPU:
            assert k in obj["cpu_baseline"], k
        assert obj["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]
        assert obj["full"] == "gpurun_out/bench_full.json"
        assert "truncated" not in obj
        # every leg is summarised with its rate and oracle agreement
        for name, leg in full["legs"].items():
            assert name in obj["legs"]
            if "value" in leg:
                assert abs(obj["legs"][name]["value"] / leg["value"] - 1) < 1e-3
                assert "oracle_agree" in obj["legs"][name]


def test_oversized_object_still_carries_the_contract():
    full = recorded()[0]
    full = dict(full, legs={f"leg{i}": full["legs"]["c5_10db"] for i in range(40)})
    obj = bench.compact_line(full)
    line = json.dumps(obj, separators=(",", ":"))
    assert len(line) <= bench.LINE_MAX and obj.get("truncated")
    for k in REQUIRED:
        assert k in obj


def test_full_object_written(tmp_path, monkeypatch):
    p = tmp_path / "full.json"
    monkeypatch.setenv("AMOD_BENCH_FULL", str(p))
    full = recorded()[0]
    assert bench.write_full(full) == str(p)
    assert json.loads(p.read_text()) == full
