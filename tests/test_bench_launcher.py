"""bench.py --gpus N: the launcher's world-size logic (no GPU needed).

A rank started by torch.distributed.run runs in place with the environment's world; a
bare `bench.py --gpus N` (N > 1) starts N ranks itself, and refuses when RCCL cannot give
each rank its own device; the gloo rehearsal may share devices."""
import os
import subprocess
import sys

import bench
from helpers import ROOT


def test_rank_runs_in_place():
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}, 8, "nccl") == ("run", 8)
    assert bench.launch_plan(1, {"WORLD_SIZE": "2"}, 1, "gloo") == ("run", 2)


def test_single_gpu_runs_in_place():
    assert bench.launch_plan(1, {}, 0, "nccl") == ("run", 1)
    assert bench.launch_plan(1, {}, 8, "nccl") == ("run", 1)


def test_spawns_n_ranks():
    assert bench.launch_plan(8, {}, 8, "nccl") == ("spawn", 8)
    assert bench.launch_plan(2, {}, 8, "nccl") == ("spawn", 2)
    assert bench.launch_plan(2, {}, 1, "gloo") == ("spawn", 2)


def test_too_few_devices_fails():
    kind, msg = bench.launch_plan(2, {}, 1, "nccl")
    assert kind == "error" and "only 1 GPU" in msg
    assert bench.launch_plan(4, {}, 0, "gloo")[0] == "error"


def test_cli_fails_loudly_without_gpus():
    """This container has no GPU: `bench.py --gpus 2` must exit non-zero with the reason,
    before any rank starts."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr, (r.returncode, r.stderr[-500:])
