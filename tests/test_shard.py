"""Multi-GPU sharding logic (audio-modem_amd/amodem/shard.py) on CPU: frame
partitioning balanced by samples, and the result all-gather over gloo with
world_size 2 (the same code runs over RCCL with one process per GPU)."""
import os
import socket

import numpy as np
import pytest

from amodem import RESULT_DTYPE
from amodem.shard import gather_records, partition_frames


def test_partition_covers_and_balances():
    rng = np.random.default_rng(7)
    lens = rng.integers(16000, 40000, 1000)
    for world in (1, 2, 3, 4, 8):
        parts = partition_frames(lens, world)
        assert parts[0][0] == 0 and parts[-1][1] == len(lens)
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        loads = [int(lens[a:b].sum()) for a, b in parts]
        assert max(loads) - min(loads) <= 2 * int(lens.max())


def test_partition_edge_cases():
    assert partition_frames([], 4) == [(0, 0)] * 4
    assert partition_frames([100], 3) == [(0, 1), (1, 1), (1, 1)]
    assert partition_frames([5, 5, 5, 5], 2) == [(0, 2), (2, 4)]
    with pytest.raises(ValueError):
        partition_frames([1, 2], 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, nframes, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lens = (np.arange(nframes) % 7 + 1) * 1000
        parts = partition_frames(lens, world)
        a, b = parts[rank]
        rec = np.zeros(b - a, RESULT_DTYPE)
        rec["status"] = np.arange(a, b)  # stand-in per-frame outcome: the frame index
        rec["preamble_idx"] = rank
        pay = np.zeros((b - a, 32), np.uint8)
        pay[:, 0] = np.arange(a, b) & 0xFF
        allrec, allpay = gather_records(rec, pay, [e - s for s, e in parts])
        q.put((rank, allrec["status"].tolist(), allrec["preamble_idx"].tolist(), allpay[:, 0].tolist()))
    finally:
        dist.destroy_process_group()


def test_gather_records_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n = 37
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    parts = partition_frames((np.arange(n) % 7 + 1) * 1000, 2)
    owner = [r for r, (a, b) in enumerate(parts) for _ in range(a, b)]
    for rank, status, pidx, p0 in out:
        assert status == list(range(n))            # rank order = frame order
        assert pidx == owner                       # each frame decoded by its owner
        assert p0 == [i & 0xFF for i in range(n)]  # payload rows follow their records
