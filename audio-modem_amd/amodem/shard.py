"""Frame sharding across GPUs (one process per GPU, torch.distributed).

OFDM frames are independent (modem.js decodes each with no cross-frame state,
modem.js:557, 770), so a batch splits into contiguous frame ranges, one per rank,
balanced by sample count; each rank decodes its range on its own device with no
data-path collective. Only the 96-byte result records (and, if wanted, the
payload slots) travel back to rank 0, through one all-gather of fixed-size
buffers (RCCL over xGMI with the nccl backend, gloo on CPU).
"""
from __future__ import annotations

import numpy as np

from .modem import RESULT_DTYPE


def partition_frames(lengths, world: int) -> list[tuple[int, int]]:
    """Contiguous [start, end) frame ranges, one per rank, with nearly equal sample
    counts: rank r takes the frames whose first sample falls in the r-th 1/world
    of the total."""
    lengths = np.asarray(lengths, np.int64)
    n = len(lengths)
    if world < 1:
        raise ValueError("world must be >= 1")
    starts = np.concatenate([[0], np.cumsum(lengths)[:-1]]) if n else np.zeros(0, np.int64)
    total = int(lengths.sum())
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        cuts.append(max(cuts[-1], int(np.searchsorted(starts, target, side="left"))))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def gather_records(records: np.ndarray, payload: np.ndarray | None, counts: list[int], group=None,
                   device=None):
    """All-gather every rank's result records (and payload rows) in rank order.

    records: RESULT_DTYPE array of this rank's frames; payload: uint8 [n, stride] or None.
    counts: frames per rank (from partition_frames). Returns (records, payload) of the
    whole batch on every rank. Buffers are padded to the largest count so one
    fixed-size collective suffices."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    assert len(counts) == world and len(records) == counts[rank]
    m = max(counts) if counts else 0
    dev = device if device is not None else torch.device("cpu")

    def allgather_rows(rows: np.ndarray, width: int) -> np.ndarray:
        buf = torch.zeros((m, width), dtype=torch.uint8, device=dev)
        if len(rows):
            buf[: len(rows)] = torch.from_numpy(np.ascontiguousarray(rows).view(np.uint8).reshape(len(rows), width))
        out = torch.empty((world * m, width), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, buf, group=group)
        out = out.cpu().numpy().reshape(world, m, width)
        return np.concatenate([out[r, : counts[r]] for r in range(world)]) if world else out.reshape(0, width)

    rec = allgather_rows(records, RESULT_DTYPE.itemsize).reshape(-1).view(RESULT_DTYPE)
    pay = None
    if payload is not None:
        pay = allgather_rows(payload, payload.shape[1])
    return rec, pay


def decode_sharded(dm, samples: np.ndarray, offsets, lengths, cfg, mode, group=None):
    """Decode this rank's share of a host batch on its own GPU, then all-gather the
    results. `dm` is the rank's amodem.Demodulator (opened on its local device)."""
    import torch.distributed as dist

    from .modem import payload_stride

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    offsets = np.asarray(offsets, np.int64)
    lengths = np.asarray(lengths, np.int32)
    parts = partition_frames(lengths, world)
    a, b = parts[rank]
    stride = payload_stride(cfg, int(lengths.max()) if len(lengths) else 0)  # one width on every rank
    rec, pay = dm.decode_batch(samples, offsets[a:b], lengths[a:b], cfg=cfg, mode=mode, stride=stride)
    dev = None
    if dist.get_backend(group) == "nccl":  # RCCL moves device buffers only
        import torch
        dev = torch.device("cuda", dm.device)
    return gather_records(rec, pay, [e - s for s, e in parts], group, device=dev)
