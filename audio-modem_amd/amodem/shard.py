"""Frame sharding across GPUs (one process per GPU, torch.distributed).

OFDM frames are independent (modem.js decodes each with no cross-frame state,
modem.js:557, 770), so a batch splits into contiguous frame ranges, one per rank,
balanced by sample count; each rank decodes its range on its own device with no
data-path collective. Only the 96-byte result records (and, if wanted, the
payload slots) travel back to rank 0, through one all-gather of fixed-size
buffers (RCCL over xGMI with the nccl backend, gloo on CPU), or — for the device-
resident bench path — one gather into rank 0 (`gather_to_root`).
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


def gather_to_root(rows, counts: list[int], dst: int = 0, group=None):
    """Gather every rank's rows (a uint8 tensor [counts[rank], width], device-resident
    under RCCL) to rank `dst`, in rank order, without leaving the device.

    This is the C4 collective of SURVEY.md §8e: one gather (RCCL over xGMI, point to
    point into the root) of the fixed-size result records and of the payload slots;
    no all-reduce, no halo exchange. Rows are padded to the largest count so one
    fixed-size collective suffices. Returns the [sum(counts), width] tensor on `dst`
    and None elsewhere."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(counts) != world or rows.shape[0] != counts[rank] or rows.dtype != torch.uint8 or rows.dim() != 2:
        raise ValueError(f"gather_to_root: rows {tuple(rows.shape)} {rows.dtype} vs counts {counts} at rank {rank}")
    m = max(counts)
    buf = rows
    if rows.shape[0] != m:
        buf = torch.zeros((m, rows.shape[1]), dtype=torch.uint8, device=rows.device)
        buf[: rows.shape[0]] = rows
    buf = buf.contiguous()
    if dist.get_backend(group) == "gloo" and buf.is_cuda:  # gloo gathers host buffers only
        buf = buf.cpu()
    outs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, outs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([outs[r][: counts[r]] for r in range(world)])


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


# ------------------------------------------------------- sharded stream receive --
BLOCK = 4096        # ScriptProcessor block (app.js:1103)
EMA_CHUNK = 8192    # k_ema chunk: shard boundaries and lo sit on multiples of it
EMA_WARM = 2 * 65536  # samples of history before a shard's first block (EMA convergence)


def _after_key(st) -> tuple:
    return (st.block, st.state, st.ac_init, st.ac_pos, st.pre_pos, st.frame_end, st.meta_received, st.chunk_size)


def stream_bounds(n: int, world: int, halo: int) -> list[tuple[int, int, int, int]]:
    """(lo, hi, own_lo, own_hi) per rank for an n-sample stream: owned block ranges of
    nearly equal length on EMA-chunk boundaries; lo = own_lo - EMA_WARM (history for
    the DC removal), hi = own_hi + halo (the continuation that meets the next shard)."""
    npad = -(-n // BLOCK) * BLOCK
    nch = -(-npad // EMA_CHUNK)
    cuts = [min(npad, (nch * r // world) * EMA_CHUNK) for r in range(world)] + [npad]
    out = []
    for r in range(world):
        own_lo, own_hi = cuts[r], cuts[r + 1]
        lo = max(0, own_lo - EMA_WARM)
        hi = min(npad, -(-(own_hi + halo) // BLOCK) * BLOCK)
        out.append((lo, hi, own_lo, own_hi))
    return out


def merge_trajectories(shards: list[dict]) -> tuple[list, list, list[str]]:
    """Rank-ordered shard results -> the receiver's true trajectory. Shard 0 is true
    from its start; shard k's speculative trajectory is adopted from the first window
    that the true run (carried from shard k-1 into its halo) also demodulated from the
    identical post-reset state: both continue identically from there (_resetToIdle
    re-initialises the scan). Returns (events [(event, payload row)], fails [(block,
    pos)], warnings)."""
    warn = []
    traj = [(e, p) for e, p in zip(shards[0]["events"], shards[0]["payload"])]
    fails = list(shards[0]["fails"])
    for k in range(1, len(shards)):
        sk = shards[k]
        own_lo = sk["own_lo"]
        if not np.isnan(sk["ema"][0]) and sk["ema"][0] != shards[k - 1]["ema"][1]:
            warn.append(f"shard {k}: DC-removal state at its first sample differs from shard {k - 1}'s")
        idx = {}
        for j, e in enumerate(sk["events"]):
            idx.setdefault((e.frame.pos, e.frame.end) + _after_key(e.after), j)
        sync = None
        for i, (e, _) in enumerate(traj):
            if e.frame.pos < own_lo:
                continue
            j = idx.get((e.frame.pos, e.frame.end) + _after_key(e.after))
            if j is not None:
                sync = (i, j)
                break
        if sync is None:
            raise RuntimeError(f"shard {k}: no common window with the previous shard inside the halo")
        i, j = sync
        after_block = sk["events"][j].after.block
        fails = [f for f in fails if f[0] < traj[i][0].after.block] + \
                [f for f in sk["fails"] if f[0] >= after_block]
        traj = traj[: i + 1] + [(e, p) for e, p in zip(sk["events"][j + 1:], sk["payload"][j + 1:])]
    return traj, fails, warn


def dispatch_events(traj, assembler) -> dict:
    """StreamingReceiver._demodulateFrame's dispatch (app.js:926-961) of the merged
    trajectory into a ChunkAssembler; returns the receiver counters."""
    decoded = errors = 0
    rec = np.zeros(1, RESULT_DTYPE)
    for e, row in traj:
        r = e.frame.result
        rec.view(np.uint8)[:] = np.frombuffer(bytes(r), np.uint8)
        assembler.feed(rec, row[None, :])
    st = assembler.state()
    return {"frames_decoded": st["frames_decoded"], "frame_errors": st["frame_errors"]}


def stream_receive_sharded(dm, cfg, samples_for, n: int, rank: int, world: int, group=None, assembler=None):
    """The StreamingReceiver over an n-sample stream split across `world` ranks (one
    process per GPU). samples_for(lo, hi) returns stream samples [lo, hi) as float32
    (each rank reads only its slice). Rank 0 finds the metadata frame (its result sets
    every later window length) and broadcasts the receiver state after it; every rank
    runs its shard on its own GPU (no data-path collective); one gather brings the
    shards' windows, results and payload rows to rank 0, which merges them and feeds
    its ChunkAssembler. Returns (events, fails, counters, warnings) on rank 0, None
    elsewhere."""
    import torch.distributed as dist
    from . import _lib as L
    from .modem import estimate_frame_samples

    stride = None
    # phase A (rank 0): up to the metadata frame, one window at a time
    if rank == 0:
        lo, hi = 0, min(-(-n // BLOCK) * BLOCK, max(EMA_CHUNK, 64 * BLOCK * 16))
        init = L.StreamState()  # the receiver as constructed (app.js:706-745)
        init.pre_pos = init.frame_end = -1
        while True:
            evA, payA, failsA, _, endA = dm.stream_shard(cfg, samples_for(lo, hi), lo, hi, 0, min(hi, EMA_CHUNK),
                                                          start=init, until_meta=True)
            if endA.meta_received or hi >= -(-n // BLOCK) * BLOCK:
                break
            hi = min(-(-n // BLOCK) * BLOCK, 2 * hi)  # no metadata yet: look further
        msg = [bytes(endA), [bytes(e) for e in evA], payA, failsA]
    else:
        msg = [None, None, None, None]
    if world > 1:
        dist.broadcast_object_list(msg, src=0, group=group)
    endA = L.StreamState.from_buffer_copy(msg[0])
    chunk = endA.chunk_size if endA.meta_received else 0
    mod = {0: "BPSK", 1: "QPSK", 2: "QAM16"}[cfg.modulation]
    win = estimate_frame_samples((chunk or 4096) + 11 if endA.meta_received else 280, mod, cfg.repetition)
    halo = 4 * (win + cfg.sample_rate) + 2 * EMA_CHUNK
    bounds = stream_bounds(n, world, halo)
    lo, hi, own_lo, own_hi = bounds[rank]
    from .modem import payload_stride
    stride = payload_stride(cfg, win)
    if rank == 0:
        ev, pay, fl, ema, end = dm.stream_shard(cfg, samples_for(lo, hi), lo, hi, own_lo, own_hi, start=endA,
                                                stride=stride)
        evA = [L.StreamEvent.from_buffer_copy(b) for b in msg[1]]
        payA = np.asarray(msg[2], np.uint8).reshape(len(evA), -1) if len(evA) else np.zeros((0, stride), np.uint8)
        rowsA = np.zeros((len(evA), stride), np.uint8)
        w = min(stride, payA.shape[1])
        rowsA[:, :w] = payA[:, :w]
        ev = evA + ev
        pay = np.concatenate([rowsA, pay]) if len(evA) else pay
        fl = list(msg[3]) + fl
    else:
        ev, pay, fl, ema, end = dm.stream_shard(cfg, samples_for(lo, hi), lo, hi, own_lo, own_hi,
                                                meta_received=bool(endA.meta_received), chunk_size=chunk,
                                                stride=stride)
    mine = {"own_lo": own_lo, "events": [bytes(e) for e in ev], "payload": pay, "fails": fl, "ema": ema}
    gathered = [None] * world if rank == 0 else None
    if world > 1:
        dist.gather_object(mine, gathered, dst=0, group=group)
    else:
        gathered = [mine]
    if rank != 0:
        return None
    for g in gathered:
        g["events"] = [L.StreamEvent.from_buffer_copy(b) for b in g["events"]]
    traj, fails, warn = merge_trajectories(gathered)
    # A metadata frame past phase A that changes the window length (metaReceived /
    # chunkSize, app.js:889-896, 939-949) invalidates every later window the shards cut
    # with the old length: rank 0 keeps the trajectory up to it and re-runs the rest of
    # the stream from the receiver state right after it (updated), until no change is left.
    npad = -(-n // BLOCK) * BLOCK
    meta, chunk_now = bool(endA.meta_received), chunk
    i = len(msg[1])  # events before it are phase A's (already applied)
    while i < len(traj):
        r = traj[i][0].frame.result
        if r.status == 0 and r.frame_type == 0xFE and r.crc_valid:
            new_meta = meta or r.total_chunks > -8  # apply_meta (stream.cpp): bitmap allocation throws at <= -8
            new_chunk = r.chunk_size
            if new_meta != meta or (new_meta and new_chunk != chunk_now):
                st = L.StreamState.from_buffer_copy(bytes(traj[i][0].after))
                st.meta_received, st.chunk_size = int(new_meta), int(new_chunk)
                warn.append(f"metadata change at stream sample {traj[i][0].frame.pos}: "
                            f"the rest re-run from there on rank 0")
                own = st.block * BLOCK
                lo2 = max(0, (own - EMA_WARM) // EMA_CHUNK * EMA_CHUNK)
                # (payload rows as wide as the longest window the new chunk size cuts:
                # dispatch feeds them one by one)
                ev2, pay2, fl2, _, _ = dm.stream_shard(cfg, samples_for(lo2, npad), lo2, npad, own, npad, start=st,
                                                       chunk_size=int(new_chunk) if new_meta else 0)
                fails = [f for f in fails if f[0] < st.block] + [f for f in fl2 if f[0] >= st.block]
                traj = traj[: i + 1] + list(zip(ev2, pay2))
                meta, chunk_now = new_meta, new_chunk
        i += 1
    counters = dispatch_events(traj, assembler) if assembler is not None else {}
    return traj, fails, counters, warn
