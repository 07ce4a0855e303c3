"""Sharded streaming receive (raw single stream): two ranks (processes,
gloo for the small control/gather collectives) each run amod_stream_shard on their
slice of one C4-shaped stream on the GPU; rank 0 merges the trajectories
(amodem.shard.merge_trajectories) and assembles the file. The merged result must equal
the single-process receiver's: every window, result, failed refinement, counter and
the file."""
import json
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(n_chunks, chunk=1024):
    import amodem
    from amodem import _lib as L
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0x5AD, n_chunks * chunk - 77)
    parts = [np.zeros(3000, np.float32), amodem.build_metadata_frame(n_chunks, len(data), chunk, "sh.bin", cfg=cfg)]
    for i in range(n_chunks):
        parts.append(amodem.build_data_chunk_frame(data[i * chunk:(i + 1) * chunk], i, cfg=cfg))
        parts.append(np.zeros((i * 1231) % 5000, np.float32))
    x = np.concatenate(parts + [np.zeros(30000, np.float32)])
    x = np.concatenate([x, np.zeros(-len(x) % 4096, np.float32)])
    return cfg, x, data


def _worker(rank, world, port, out, n_chunks):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "audio-modem_amd"))
    import torch.distributed as dist
    import amodem
    from amodem import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, x, data = _stream(n_chunks)
    dm = amodem.Demodulator(0)
    asm = amodem.ChunkAssembler() if rank == 0 else None
    res = shard.stream_receive_sharded(dm, cfg, lambda lo, hi: x[lo:hi], len(x), rank, world, assembler=asm)
    if rank == 0:
        traj, fails, counters, warn = res
        ref_asm = amodem.ChunkAssembler()
        frames, rfails, stats = dm.stream_receive(cfg, x, ref_asm)
        got = [(int(e.frame.pos), int(e.frame.end), int(e.frame.window_len), bytes(e.frame.result).hex())
               for e, _ in traj]
        want = [(int(f["pos"]), int(f["end"]), int(f["window_len"]), f["result"].tobytes().hex()) for f in frames]
        rec = {"same_frames": got == want, "n": len(got), "n_ref": len(want),
               "fails": [p for _, p in fails], "ref_fails": rfails, "warn": warn,
               "counters": counters, "ref_counters": [stats["frames_decoded"], stats["frame_errors"]],
               "file_ok": asm.is_complete() and asm.assemble_file() == data,
               "ref_file_ok": ref_asm.is_complete() and ref_asm.assemble_file() == data}
        with open(out, "w") as f:
            json.dump(rec, f)
    dm.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_chunks", [(2, 60), (3, 90)])
def test_sharded_stream_equals_single(tmp_path, world, n_chunks):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.json")
    mp.spawn(_worker, args=(world, _free_port(), out, n_chunks), nprocs=world, join=True)
    rec = json.load(open(out))
    assert rec["same_frames"], rec
    assert rec["n"] == n_chunks + 1 and rec["fails"] == rec["ref_fails"] and rec["warn"] == []
    assert [rec["counters"]["frames_decoded"], rec["counters"]["frame_errors"]] == rec["ref_counters"]
    assert rec["file_ok"] and rec["ref_file_ok"]
