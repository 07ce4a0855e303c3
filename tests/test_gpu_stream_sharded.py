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


def _stream(n_chunks, chunk=1024, second=None):
    """Metadata + n_chunks data frames with varying gaps. second = (after, n2, chunk2):
    after `after` chunks a second file starts mid-stream (its metadata frame changes
    the chunk size, hence every later window length); data = the file the stream ends with."""
    import amodem
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0x5AD, n_chunks * chunk - 77)
    parts = [np.zeros(3000, np.float32), amodem.build_metadata_frame(n_chunks, len(data), chunk, "sh.bin", cfg=cfg)]
    last = n_chunks if second is None else second[0]
    for i in range(last):
        parts.append(amodem.build_data_chunk_frame(data[i * chunk:(i + 1) * chunk], i, cfg=cfg))
        parts.append(np.zeros((i * 1231) % 5000, np.float32))
    if second is not None:
        _, n2, c2 = second
        data = amodem.synth_payload(0x5AE, n2 * c2 - 5)
        parts.append(amodem.build_metadata_frame(n2, len(data), c2, "two.bin", cfg=cfg))
        # the metadata frame's window is cut with the old (data-frame) length: silence
        # after it, so the receiver does not resume past the next frame's preamble
        parts.append(np.zeros(60000, np.float32))
        for i in range(n2):
            parts.append(amodem.build_data_chunk_frame(data[i * c2:(i + 1) * c2], i, cfg=cfg))
            parts.append(np.zeros((i * 733) % 4000, np.float32))
    x = np.concatenate(parts + [np.zeros(30000, np.float32)])
    x = np.concatenate([x, np.zeros(-len(x) % 4096, np.float32)])
    return cfg, x, data


def _worker(rank, world, port, out, n_chunks, second=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "audio-modem_amd"))
    import torch.distributed as dist
    import amodem
    from amodem import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, x, data = _stream(n_chunks, second=second)
    dm = amodem.Demodulator(0)
    asm = amodem.ChunkAssembler() if rank == 0 else None
    res = shard.stream_receive_sharded(dm, cfg, lambda lo, hi: x[lo:hi], len(x), rank, world, assembler=asm)
    if rank == 0:
        traj, fails, counters, warn = res
        ref_asm = amodem.ChunkAssembler()
        dref = dm if os.environ.get("AMOD_TEST_REUSE_CTX") else amodem.Demodulator(0)  # fresh context
        frames, rfails, stats = dref.stream_receive(cfg, x, ref_asm)
        if dref is not dm:
            dref.close()
        got = [(int(e.frame.pos), int(e.frame.end), int(e.frame.window_len), bytes(e.frame.result).hex())
               for e, _ in traj]
        want = [(int(f["pos"]), int(f["end"]), int(f["window_len"]), f["result"].tobytes().hex()) for f in frames]
        diffs = []
        for i, (g, w) in enumerate(zip(got, want)):
            if g == w:
                continue
            rg = np.frombuffer(bytes.fromhex(g[3]), amodem.RESULT_DTYPE)[0]
            rw = np.frombuffer(bytes.fromhex(w[3]), amodem.RESULT_DTYPE)[0]
            fd = {n: (str(rg[n]), str(rw[n])) for n in amodem.RESULT_DTYPE.names if str(rg[n]) != str(rw[n])}
            diffs.append({"i": i, "got": g[:3], "want": w[:3], "fields": fd})
        # what the reference receiver exposes (app.js:907-972): window, outcome and the
        # decodeChunkFrame fields; `same_bytes` compares whole records (flags /
        # payload_valid / fine_metric / coarse_idx too: every window batch reserves its own
        # longest window, so a window's route depends on the window only)
        vis = [n for n in amodem.RESULT_DTYPE.names
               if n not in ("flags", "payload_valid", "fine_metric", "coarse_idx", "reserved")]
        def key(t):
            r = np.frombuffer(bytes.fromhex(t[3]), amodem.RESULT_DTYPE)[0]
            return t[:3] + tuple(int(r[n]) for n in vis)
        rec = {"same_frames": [key(t) for t in got] == [key(t) for t in want], "same_bytes": got == want,
               "n": len(got), "n_ref": len(want), "diffs": diffs[:8],
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
    assert rec["same_frames"], rec["diffs"]
    assert rec["same_bytes"], rec["diffs"]  # whole records, engine-side fields included
    assert rec["n"] == n_chunks + 1 and rec["fails"] == rec["ref_fails"] and rec["warn"] == []
    assert [rec["counters"]["frames_decoded"], rec["counters"]["frame_errors"]] == rec["ref_counters"]
    assert rec["file_ok"] and rec["ref_file_ok"]


def test_sharded_stream_second_file_mid_stream(tmp_path):
    """A second metadata frame (a new file with a larger chunk size) lands inside rank 1's
    shard: the windows the shards cut after it with the old length are dropped and rank 0
    re-runs the rest with the new one; the merged trajectory still equals the
    single-process receiver's, which rolls back the same way (stream.cpp)."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.json")
    mp.spawn(_worker, args=(2, _free_port(), out, 60, (40, 12, 2048)), nprocs=2, join=True)
    rec = json.load(open(out))
    assert rec["same_frames"], rec["diffs"]
    assert rec["n"] == rec["n_ref"] == 40 + 1 + 12 + 1 and rec["fails"] == rec["ref_fails"]
    assert [rec["counters"]["frames_decoded"], rec["counters"]["frame_errors"]] == rec["ref_counters"]
    assert rec["file_ok"] and rec["ref_file_ok"]
    assert any("metadata change" in w for w in rec["warn"])
