"""Chunk assembly (app.js ChunkAssembler 597-704) against the reference class itself:
tests/golden/assembler.json holds the reference's state after every step of scripted
scenarios (in order, shuffled, duplicates, CRC errors, out-of-range and negative
sequence numbers, overflowing chunks, negative sizes, re-sent metadata, assembling
before any metadata) and the assembled file or the error it threw. Memory and
file-backed stores both replay them exactly. No GPU needed."""
import json
import os

import pytest

from helpers import GOLDEN

import amodem


def scenarios():
    with open(os.path.join(GOLDEN, "assembler.json")) as f:
        return json.load(f)["scenarios"]


def payload_bytes(seed, n):  # gen_assembler.js payloadBytes (xorshift32, little-endian)
    return amodem.synth_payload(seed, n)


def check_state(a, want, name):
    st = a.state()
    assert st["total_chunks"] == want["totalChunks"], name
    assert st["total_size"] == want["totalFileSize"], name
    assert st["chunk_size"] == want["chunkSize"], name
    assert st["received"] == want["receivedCount"], name
    assert st["crc_errors"] == want["crcErrors"], name
    assert bool(st["complete"]) == want["complete"], name
    assert st["bitmap_len"] == want["bitmapLen"], name
    if want["bitmap"] is not None:
        assert a.bitmap()[:64].tolist() == want["bitmap"], name
    if want["missing"] is not None:
        assert a.get_missing_chunks() == want["missing"], name
    assert a.file_name() == (want["fileName"] or "").encode(), name


@pytest.mark.parametrize("store", ["memory", "files"])
@pytest.mark.parametrize("name", sorted(scenarios()))
def test_reference_scenarios(name, store, tmp_path):
    sc = scenarios()[name]
    a = amodem.ChunkAssembler(str(tmp_path) if store == "files" else None)
    for op, step in zip(sc["ops"], sc["steps"]):
        err, got = None, None
        try:
            if op["op"] == "meta":
                a.handle_metadata_frame(op["totalChunks"], op["totalFileSize"], op["chunkSize"], op["fileName"].encode())
            elif op["op"] == "chunk":
                a.handle_data_chunk(op["seq"], payload_bytes(op["seed"], op["len"]), op["crc"])
            else:
                got = a.assemble_file().hex()
        except amodem.AssemblerError as e:
            err = e.name
        assert err == step["error"], (name, op)
        assert got == step["file"], (name, op)
        check_state(a, step["state"], (name, op))
    a.close()


def test_feed_dispatch_counts():
    """StreamingReceiver's dispatch: errors and bad metadata CRC count as frame errors."""
    import numpy as np
    rec = np.zeros(4, amodem.RESULT_DTYPE)
    pay = np.zeros((4, 32), np.uint8)
    rec["status"] = [0, 0, 1, 0]
    rec["frame_type"] = [0xFE, 0xFE, -1, 0xFF]
    rec["crc_valid"] = [0, 1, 0, 1]
    rec[1]["total_chunks"], rec[1]["total_size"], rec[1]["chunk_size"] = 1, 3, 3
    rec[1]["name_off"], rec[1]["name_len"] = 0, 2
    pay[1, :2] = [ord("o"), ord("k")]
    rec[3]["seq_num"], rec[3]["data_off"], rec[3]["data_len"] = 0, 4, 3
    pay[3, 4:7] = [1, 2, 3]
    a = amodem.ChunkAssembler()
    a.feed(rec, pay)
    st = a.state()
    assert (st["frames_decoded"], st["frame_errors"], st["received"], st["complete"]) == (3, 2, 1, 1)
    assert a.file_name() == b"ok" and a.assemble_file() == bytes([1, 2, 3])
