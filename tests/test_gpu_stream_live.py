"""Live per-block streaming receive (StreamingReceiver.processAudioBlock, app.js:749-773)
against the reference: the golden streams of tests/golden/stream.json fed one
4096-sample block per call, as the reference's ScriptProcessor callback feeds them
(app.js:1103-1112), must produce exactly the windows, results, failed refinements,
counters, final scan position, assembler state and offered file the reference
produced; and on a C4-shaped stream the live receiver equals the recorded-stream one."""
import hashlib

import numpy as np
import pytest

from test_gpu_stream import build_stream, c4_stream, result_view, streams

import amodem

pytestmark = pytest.mark.gpu


def _feed(cfg, x, asm, block=4096):
    dm = amodem.Demodulator(0)
    rx = amodem.StreamingReceiver(dm, cfg, asm)
    frames = []
    for b0 in range(0, len(x), block):
        f = rx.process_audio_block(x[b0:b0 + block])
        if f is not None:
            frames.append(f)
    st, fails = rx.state(), rx.refine_fails()
    rx.close()
    dm.close()
    return frames, fails, st


@pytest.mark.parametrize("sp", streams(), ids=lambda s: s["name"])
def test_live_blocks_match_reference(sp):
    cfg, x, data = build_stream(sp)
    assert hashlib.sha256(x.tobytes()).hexdigest() == sp["sha256"]
    asm = amodem.ChunkAssembler()
    frames, fails, st = _feed(cfg, x, asm)
    got = [{"pos": int(f["pos"]), "end": int(f["end"]), "len": int(f["window_len"]), **result_view(f["result"])}
           for f in frames]
    assert got == [{k: v for k, v in w.items() if k != "fileName"} for w in sp["frames"]]
    assert fails == sp["refineFail"]
    assert (st["frames_decoded"], st["frame_errors"]) == (sp["framesDecoded"], sp["frameErrors"])
    assert (st["state"], st["ac_pos"]) == (sp["final"]["state"], sp["final"]["acScanPos"])
    assert st["total_written"] == len(x)
    a = asm.state()
    ref = sp["assembler"]
    assert (a["total_chunks"], a["total_size"], a["chunk_size"], a["received"], a["crc_errors"], bool(a["complete"])) == \
        (ref["totalChunks"], ref["totalFileSize"], ref["chunkSize"], ref["receivedCount"], ref["crcErrors"],
         ref["complete"])
    if sp["offered"] is not None:
        f = asm.assemble_file()
        assert hashlib.sha256(f).hexdigest() == sp["offered"]["sha256"]


def test_live_equals_recorded_on_c4_stream():
    cfg, x, data, _ = c4_stream(120)
    asm = amodem.ChunkAssembler()
    frames, fails, st = _feed(cfg, x, asm)
    dm = amodem.Demodulator(0)
    ref, ref_fails, ref_st = dm.stream_receive(cfg, x, amodem.ChunkAssembler())
    dm.close()
    assert len(frames) == len(ref) == 121 and fails == ref_fails == []
    for f, r in zip(frames, ref):
        assert (int(f["pos"]), int(f["end"]), int(f["window_len"])) == (int(r["pos"]), int(r["end"]), int(r["window_len"]))
        for k in ("status", "frame_type", "seq_num", "data_len", "expected_crc", "actual_crc", "crc_valid"):
            assert f["result"][k] == r["result"][k], k
    assert asm.is_complete() and asm.assemble_file() == data
