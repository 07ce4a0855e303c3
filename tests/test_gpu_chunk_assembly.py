"""C4 end to end at test size: a file cut into 2 KB chunks, framed by the GPU
transmitter (metadata frame + data-chunk frames, modem.js:758-766), cut into the
windows StreamingReceiver hands to decodeChunkFrame (pre1 onwards, length
estimateFrameSamples(chunkSize + 11 | 280), per-window peak normalisation,
app.js:892-925), decoded on the GPU in chunk mode, and assembled by the host
ChunkAssembler (app.js:597-704): the file comes back bit for bit. A duplicated chunk
is suppressed and a corrupted chunk counts as a CRC error and stays missing."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L

pytestmark = pytest.mark.gpu


def test_file_round_trip_through_chunks():
    cfg = amodem.preset("standard", "QPSK", 1)
    chunk = 2048
    data = amodem.synth_payload(0xC4C4C4C4, 9 * chunk + 777)
    nch = (len(data) + chunk - 1) // chunk
    pkts = [amodem.packet_meta(nch, len(data), chunk, "c4.bin")]
    kinds = [L.TX_META]
    order = list(range(nch)) + [3]  # chunk 3 sent twice
    for s in order:
        pkts.append(amodem.packet_chunk(data[s * chunk:(s + 1) * chunk], s))
        kinds.append(L.TX_CHUNK)
    dm = amodem.Demodulator(0)
    sig, offs, lens = dm.transmit_batch(cfg, pkts, kinds)
    # StreamingReceiver windows: from pre1, estimateFrameSamples(maxPayload) samples
    wins = []
    for i in range(len(pkts)):
        pre, _ = amodem.tx_silence(cfg, kinds[i])
        start = offs[i] + pre
        n = amodem.estimate_frame_samples(280 if i == 0 else chunk + 11, "QPSK", 1)
        w = np.zeros(n, np.float32)
        seg = sig[start:start + n]
        w[:len(seg)] = seg
        mx = float(np.max(np.abs(w)))
        if mx > 1e-6:
            w = (w.astype(np.float64) / mx).astype(np.float32)
        wins.append(w)
    wins[5] = wins[5].copy()
    wins[5][3000:3100] = 0.5  # corrupt chunk 4's data symbols
    wl = np.array([len(w) for w in wins], np.int32)
    wo = np.concatenate([[0], np.cumsum(wl)[:-1]]).astype(np.int64)
    rec, pay = dm.decode_batch(np.concatenate(wins), wo, wl, cfg=cfg, mode=L.MODE_CHUNK)
    dm.close()
    assert (rec["status"] == 0).all()
    assert rec[0]["frame_type"] == amodem.FRAME_META and rec[0]["crc_valid"] == 1
    assert int(rec[5]["crc_valid"]) == 0 and (rec["crc_valid"][np.arange(len(rec)) != 5] == 1).all()
    a = amodem.ChunkAssembler()
    a.feed(rec, pay)
    st = a.state()
    assert (st["total_chunks"], st["total_size"], st["chunk_size"]) == (nch, len(data), chunk)
    assert st["crc_errors"] == 1 and st["received"] == nch - 1 and not st["complete"]
    assert a.get_missing_chunks() == [4] and a.file_name() == b"c4.bin"
    # the retransmission of chunk 4 completes the file
    assert a.handle_data_chunk(4, data[4 * chunk:5 * chunk], True)
    assert a.is_complete() and a.assemble_file() == data
