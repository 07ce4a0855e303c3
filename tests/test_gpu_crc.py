"""k_demod's frame-end CRC-32 (modem.js:443-457) at message lengths around its chunking:
16-byte chunks (chunk 0 left-padded from the inverse-shift register table), one pass up to
kCrcMats chunks (8 KB), the block-carry form beyond. Legacy frames whose CRC covers
[0, 1 + nameLen + 4 + dataLen) bytes: every length class gives the oracle's CRC and a valid
check, on the fast path (flags 0)."""
import numpy as np
import pytest

import amodem
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("plen", [1, 6, 7, 8, 22, 1024, 2000, 4096, 8170, 8171, 8172, 8187, 8200, 12000])
def test_crc_lengths(plen):
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0xC0C0 + plen, plen)
    x = amodem.build_transmit_signal(data, file_name="f.bin", cfg=cfg)  # CRC over 10 + plen bytes
    dm = amodem.Demodulator(0)
    rec, pay = dm.decode_batch(x, [0], [len(x)], cfg=cfg)
    dm.close()
    r, refpay = O.decode(O.cfg("standard"), x, "QPSK", 1, False)
    assert int(rec["status"][0]) == r.status == 0
    assert int(rec["actual_crc"][0]) == r.actual_crc and int(rec["crc_valid"][0]) == 1
    assert int(rec["flags"][0]) == 0, hex(int(rec["flags"][0]))
    d = amodem.to_reference(rec[0], pay[0].tobytes(), True)
    assert d["data"] == data


@pytest.mark.parametrize("rep", [2, 3, 4, 5, 7])
def test_vote_repetitions(rep):
    """majorityVote over the unrolled (rep 2-5) and generic (7) wave votes: BPSK legacy
    frames decode to the oracle's bytes and CRC."""
    cfg = amodem.preset("standard", "BPSK", rep)
    data = amodem.synth_payload(0xB0B0 + rep, 300)
    x = amodem.build_transmit_signal(data, file_name="v.bin", cfg=cfg)
    dm = amodem.Demodulator(0)
    rec, pay = dm.decode_batch(x, [0], [len(x)], cfg=cfg)
    dm.close()
    r, _ = O.decode(O.cfg("standard"), x, "BPSK", rep, False)
    assert int(rec["status"][0]) == r.status == 0 and int(rec["actual_crc"][0]) == r.actual_crc
    assert amodem.to_reference(rec[0], pay[0].tobytes(), True)["data"] == data
