"""The fast kernel answers clean frames itself: no exact-path routing on the presets
whose fine search window fits its LDS stage (standard, acoustic). A regression here
is a silent slowdown (the exact replica still gives the right bytes), so it is pinned
on the flags the kernel reports, not on the results."""
import numpy as np
import pytest

import amodem

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset", ["standard", "acoustic"])
@pytest.mark.parametrize("mod", ["BPSK", "QPSK", "QAM16"])
def test_clean_frames_stay_on_fast_path(preset, mod):
    cfg = amodem.preset(preset, mod, 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 64, payload_len=512, threads=8)
    dm = amodem.Demodulator(0)
    rec, _ = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    assert (rec["status"] == 0).all() and (rec["crc_valid"] == 1).all()
    flags = rec["flags"] & ~(1 << 15)
    assert (flags == 0).all(), np.unique(flags)
