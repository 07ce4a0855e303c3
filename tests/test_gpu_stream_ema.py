"""processAudioBlock's DC removal (app.js:751-755) on the GPU: the parallel EMA (chunk
contributions, affine-map scan, per-chunk warm-up from the approximate state, bit
comparison of every chunk boundary, in-order recomputation of the ones that differ)
must equal the sequential IEEE-double recurrence sample for sample (oracle
orc_dc_remove), including the end state, on signals built to stress it: DC steps, long
silences, tiny and huge samples, lengths that are not multiples of the chunk."""
import ctypes as C

import numpy as np
import pytest

import amodem
from amodem import _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _signal(n, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = 0.3 * np.sin(2 * np.pi * t / 97.3) + 0.05 * rng.standard_normal(n)
    x += np.where((t // 50000) % 3 == 1, 0.7, -0.2)            # DC steps
    x[(t % 400000) < 30000] = 0.0                                # silences
    x[rng.integers(0, n, 200)] = rng.choice([1e-30, -3e-9, 7e-20, 1e-38], 200)
    x[rng.integers(0, n, 50)] = rng.choice([30.0, -45.0, 1e4], 50)  # clipping bursts
    return x.astype(np.float32)


@pytest.mark.parametrize("n,seed", [(1, 1), (777, 2), (1024, 3), (100_003, 4), (3_000_000, 5)])
def test_dc_remove_bit_exact(n, seed):
    import torch
    x = _signal(n, seed)
    ref, ref_state = O.dc_remove(x)
    dev = torch.device("cuda", 0)
    dx = torch.from_numpy(x).to(dev)
    dy = torch.empty_like(dx)
    dm = amodem.Demodulator(0)
    st, fixed = C.c_double(), C.c_int64()
    torch.cuda.synchronize()
    L.check(L.load().amod_dc_remove_device(dm.ctx, dx.data_ptr(), n, dy.data_ptr(), C.byref(st), C.byref(fixed), None),
            dm.ctx)
    y = dy.cpu().numpy()
    dm.close()
    bad = np.nonzero(y.view(np.uint32) != ref.view(np.uint32))[0]
    assert bad.size == 0, (bad[:5], y[bad[:5]], ref[bad[:5]], fixed.value)
    assert st.value == ref_state
