"""The golden stream recipes rebuild bit for bit on the CPU (product TX builders +
oracle post-ops), so the GPU-side stream tests start from the reference's exact input."""
import hashlib

import pytest

from test_gpu_stream import build_stream, streams


@pytest.mark.parametrize("sp", streams(), ids=lambda s: s["name"])
def test_stream_recipe_rebuilds(sp):
    _, x, _ = build_stream(sp)
    assert len(x) == sp["n"] and hashlib.sha256(x.tobytes()).hexdigest() == sp["sha256"]
