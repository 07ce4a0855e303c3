"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/).

Every check here is bit-exact: the oracle restates modem.js in IEEE double with
the same operation order, and the fixtures were produced by the unmodified
reference (tests/golden/gen_golden.js).
"""
import ctypes as C

import numpy as np
import pytest

from helpers import frames, kat, ref_dict, sha, struct_to_dict
from oracle import oracle as O


def test_crc32_kat():
    for k in kat()["crc32"]:
        assert O.crc32(bytes.fromhex(k["hex"])) == k["crc"], k["label"]
    assert O.crc32(b"123456789") == 0xCBF43926


def test_seeded_random():
    for seed, seq in kat()["seededRandom"].items():
        st = C.c_double(float(seed))
        got = [O.lib().orc_seeded_next(C.byref(st)) for _ in seq]
        assert got == seq


@pytest.mark.parametrize("name", ["standard", "acoustic", "narrowband"])
def test_config_templates(name):
    k = kat()["configs"][name]
    c = O.cfg(name)
    assert (c.fft_size, c.cp_len, c.symbol_len, c.sample_rate, c.sub_start, c.sub_end) == \
        (k["FFT_SIZE"], k["CP_LEN"], k["SYMBOL_LEN"], k["SAMPLE_RATE"], k["SUB_START"], k["SUB_END"])
    assert O.pilots(c) == k["PILOTS"]
    assert O.lib().orc_num_data_subs(C.byref(c)) == k["numDataSubs"]
    p1 = np.zeros(c.symbol_len, np.float32)
    O.lib().orc_preamble1(C.byref(c), p1)
    assert p1.tolist() == k["pre1"]
    p2 = np.zeros(c.symbol_len, np.float32)
    O.lib().orc_preamble2(C.byref(c), p2)
    assert p2.tolist() == k["pre2"]
    ce = np.zeros(c.symbol_len, np.float32)
    known = np.zeros(c.fft_size)
    O.lib().orc_ce_symbol(C.byref(c), ce, known)
    assert ce.tolist() == k["ceSamples"]
    assert known[c.sub_start:c.sub_end + 1].tolist() == k["knownRe"]
    for e in k["estimateFrameSamples"]:
        assert O.lib().orc_estimate_frame_samples(C.byref(c), e["payload"], O.MODS[e["mod"]], e["rep"]) == e["samples"]


def test_fft_vectors():
    for v in kat()["fft"]:
        fr, fi = O.fft(v["inRe"], v["inIm"])
        assert fr.tolist() == v["fftRe"] and fi.tolist() == v["fftIm"], v["label"]
        if "ifftRe" in v:
            ir, ii = O.fft(v["inRe"], v["inIm"], inverse=True)
            assert ir.tolist() == v["ifftRe"] and ii.tolist() == v["ifftIm"], v["label"]


def test_constellations_and_demap():
    for m, spec in kat()["constellations"].items():
        for i, (pr, pi) in enumerate(spec["points"]):
            a, b = C.c_double(), C.c_double()
            O.lib().orc_const_point(O.MODS[m], i, C.byref(a), C.byref(b))
            assert (a.value, b.value) == (pr, pi)
    for m, pts in kat()["demap"].items():
        bps = kat()["constellations"][m]["bps"]
        for p in pts:
            idx = O.lib().orc_demap(O.MODS[m], p["re"], p["im"])
            assert [(idx >> (bps - 1 - j)) & 1 for j in range(bps)] == p["bits"], (m, p)


def test_majority_and_pack():
    for v in kat()["majorityVote"]:
        bits = np.array(v["bits"] + [0], np.uint8)
        out = np.zeros(len(bits), np.uint8)
        n = O.lib().orc_majority(bits, len(v["bits"]), v["n"], out)
        assert out[:n].tolist() == v["out"]
    for v in kat()["bitsToBytes"]:
        bits = np.array(v["bits"] + [0], np.uint8)
        out = np.zeros(len(bits) // 8 + 1, np.uint8)
        n = O.lib().orc_bits_to_bytes(bits, len(v["bits"]), out)
        assert out[:n].tobytes().hex() == v["hex"]


def test_preprocess_kat():
    for v in kat()["preprocess"]:
        out, _, _ = O.preprocess(np.array(v["x"], np.float32))
        assert out.tolist() == v["out"], v["label"]


def test_payload_recipe():
    k = kat()["payloadXs32"]
    assert O.payload(k["seed"], 16).tobytes().hex() == k["hex16"]


def _packbits(bits):
    return np.packbits(bits).tobytes().hex() if len(bits) else ""


@pytest.mark.parametrize("case", frames(), ids=lambda c: c["name"])
def test_frame_parity(case):
    c = O.cfg(case["config"])
    x = O.build_case(case)
    assert len(x) == case["n"]
    assert sha(x) == case["sigSha"], "synthetic signal differs from the reference TX"
    inter = case["inter"]
    if case["rx"] == "legacy":
        sig, mean, mx = O.preprocess(x)
        if len(x):
            assert mean == inter["mean"] and mx == inter["mx"]
        assert sha(sig) == inter["preSha"]
        coarse = O.detect_preamble(c, sig)
        assert coarse == inter["coarseIdx"]
        if coarse >= 0:
            start, best = O.fine_timing(c, sig, coarse)
            assert start == inter["startIdx"]
            if inter["fineMetric"] is not None:
                assert best == inter["fineMetric"]
        data0 = inter.get("startIdx", 0) + 3 * c.symbol_len
        ce0 = data0 - c.symbol_len
    else:
        sig = x
        ce0, data0 = 2 * c.symbol_len, 3 * c.symbol_len
    if "H" in inter:
        hr, hi = O.estimate_channel(c, sig[ce0:ce0 + c.symbol_len])
        assert hr[c.sub_start:c.sub_end + 1].tolist() == inter["H"]["re"]
        assert hi[c.sub_start:c.sub_end + 1].tolist() == inter["H"]["im"]
    if "nbits" in inter:
        data = sig[data0:]
        for s in range(min(2, inter["numSymbols"])):
            xr, xi, er, ei, ph = O.symbol_detail(c, data, s, hr, hi)
            band = slice(c.sub_start, c.sub_end + 1)
            d = inter[f"sym{s}"]
            assert xr[band].tolist() == d["fftRe"] and xi[band].tolist() == d["fftIm"]
            assert er[band].tolist() == d["eqRe"] and ei[band].tolist() == d["eqIm"]
            assert ph == inter["phases"][s]
        bits = O.demodulate(c, data, case["mod"], hr, hi)
        assert len(bits) == inter["nbits"]
        assert _packbits(bits) == inter["bitsHex"]
    rec, payload = O.decode(c, x, case["mod"], case["rep"], chunk=case["rx"] == "chunk")
    if "bytesHex" in inter:
        assert payload.tobytes().hex() == inter["bytesHex"]
    got = ref_dict(struct_to_dict(rec), payload.tobytes(), via_legacy=case["rx"] == "legacy")
    assert got == case["result"]
