"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol
include/amodem.h declares, and its host-side (reference-equivalent) utilities —
presets, preamble template, CRC-32, transmit builders — match the reference's
golden vectors bit for bit."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from helpers import ROOT, frames, kat, sha

import amodem
from amodem import _lib as L


def header_symbols():
    src = open(os.path.join(ROOT, "include", "amodem.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(amod_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    lib = L.load()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(L.SIGNATURES), "ctypes signatures out of sync with the header"


def test_struct_layouts():
    assert C.sizeof(L.Result) == 96
    assert C.sizeof(L.Cfg) == 4 * (7 + 32 + 2)
    assert amodem.RESULT_DTYPE.itemsize == 96


@pytest.mark.parametrize("name", ["standard", "acoustic", "narrowband", "bogus"])
def test_presets_match_reference(name):
    k = kat()["configs"].get(name, kat()["configs"]["standard"])  # unknown -> standard (modem.js:96)
    c = amodem.preset(name, "QPSK", 1)
    assert (c.fft_size, c.cp_len, c.symbol_len, c.sub_start, c.sub_end) == \
        (k["FFT_SIZE"], k["CP_LEN"], k["SYMBOL_LEN"], k["SUB_START"], k["SUB_END"])
    assert [c.pilots[i] for i in range(c.npilots)] == k["PILOTS"]
    assert L.load().amod_num_data_subs(C.byref(c)) == k["numDataSubs"]
    assert amodem.generate_preamble_symbol1(c).tolist() == k["pre1"]
    for e in k["estimateFrameSamples"]:
        cc = amodem.preset(name, e["mod"], e["rep"])
        assert L.load().amod_estimate_frame_samples(C.byref(cc), e["payload"]) == e["samples"]


def test_crc32():
    for k in kat()["crc32"]:
        assert amodem.crc32(bytes.fromhex(k["hex"])) == k["crc"]


def test_payload_generator():
    k = kat()["payloadXs32"]
    assert amodem.synth_payload(k["seed"], 16).hex() == k["hex16"]


TX_CASES = [c for c in frames() if c["tx"]["kind"] in ("legacy", "meta", "chunk", "test")]


@pytest.mark.parametrize("case", TX_CASES, ids=lambda c: c["name"])
def test_tx_builders_match_reference(case):
    tx = case["tx"]
    cfg = amodem.preset(case["config"], tx.get("mod", case["mod"]), tx.get("rep", case["rep"]))
    if tx["kind"] == "legacy":
        sig = amodem.build_transmit_signal(amodem.synth_payload(tx["seed"], tx["len"]), file_name=tx["name"], cfg=cfg)
    elif tx["kind"] == "meta":
        sig = amodem.build_metadata_frame(tx["totalChunks"], tx["totalFileSize"], tx["chunkSize"], tx["name"], cfg=cfg)
    elif tx["kind"] == "chunk":
        sig = amodem.build_data_chunk_frame(amodem.synth_payload(tx["seed"], tx["len"]), tx["seq"], cfg=cfg)
    else:
        sig, _ = amodem.generate_test_signal(cfg=cfg)
    assert len(sig) == case["txLen"]
    assert sha(sig) == case["txSha"]


def test_synth_batch_layout():
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 5, payload_len=1024, first=3, threads=2)
    assert (lens == 35874).all() and (np.diff(offs) == 35874).all()
    one = amodem.build_transmit_signal(amodem.synth_payload(0x9E3779B9 ^ 4, 1024), file_name="f.bin", cfg=cfg)
    assert np.array_equal(x[offs[1]:offs[1] + lens[1]], one)


def test_payload_stride():
    cfg = amodem.preset("standard", "QPSK", 1)
    s = amodem.payload_stride(cfg, 35874)
    assert s % 16 == 0 and s >= (35874 // 576) * 410 // 8


def test_pipe_rejects_bad_arguments_without_a_gpu():
    """amod_pipe_*: argument errors come back as AMOD_ERR_ARG before any HIP call (NULL
    contexts, a NULL pipe); a NULL pipe has no next stream and closes as a no-op (the same
    context twice: tests/test_gpu_pipe.py, it needs a real context)."""
    lib = L.load()
    h = C.c_void_p()
    assert lib.amod_pipe_open(None, None, C.byref(h)) == -1
    assert not h.value
    cfg = amodem.make_cfg("QPSK", 1)
    assert lib.amod_pipe_decode_device(None, C.byref(cfg), 0, None, None, None, 0, None, None, 16, 0, None) == -1
    assert lib.amod_pipe_flush(None, None) == -1
    assert lib.amod_pipe_synchronize(None) == -1
    assert not lib.amod_pipe_next_stream(None)
    assert lib.amod_pipe_close(None) == 0
