"""ctypes view of the CPU oracle (oracle/amodem_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product (audio-modem_amd/).

Besides the receive-chain restatement it rebuilds the synthetic signals the
golden fixtures describe as recipes (tests/golden/gen_golden.js: payload
xorshift32, transmit builders, noise, slicing) so fixtures stay small.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

MODS = {"BPSK": 0, "QPSK": 1, "QAM16": 2}


class Cfg(C.Structure):
    _fields_ = [("fft_size", C.c_int), ("cp_len", C.c_int), ("symbol_len", C.c_int),
                ("sample_rate", C.c_int), ("sub_start", C.c_int), ("sub_end", C.c_int),
                ("npilots", C.c_int), ("pilots", C.c_int * 32)]


class Result(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("status", "preamble_idx", "coarse_idx", "frame_type", "aux",
                                          "nbytes", "name_off", "name_len", "data_off", "data_len",
                                          "seq_num", "total_chunks", "total_size", "chunk_size")] + \
               [("expected_crc", C.c_uint32), ("actual_crc", C.c_uint32), ("crc_valid", C.c_int32),
                ("nbits", C.c_int32), ("fine_metric", C.c_double)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        cfgp = C.POINTER(Cfg)
        sig = {
            "orc_config": (None, [C.c_char_p, cfgp]),
            "orc_num_data_subs": (C.c_int, [cfgp]),
            "orc_fft": (None, [f64p, f64p, C.c_int, C.c_int]),
            "orc_seeded_next": (C.c_double, [C.POINTER(C.c_double)]),
            "orc_preamble1": (None, [cfgp, f32p]),
            "orc_preamble2": (None, [cfgp, f32p]),
            "orc_ce_symbol": (None, [cfgp, f32p, f64p]),
            "orc_const_point": (None, [C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
            "orc_demap": (C.c_int, [C.c_int, C.c_double, C.c_double]),
            "orc_crc32": (C.c_uint32, [C.c_char_p, C.c_size_t]),
            "orc_majority": (C.c_int, [u8p, C.c_int, C.c_int, u8p]),
            "orc_bits_to_bytes": (C.c_int, [u8p, C.c_int, u8p]),
            "orc_estimate_frame_samples": (C.c_int, [cfgp, C.c_int, C.c_int, C.c_int]),
            "orc_preprocess": (None, [f32p, C.c_int, f32p, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
            "orc_dc_remove": (None, [f32p, C.c_long, f32p, C.POINTER(C.c_double)]),
            "orc_detect_preamble": (C.c_int, [f32p, C.c_int, cfgp]),
            "orc_fine_timing": (C.c_int, [f32p, C.c_int, cfgp, C.c_int, C.POINTER(C.c_double)]),
            "orc_estimate_channel": (None, [f32p, cfgp, f64p, f64p]),
            "orc_symbol_detail": (None, [f32p, C.c_int, C.c_int, cfgp, f64p, f64p, f64p, f64p, f64p, f64p,
                                         C.POINTER(C.c_double)]),
            "orc_demodulate": (C.c_int, [f32p, C.c_int, cfgp, C.c_int, f64p, f64p, u8p]),
            "orc_decode_received": (C.c_int, [cfgp, f32p, C.c_int, C.c_int, C.c_int, C.POINTER(Result), u8p, C.c_int]),
            "orc_decode_chunk": (C.c_int, [cfgp, f32p, C.c_int, C.c_int, C.c_int, C.POINTER(Result), u8p, C.c_int]),
            "orc_build_legacy": (C.c_int, [cfgp, C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_void_p]),
            "orc_build_meta": (C.c_int, [cfgp, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_void_p]),
            "orc_build_chunk": (C.c_int, [cfgp, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]),
            "orc_build_test_signal": (C.c_int, [cfgp, C.c_int, C.c_int, C.c_void_p]),
            "orc_xs32": (C.c_uint32, [C.c_uint32]),
            "orc_payload": (None, [C.c_uint32, C.c_int, u8p]),
            "orc_add_noise": (None, [f32p, C.c_int, C.c_int, C.c_uint32, f32p]),
            "orc_add_noise_div": (None, [f32p, C.c_int, C.c_double, C.c_uint32, f32p]),
            "orc_bench_decode": (C.c_double, [cfgp, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                              C.c_int, C.c_void_p, C.c_void_p]),
            "orc_bench_decode_chunk": (C.c_double, [cfgp, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                              C.c_int, C.c_void_p, C.c_void_p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def cfg(name: str) -> Cfg:
    c = Cfg()
    lib().orc_config(name.encode(), C.byref(c))
    return c


def pilots(c: Cfg):
    return [c.pilots[i] for i in range(c.npilots)]


# ----------------------------------------------------------------- recipes --
def payload(seed: int, length: int) -> np.ndarray:
    out = np.zeros(max(length, 1), np.uint8)
    lib().orc_payload(seed & 0xFFFFFFFF, length, out)
    return out[:length]


def _build(fn, *args):
    n = fn(*args, None)
    out = np.zeros(max(n, 1), np.float32)
    fn(*args, out.ctypes.data_as(C.c_void_p))
    return out[:n]


def build_tx(c: Cfg, tx: dict) -> np.ndarray:
    L = lib()
    k = tx["kind"]
    if k == "legacy":
        data = payload(tx["seed"], tx["len"]).tobytes()
        name = tx["name"].encode("utf-8")
        return _build(L.orc_build_legacy, C.byref(c), data, len(data), name, len(name), MODS[tx["mod"]], tx["rep"])
    if k == "meta":
        name = tx["name"].encode("utf-8")
        return _build(L.orc_build_meta, C.byref(c), tx["totalChunks"], tx["totalFileSize"], tx["chunkSize"],
                      name, len(name), MODS[tx["mod"]], tx["rep"])
    if k == "chunk":
        data = payload(tx["seed"], tx["len"]).tobytes()
        return _build(L.orc_build_chunk, C.byref(c), data, len(data), tx["seq"], MODS[tx["mod"]], tx["rep"])
    if k == "test":
        return _build(L.orc_build_test_signal, C.byref(c), MODS[tx["mod"]], tx["rep"])
    if k == "zeros":
        return np.zeros(tx["n"], np.float32)
    if k == "periodic":
        vals = np.asarray(tx["values"], np.float32)
        return np.resize(vals, tx["n"]).astype(np.float32)
    raise ValueError(k)


def add_noise(x: np.ndarray, snr: int, seed: int, div: float | None = None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    if len(x):
        if div is None:
            lib().orc_add_noise(x, len(x), snr, seed & 0xFFFFFFFF, out)
        else:
            lib().orc_add_noise_div(x, len(x), float(div), seed & 0xFFFFFFFF, out)
    return out


def apply_post(x: np.ndarray, post) -> np.ndarray:
    for op in post or []:
        if op["op"] == "slice":
            x = x[op["start"]:op.get("end")]
        elif op["op"] == "noise":
            x = add_noise(x, op.get("snr", 0), op["seed"], op.get("div"))
        elif op["op"] == "dc":
            x = (x.astype(np.float64) + op["dc"]).astype(np.float32)
        elif op["op"] == "gain":
            x = (x.astype(np.float64) * op["gain"]).astype(np.float32)
        else:
            raise ValueError(op)
    return np.ascontiguousarray(x, np.float32)


def build_case(case: dict) -> np.ndarray:
    c = cfg(case["config"])
    return apply_post(build_tx(c, case["tx"]), case.get("post"))


# ----------------------------------------------------------------- decode --
def _f32(x):
    x = np.ascontiguousarray(x, np.float32)
    return x if len(x) else np.zeros(1, np.float32)


def decode(c: Cfg, x: np.ndarray, mod: str, rep: int, chunk: bool):
    n = len(x)
    xx = _f32(x)
    r = Result()
    cap = max(1, n // c.symbol_len * 221 * 4 // 8 + 8)
    buf = np.zeros(cap, np.uint8)
    fn = lib().orc_decode_chunk if chunk else lib().orc_decode_received
    fn(C.byref(c), xx, n, MODS[mod], rep, C.byref(r), buf, cap)
    return r, buf[:max(0, min(r.nbytes, cap))].copy()


def dc_remove(x: np.ndarray, state: float = 0.0):
    """processAudioBlock's EMA DC removal (app.js:751-755) -> (cleaned, end state)."""
    xx = _f32(x)
    out = np.zeros(len(xx), np.float32)
    st = C.c_double(state)
    lib().orc_dc_remove(xx, len(x), out, C.byref(st))
    return out[:len(x)], st.value


def preprocess(x: np.ndarray):
    xx = _f32(x)
    out = np.zeros(len(xx), np.float32)
    mean, mx = C.c_double(), C.c_double()
    lib().orc_preprocess(xx, len(x), out, C.byref(mean), C.byref(mx))
    return out[:len(x)], mean.value, mx.value


def detect_preamble(c: Cfg, sig: np.ndarray) -> int:
    return lib().orc_detect_preamble(_f32(sig), len(sig), C.byref(c))


def fine_timing(c: Cfg, sig: np.ndarray, coarse: int):
    best = C.c_double()
    idx = lib().orc_fine_timing(_f32(sig), len(sig), C.byref(c), coarse, C.byref(best))
    return idx, best.value


def estimate_channel(c: Cfg, ce: np.ndarray):
    hr = np.zeros(c.fft_size)
    hi = np.zeros(c.fft_size)
    lib().orc_estimate_channel(_f32(ce), C.byref(c), hr, hi)
    return hr, hi


def symbol_detail(c: Cfg, data: np.ndarray, s: int, hr, hi):
    n = c.fft_size
    xr, xi, er, ei = (np.zeros(n) for _ in range(4))
    ph = C.c_double()
    lib().orc_symbol_detail(_f32(data), len(data), s, C.byref(c), hr, hi, xr, xi, er, ei, C.byref(ph))
    return xr, xi, er, ei, ph.value


def demodulate(c: Cfg, data: np.ndarray, mod: str, hr, hi) -> np.ndarray:
    nsym = len(data) // c.symbol_len
    bits = np.zeros(max(1, nsym * 221 * 4), np.uint8)
    nb = lib().orc_demodulate(_f32(data), len(data), C.byref(c), MODS[mod], hr, hi, bits)
    return bits[:nb]


def fft(re, im, inverse=False):
    re = np.array(re, np.float64)
    im = np.array(im, np.float64)
    lib().orc_fft(re, im, len(re), 1 if inverse else 0)
    return re, im


def crc32(b: bytes) -> int:
    return lib().orc_crc32(b, len(b))


def bench_decode(c: Cfg, x: np.ndarray, offs: np.ndarray, lens: np.ndarray, mod: str, rep: int, threads: int,
                 chunk: bool = False):
    offs = np.ascontiguousarray(offs, np.int64)
    lens = np.ascontiguousarray(lens, np.int32)
    status = np.zeros(len(offs), np.int32)
    crc = np.zeros(len(offs), np.uint32)
    fn = lib().orc_bench_decode_chunk if chunk else lib().orc_bench_decode
    t = fn(C.byref(c), x.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(offs),
                               MODS[mod], rep, threads, status.ctypes.data, crc.ctypes.data)
    return t, status, crc
