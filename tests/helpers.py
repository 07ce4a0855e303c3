"""Shared test helpers: golden-fixture loading and reference-shaped results."""
from __future__ import annotations

import functools
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))

ERRORS = {
    1: "Preamble not detected",
    2: "Preamble not detected (low correlation)",
    3: "Signal too short for CE",
    4: "No data after CE",
    5: "Decoded data too short",
    6: "Decoded data too short for header",
    8: "Metadata frame too short",
    9: "Metadata frame truncated",
    10: "Data chunk frame too short",
    11: "Data chunk truncated",
    12: "Frame too short for CE",
}


@functools.lru_cache(None)
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


@functools.lru_cache(None)
def frames():
    with open(os.path.join(GOLDEN, "frames.json")) as f:
        return json.load(f)["frames"]


@functools.lru_cache(None)
def loopback():
    with open(os.path.join(GOLDEN, "loopback.json")) as f:
        return json.load(f)["loopback"]


def frame(name):
    for c in frames():
        if c["name"] == name:
            return c
    raise KeyError(name)


def open_with_env(device=0, **env):
    """A Demodulator opened under the given AMOD_* knobs (libamodem reads them once,
    when a context opens: amod::Knobs); the process environment is restored after."""
    import amodem
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return amodem.Demodulator(device)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def sha(x: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def text_decode(b: bytes) -> str:
    """TextDecoder().decode: UTF-8, replacement characters, leading BOM dropped."""
    if b[:3] == b"\xef\xbb\xbf":
        b = b[3:]
    return b.decode("utf-8", errors="replace")


def ref_dict(rec, payload: bytes, via_legacy: bool) -> dict:
    """Format a decode record the way modem.js returns it (golden JSON shape:
    Uint8Array fields are {'hex': ...}). `rec` has the amod_result/orc_result fields."""
    st = int(rec["status"])
    ft = int(rec["frame_type"])
    chunkish = ft in (0xFE, 0xFF)
    out: dict
    if st == 0:
        if ft == 0xFE:
            nm = payload[rec["name_off"]:rec["name_off"] + rec["name_len"]]
            out = {"frameType": 254, "totalChunks": int(rec["total_chunks"]), "totalFileSize": int(rec["total_size"]),
                   "chunkSize": int(rec["chunk_size"]), "fileName": text_decode(nm)}
        elif ft == 0xFF:
            d = payload[rec["data_off"]:rec["data_off"] + rec["data_len"]]
            out = {"frameType": 255, "seqNum": int(rec["seq_num"]), "data": {"hex": d.hex()},
                   "dataLen": int(rec["data_len"])}
        else:
            d = payload[rec["data_off"]:rec["data_off"] + rec["data_len"]]
            nm = payload[rec["name_off"]:rec["name_off"] + rec["name_len"]]
            out = {"data": {"hex": d.hex()}, "dataLen": int(rec["data_len"]), "fileName": text_decode(nm)}
        out.update({"crcValid": bool(rec["crc_valid"]), "expectedCRC": int(rec["expected_crc"]) & 0xFFFFFFFF,
                    "actualCRC": int(rec["actual_crc"]) & 0xFFFFFFFF})
        if ft == 0:
            out.update({"preambleIdx": int(rec["preamble_idx"]), "frameType": "legacy"})
        elif via_legacy:
            out["preambleIdx"] = int(rec["preamble_idx"])
        return out
    if st == 7:
        return {"error": f"Invalid data length: {int(rec['aux'])}"}
    if st == 13:
        return {"error": f"Unknown frame type: 0x{int(rec['aux']):x}", "frameType": int(rec["aux"])}
    out = {"error": ERRORS[st]}
    if via_legacy and chunkish and st in (8, 9, 10, 11):
        out["preambleIdx"] = int(rec["preamble_idx"])
    return out


def struct_to_dict(s) -> dict:
    return {f[0]: getattr(s, f[0]) for f in s._fields_}
