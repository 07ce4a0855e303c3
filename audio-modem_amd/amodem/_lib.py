"""ctypes binding of libamodem.so (include/amodem.h).

This is the host plumbing the tests and bench.py use to drive the HIP product;
the JavaScript surface (audio-modem_amd/js/modem.js) binds the same C ABI through
N-API. There is no CPU fallback: if the library is missing this import fails.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(HERE), "lib")
LIB_PATH = os.environ.get("AMODEM_LIB") or os.path.join(LIB_DIR, "libamodem.so")  # override: experiments only

MAX_PILOTS = 32
BPSK, QPSK, QAM16 = 0, 1, 2
MODS = {"BPSK": BPSK, "QPSK": QPSK, "QAM16": QAM16}
MODE_RECEIVED, MODE_CHUNK, MODE_LOOPBACK = 0, 1, 2
TX_LEGACY, TX_META, TX_CHUNK = 0, 1, 2
OPT_FORCE_EXACT = 1
OPT_SOFT_COMBINE = 2  # not reference behaviour: soft repetition combining (opt-in)

OK = 0
E_CAPACITY = 100
# amod_kernel_stages slots
STAGE_DETECT, STAGE_DEMOD, STAGE_EXACT_B, STAGE_AUX, STAGE_JOIN_WAIT, STAGE_DEMOD_PATH, STAGE_COUNT = range(7)
FLAG_SPAN = 1 << 9
FLAG_SOFT = 1 << 10
FLAG_REPLAY = 1 << 11
FLAG_EXACT = 1 << 15


class Cfg(C.Structure):
    _fields_ = [("fft_size", C.c_int32), ("cp_len", C.c_int32), ("symbol_len", C.c_int32),
                ("sample_rate", C.c_int32), ("sub_start", C.c_int32), ("sub_end", C.c_int32),
                ("npilots", C.c_int32), ("pilots", C.c_int32 * MAX_PILOTS),
                ("modulation", C.c_int32), ("repetition", C.c_int32)]


class Result(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("status", "preamble_idx", "coarse_idx", "frame_type", "aux", "nbytes",
                                          "name_off", "name_len", "data_off", "data_len", "seq_num",
                                          "total_chunks", "total_size", "chunk_size")] + \
               [("expected_crc", C.c_uint32), ("actual_crc", C.c_uint32), ("crc_valid", C.c_int32),
                ("nbits", C.c_int32), ("flags", C.c_int32), ("fine_metric", C.c_float),
                ("payload_valid", C.c_int32), ("reserved", C.c_int32 * 3)]


DBG_BAND = 256
DBG_SYMS = 256


class Debug(C.Structure):
    _fields_ = [("mean", C.c_double), ("mx", C.c_double), ("coarse_metric", C.c_double),
                ("coarse_lo", C.c_int32), ("coarse_hi", C.c_int32), ("fine_metric", C.c_double),
                ("fine_idx", C.c_int32), ("nsym", C.c_int32),
                ("h_re", C.c_double * DBG_BAND), ("h_im", C.c_double * DBG_BAND),
                ("x_re", C.c_double * DBG_BAND), ("x_im", C.c_double * DBG_BAND),
                ("eq_re", C.c_double * DBG_BAND), ("eq_im", C.c_double * DBG_BAND),
                ("phase", C.c_double * DBG_SYMS)]


assert C.sizeof(Result) == 96, C.sizeof(Result)


class AsmState(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("total_chunks", "total_size", "chunk_size", "received", "crc_errors",
                                          "complete", "has_bitmap", "frames_decoded", "frame_errors", "name_len",
                                          "reserved")] + [("bitmap_len", C.c_int64)]


ASM_RANGE_ERROR, ASM_TYPE_ERROR = -10, -11
E_STREAM_LOST = 101


class StreamFrame(C.Structure):
    _fields_ = [("pos", C.c_int64), ("end", C.c_int64), ("window_len", C.c_int32), ("reserved", C.c_int32),
                ("result", Result)]


class StreamState(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("block", "ac_pos", "pre_pos", "frame_end")] + \
               [(n, C.c_double) for n in ("ac_p", "ac_ra", "ac_rb")] + \
               [(n, C.c_int32) for n in ("state", "ac_init", "meta_received", "chunk_size")]


class StreamEvent(C.Structure):
    _fields_ = [("frame", StreamFrame), ("after", StreamState)]


class StreamStats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("nframes", "nrefine_fail", "frames_decoded", "frame_errors", "final_state",
                                          "final_scan_pos", "ema_chunks_fixed", "fine_host_positions")] + \
               [(n, C.c_double) for n in ("t_ema_ms", "t_fine_ms", "t_decode_ms", "t_host_ms", "t_total_ms")]

class Shard(C.Structure):
    """amod_shard: one group member's device-resident batch (include/amodem.h)."""
    _fields_ = [("samples", C.c_void_p), ("offsets", C.c_void_p), ("lengths", C.c_void_p), ("results", C.c_void_p),
                ("payload", C.c_void_p), ("payload_stride", C.c_int64), ("stream", C.c_void_p),
                ("nframes", C.c_int32), ("reserved", C.c_int32)]


class LiveStats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("total_written", "frames_decoded", "frame_errors", "refine_fails",
                                          "last_refine_fail", "fine_host_positions")]


# (restype, argtypes) for every symbol the header declares
_P = C.c_void_p
# amod_progress_fn (include/amodem.h): void (*)(void *user, int32_t frames_done)
PROGRESS_FN = C.CFUNCTYPE(None, _P, C.c_int32)
SIGNATURES = {
    "amod_open": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "amod_close": (C.c_int, [_P]),
    "amod_last_error": (C.c_char_p, [_P]),
    "amod_abi_version": (C.c_int, []),
    "amod_config_preset": (C.c_int, [C.c_char_p, C.c_int32, C.c_int32, C.POINTER(Cfg)]),
    "amod_num_data_subs": (C.c_int32, [C.POINTER(Cfg)]),
    "amod_estimate_frame_samples": (C.c_int32, [C.POINTER(Cfg), C.c_int32]),
    "amod_payload_stride": (C.c_int64, [C.POINTER(Cfg), C.c_int64]),
    "amod_reserve": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, C.c_int64]),
    "amod_decode_device": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, _P, _P, C.c_int32, _P, _P, C.c_int64,
                                     C.c_uint32, _P]),
    "amod_decode_host": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, C.c_int64, _P, _P, C.c_int32, _P, _P,
                                   C.c_int64, C.c_uint32]),
    "amod_decode_host_progress": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, C.c_int64, _P, _P, C.c_int32, _P,
                                            _P, C.c_int64, C.c_uint32, _P, _P]),
    "amod_synchronize": (C.c_int, [_P]),
    "amod_pipe_open": (C.c_int, [_P, _P, C.POINTER(_P)]),
    "amod_pipe_close": (C.c_int, [_P]),
    "amod_pipe_next_stream": (_P, [_P]),
    "amod_pipe_decode_device": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, _P, _P, C.c_int32, _P, _P,
                                          C.c_int64, C.c_uint32, _P]),
    "amod_pipe_flush": (C.c_int, [_P, _P]),
    "amod_pipe_synchronize": (C.c_int, [_P]),
    "amod_set_profiling": (C.c_int, [_P, C.c_int]),
    "amod_kernel_breakdown": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "amod_kernel_stages": (C.c_int, [_P, C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_int64)]),
    "amod_aux_overlap": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    "amod_kernel_times": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                    C.POINTER(C.c_int64)]),
    "amod_decode_device_debug": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, _P, _P, C.c_int32, _P, _P,
                                           C.c_int64, C.c_uint32, _P, _P]),
    "amod_debug_stamps": (C.c_int64, [_P, _P, C.c_int64]),
    "amod_analyze_loopback": (C.c_int, [_P, C.POINTER(Cfg), _P, C.c_int64, _P, _P, _P, C.c_int64]),
    "amod_crc32": (C.c_uint32, [C.c_char_p, C.c_size_t]),
    "amod_preamble1": (C.c_int, [C.POINTER(Cfg), _P]),
    "amod_tx_legacy": (C.c_int64, [C.POINTER(Cfg), C.c_char_p, C.c_int32, C.c_char_p, C.c_int32, _P]),
    "amod_tx_meta": (C.c_int64, [C.POINTER(Cfg), C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32, _P]),
    "amod_tx_chunk": (C.c_int64, [C.POINTER(Cfg), C.c_char_p, C.c_int32, C.c_int32, _P]),
    "amod_tx_test_signal": (C.c_int64, [C.POINTER(Cfg), _P]),
    "amod_synth_payload": (None, [C.c_uint32, C.c_int32, _P]),
    "amod_packet_legacy": (C.c_int64, [C.c_char_p, C.c_int32, C.c_char_p, C.c_int32, _P]),
    "amod_packet_meta": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32, _P]),
    "amod_packet_chunk": (C.c_int64, [C.c_char_p, C.c_int32, C.c_int32, _P]),
    "amod_tx_silence": (C.c_int, [C.POINTER(Cfg), C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "amod_tx_frame_samples": (C.c_int64, [C.POINTER(Cfg), C.c_int64, C.c_int32, C.c_int32]),
    "amod_tx_device": (C.c_int, [_P, C.POINTER(Cfg), _P, _P, _P, _P, _P, C.c_int32, _P, _P, _P]),
    "amod_tx_host": (C.c_int64, [_P, C.POINTER(Cfg), _P, C.c_int64, _P, _P, _P, _P, C.c_int32, _P, _P]),
    "amod_asm_open": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "amod_asm_close": (C.c_int, [_P]),
    "amod_asm_metadata": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32]),
    "amod_asm_chunk": (C.c_int, [_P, C.c_int32, C.c_char_p, C.c_int32, C.c_int32]),
    "amod_asm_feed": (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32]),
    "amod_asm_state": (C.c_int, [_P, C.POINTER(AsmState)]),
    "amod_asm_bitmap": (C.c_int64, [_P, _P, C.c_int64]),
    "amod_asm_name": (C.c_int64, [_P, _P, C.c_int64]),
    "amod_asm_missing": (C.c_int64, [_P, _P, C.c_int64]),
    "amod_asm_file": (C.c_int64, [_P, _P, C.c_int64]),
    "amod_stream_receive": (C.c_int, [_P, C.POINTER(Cfg), _P, C.c_int64, _P, _P, C.c_int64, C.POINTER(C.c_int64),
                                      _P, C.c_int64, C.POINTER(StreamStats)]),
    "amod_stream_receive_device": (C.c_int, [_P, C.POINTER(Cfg), _P, C.c_int64, _P, _P, C.c_int64,
                                             C.POINTER(C.c_int64), _P, C.c_int64, C.POINTER(StreamStats)]),
    "amod_stream_shard": (C.c_int, [_P, C.POINTER(Cfg), _P, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                    C.POINTER(StreamState), C.c_int32, C.c_int32, C.c_int32, _P, C.c_int64,
                                    C.POINTER(C.c_int64), _P, C.c_int64, _P, C.c_int64, C.POINTER(C.c_int64), _P,
                                    C.POINTER(StreamState)]),
    "amod_synth_legacy_packets": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int32, _P, _P, _P]),
    "amod_group_open": (C.c_int, [_P, C.c_int32, C.POINTER(_P)]),
    "amod_group_close": (C.c_int, [_P]),
    "amod_group_size": (C.c_int32, [_P]),
    "amod_group_context": (_P, [_P, C.c_int32]),
    "amod_group_decode_host": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, C.c_int64, _P, _P, C.c_int32, _P, _P,
                                         C.c_int64, C.c_uint32, _P]),
    "amod_group_decode_device": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, _P, C.c_uint32]),
    "amod_group_synchronize": (C.c_int, [_P]),
    "amod_group_upload": (C.c_int, [_P, C.POINTER(Cfg), _P, C.c_int64, _P, _P, C.c_int32, C.POINTER(_P)]),
    "amod_resident_decode": (C.c_int, [_P, C.POINTER(Cfg), C.c_int32, C.c_uint32, _P, _P, C.c_int64]),
    "amod_resident_frames": (C.c_int32, [_P, _P]),
    "amod_resident_free": (C.c_int, [_P]),
    "amod_live_open": (C.c_int, [_P, C.POINTER(Cfg), _P, C.POINTER(_P)]),
    "amod_live_process_block": (C.c_int, [_P, _P, C.c_int64, _P, C.POINTER(C.c_int32)]),
    "amod_live_state": (C.c_int, [_P, C.POINTER(StreamState), C.POINTER(LiveStats)]),
    "amod_live_refine_fails": (C.c_int64, [_P, _P, C.c_int64]),
    "amod_live_close": (None, [_P]),
    "amod_dc_remove_device": (C.c_int, [_P, _P, C.c_int64, _P, C.POINTER(C.c_double), C.POINTER(C.c_int64), _P]),
    "amod_synth_legacy_batch": (C.c_int64, [C.POINTER(Cfg), C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                                            C.c_int32, _P, _P, _P, C.c_int32]),
}

_lib = None


def load():
    """Load libamodem.so (built by __graft_entry__.build / `make -C audio-modem_amd/csrc`)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 (same
        # SONAME as /opt/rocm's). If torch is importable, load it first so that
        # libamodem binds to the already-loaded runtime instead of a second copy.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libamodem.so not built: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.amod_abi_version() != 1:
            raise ImportError("libamodem ABI mismatch")
        _lib = L
    return _lib


def last_error(ctx=None) -> str:
    s = load().amod_last_error(ctx)
    return s.decode() if s else ""


def check(rc: int, ctx=None):
    if rc != 0:
        raise RuntimeError(f"libamodem error {rc}: {last_error(ctx)}")
    return rc
