"""Python mirror of the modem.js function surface, backed by libamodem (HIP, gfx950).

Names follow the reference (modem.js) in snake_case; semantics, argument meaning
and error behaviour are the reference's:

  set_ofdm_config(name)                     setOFDMConfig        modem.js:95-98
  decode_received_signal(sig, mod, rep)     decodeReceivedSignal modem.js:557-654
  decode_chunk_frame(frame, mod, rep)       decodeChunkFrame     modem.js:770-803
  estimate_frame_samples(nbytes, mod, rep)  estimateFrameSamples modem.js:863-874
  build_transmit_signal / build_metadata_frame / build_data_chunk_frame /
  generate_test_signal / generate_preamble_symbol1 / crc32
Signal-level failures come back as {'error': <exact reference string>} dicts;
device failures raise RuntimeError. Results are plain dicts with bytes for data.
"""
from __future__ import annotations

import ctypes as C
import threading
import weakref

import numpy as np

from . import _lib as L

OFDM_CONFIGS = {
    "standard": dict(FFT_SIZE=512, CP_LEN=64, SYMBOL_LEN=576, SAMPLE_RATE=44100, SUB_START=12, SUB_END=232,
                     PILOTS=[15, 29, 43, 57, 71, 85, 99, 113, 127, 141, 155, 169, 183, 197, 211, 225]),
    "acoustic": dict(FFT_SIZE=512, CP_LEN=128, SYMBOL_LEN=640, SAMPLE_RATE=44100, SUB_START=23, SUB_END=93,
                     PILOTS=[25, 35, 45, 55, 65, 75, 85]),
    "narrowband": dict(FFT_SIZE=512, CP_LEN=256, SYMBOL_LEN=768, SAMPLE_RATE=44100, SUB_START=35, SUB_END=58,
                       PILOTS=[37, 45, 53]),
}
OFDM = dict(OFDM_CONFIGS["standard"])  # mutable current config, like the reference global
FRAME_META = 0xFE
FRAME_DATA = 0xFF

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

RESULT_DTYPE = np.dtype([(n, "<i4") for n in ("status", "preamble_idx", "coarse_idx", "frame_type", "aux", "nbytes",
                                              "name_off", "name_len", "data_off", "data_len", "seq_num",
                                              "total_chunks", "total_size", "chunk_size")] +
                        [("expected_crc", "<u4"), ("actual_crc", "<u4"), ("crc_valid", "<i4"), ("nbits", "<i4"),
                         ("flags", "<i4"), ("fine_metric", "<f4"), ("payload_valid", "<i4"), ("reserved", "<i4", (3,))])
assert RESULT_DTYPE.itemsize == 96


def set_ofdm_config(name: str):
    """setOFDMConfig: unknown names fall back to 'standard' (modem.js:96)."""
    OFDM.clear()
    OFDM.update(OFDM_CONFIGS.get(name, OFDM_CONFIGS["standard"]))


def _mod_id(mod: str) -> int:
    if mod not in L.MODS:  # initConstellation on an unknown name throws (modem.js:108-109)
        raise TypeError(f"Cannot read property 'points' of undefined (modulation {mod!r})")
    return L.MODS[mod]


def make_cfg(mod: str = "QPSK", rep: int = 1, ofdm: dict | None = None) -> L.Cfg:
    o = OFDM if ofdm is None else ofdm
    c = L.Cfg()
    c.fft_size, c.cp_len, c.symbol_len = o["FFT_SIZE"], o["CP_LEN"], o["SYMBOL_LEN"]
    c.sample_rate, c.sub_start, c.sub_end = o["SAMPLE_RATE"], o["SUB_START"], o["SUB_END"]
    c.npilots = len(o["PILOTS"])
    for i, p in enumerate(o["PILOTS"]):
        c.pilots[i] = p
    c.modulation = _mod_id(mod)
    c.repetition = max(1, int(rep or 1))
    return c


def preset(name: str, mod: str = "QPSK", rep: int = 1) -> L.Cfg:
    c = L.Cfg()
    L.check(L.load().amod_config_preset(name.encode(), _mod_id(mod), int(rep or 1), C.byref(c)))
    return c


def text_decode(b: bytes) -> str:
    """TextDecoder().decode: UTF-8 with replacement characters, leading BOM removed."""
    if b[:3] == b"\xef\xbb\xbf":
        b = b[3:]
    return b.decode("utf-8", errors="replace")


def to_reference(rec, slot: bytes, via_legacy: bool) -> dict:
    """Format one amod_result the way modem.js returns it."""
    st, ft = int(rec["status"]), int(rec["frame_type"])
    if st == L.E_CAPACITY:
        raise RuntimeError("frame exceeds the reserved decode workspace (amod_reserve)")
    if st == 0:
        if ft == FRAME_META:
            out = {"frameType": FRAME_META, "totalChunks": int(rec["total_chunks"]),
                   "totalFileSize": int(rec["total_size"]), "chunkSize": int(rec["chunk_size"]),
                   "fileName": text_decode(slot[rec["name_off"]:rec["name_off"] + rec["name_len"]])}
        elif ft == FRAME_DATA:
            out = {"frameType": FRAME_DATA, "seqNum": int(rec["seq_num"]),
                   "data": bytes(slot[rec["data_off"]:rec["data_off"] + rec["data_len"]]),
                   "dataLen": int(rec["data_len"])}
        else:
            out = {"data": bytes(slot[rec["data_off"]:rec["data_off"] + rec["data_len"]]),
                   "dataLen": int(rec["data_len"]),
                   "fileName": text_decode(slot[rec["name_off"]:rec["name_off"] + rec["name_len"]])}
        out.update(crcValid=bool(rec["crc_valid"]), expectedCRC=int(rec["expected_crc"]),
                   actualCRC=int(rec["actual_crc"]))
        if ft == 0:
            out.update(preambleIdx=int(rec["preamble_idx"]), frameType="legacy")
        elif via_legacy:
            out["preambleIdx"] = int(rec["preamble_idx"])
        return out
    if st == 7:
        return {"error": f"Invalid data length: {int(rec['aux'])}"}
    if st == 13:
        return {"error": f"Unknown frame type: 0x{int(rec['aux']):x}", "frameType": int(rec["aux"])}
    out = {"error": ERRORS[st]}
    if via_legacy and ft in (FRAME_META, FRAME_DATA) and st in (8, 9, 10, 11):
        out["preambleIdx"] = int(rec["preamble_idx"])
    return out


STREAM_FRAME_DTYPE = np.dtype([("pos", np.int64), ("end", np.int64), ("window_len", np.int32),
                               ("reserved", np.int32), ("result", RESULT_DTYPE)])
assert STREAM_FRAME_DTYPE.itemsize == C.sizeof(L.StreamFrame)


class Demodulator:
    """One HIP device context (stream + workspace) of libamodem."""

    def __init__(self, device: int = 0):
        self._L = L.load()
        h = C.c_void_p()
        L.check(self._L.amod_open(int(device), C.byref(h)))
        self.ctx = h
        self.device = device
        self._lock = threading.Lock()

    def close(self):
        if self.ctx:
            # a Pipeline over this context finishes its decodes and closes first (its slot
            # streams may still run kernels on this context's workspace)
            for p in list(getattr(self, "_pipes", ())):
                p.close()
            self._L.amod_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- host path
    def decode_batch(self, samples: np.ndarray, offsets, lengths, mod="QPSK", rep=1, mode=L.MODE_RECEIVED,
                     cfg: L.Cfg | None = None, options: int = 0, stride: int | None = None, progress=None):
        """Decode frames samples[off:off+len] (host memory, PCIe round trip).
        Returns (records: RESULT_DTYPE array, payload: uint8 [nframes, stride]).
        progress(done, records, payload): called (from the library's helper thread, one
        call at a time, all before this returns) whenever frames [0, done) are final in the
        returned arrays (amod_decode_host_progress), while later frames are still
        uploading and decoding. The first exception progress raises is re-raised here once
        the decode has finished (later calls are skipped); progress must not call back into
        this Demodulator (its lock is held for the whole decode)."""
        samples = np.ascontiguousarray(samples, np.float32)
        offsets = np.ascontiguousarray(offsets, np.int64)
        lengths = np.ascontiguousarray(lengths, np.int32)
        cfg = cfg or make_cfg(mod, rep)
        n = len(offsets)
        need = int(self._L.amod_payload_stride(C.byref(cfg), int(lengths.max()) if n else 0))
        if stride is None:
            stride = need
        elif stride < need or stride % 16:
            raise ValueError(f"payload stride {stride} < {need} or not a multiple of 16")
        rec = np.zeros(n, RESULT_DTYPE)
        pay = np.zeros((n, stride), np.uint8)
        with self._lock:
            if progress is None:
                L.check(self._L.amod_decode_host(self.ctx, C.byref(cfg), mode,
                                                 samples.ctypes.data if samples.size else None, samples.size,
                                                 offsets.ctypes.data, lengths.ctypes.data, n, rec.ctypes.data,
                                                 pay.ctypes.data, stride, options), self.ctx)
            else:
                failed = []

                def call(_user, done):  # (an exception would be printed and lost by ctypes)
                    if failed:
                        return
                    try:
                        progress(int(done), rec, pay)
                    except BaseException as e:  # noqa: B902 (re-raised below)
                        failed.append(e)

                fn = L.PROGRESS_FN(call)
                L.check(self._L.amod_decode_host_progress(
                    self.ctx, C.byref(cfg), mode, samples.ctypes.data if samples.size else None, samples.size,
                    offsets.ctypes.data, lengths.ctypes.data, n, rec.ctypes.data, pay.ctypes.data, stride, options,
                    fn, None), self.ctx)
                if failed:
                    raise failed[0]
        return rec, pay

    def decode_received_signal(self, signal, mod="QPSK", rep=1, options=0) -> dict:
        sig = np.ascontiguousarray(signal, np.float32)
        rec, pay = self.decode_batch(sig, [0], [len(sig)], mod, rep or 1, L.MODE_RECEIVED, options=options)
        return to_reference(rec[0], pay[0].tobytes(), via_legacy=True)

    def decode_chunk_frame(self, frame, mod="QPSK", rep=1, options=0) -> dict:
        fr = np.ascontiguousarray(frame, np.float32)
        rec, pay = self.decode_batch(fr, [0], [len(fr)], mod, rep or 1, L.MODE_CHUNK, options=options)
        return to_reference(rec[0], pay[0].tobytes(), via_legacy=False)

    # -------------------------------------------------------------- device path
    def reserve(self, cfg: L.Cfg, nframes: int, max_len: int):
        L.check(self._L.amod_reserve(self.ctx, C.byref(cfg), int(nframes), int(max_len)), self.ctx)

    def decode_device(self, cfg: L.Cfg, mode: int, samples_ptr: int, offsets_ptr: int, lengths_ptr: int,
                      nframes: int, results_ptr: int, payload_ptr: int, stride: int, stream: int = 0,
                      options: int = 0, debug_ptr: int = 0):
        """Enqueue a decode of device-resident frames (raw device pointers, e.g.
        torch tensor .data_ptr()) on `stream` (hipStream_t as int, 0 = own)."""
        if debug_ptr:
            rc = self._L.amod_decode_device_debug(self.ctx, C.byref(cfg), mode, samples_ptr, offsets_ptr,
                                                  lengths_ptr, nframes, results_ptr, payload_ptr, stride, options,
                                                  stream or None, debug_ptr)
        else:
            rc = self._L.amod_decode_device(self.ctx, C.byref(cfg), mode, samples_ptr, offsets_ptr, lengths_ptr,
                                            nframes, results_ptr, payload_ptr, stride, options, stream or None)
        L.check(rc, self.ctx)

    def synchronize(self):
        L.check(self._L.amod_synchronize(self.ctx), self.ctx)

    def pipeline(self, other: "Demodulator") -> "Pipeline":
        """A depth-2 pipeline of device decodes over this context and `other` (amod_pipe_*)."""
        return Pipeline(self, other)

    # ------------------------------------------------------------ streaming
    def stream_receive(self, cfg: L.Cfg, samples: np.ndarray, assembler: "ChunkAssembler | None" = None,
                       max_frames: int = 1 << 20):
        """app.js StreamingReceiver over a recorded stream (4096-sample blocks): returns
        (frames: STREAM_FRAME_DTYPE records, refine_fail: list of positions, stats: dict).
        Decoded chunks go to `assembler` (a private one if None)."""
        x = np.ascontiguousarray(samples, np.float32)
        frames = np.zeros(max_frames, STREAM_FRAME_DTYPE)
        rf = np.zeros(1 << 16, np.int64)
        n = C.c_int64()
        st = L.StreamStats()
        with self._lock:
            L.check(self._L.amod_stream_receive(self.ctx, C.byref(cfg), x.ctypes.data, len(x),
                                                assembler._h if assembler is not None else None, frames.ctypes.data,
                                                max_frames, C.byref(n), rf.ctypes.data, len(rf), C.byref(st)), self.ctx)
        stats = {k: getattr(st, k) for k, _ in L.StreamStats._fields_}
        return frames[:min(n.value, max_frames)], rf[:min(st.nrefine_fail, len(rf))].tolist(), stats

    def stream_receive_device(self, cfg: L.Cfg, samples_ptr: int, n: int, assembler: "ChunkAssembler | None" = None,
                              max_frames: int = 1 << 20):
        """stream_receive over n samples already in device memory (samples_ptr)."""
        frames = np.zeros(max_frames, STREAM_FRAME_DTYPE)
        rf = np.zeros(1 << 16, np.int64)
        cnt = C.c_int64()
        st = L.StreamStats()
        with self._lock:
            L.check(self._L.amod_stream_receive_device(self.ctx, C.byref(cfg), samples_ptr, n,
                                                       assembler._h if assembler is not None else None,
                                                       frames.ctypes.data, max_frames, C.byref(cnt), rf.ctypes.data,
                                                       len(rf), C.byref(st)), self.ctx)
        stats = {k: getattr(st, k) for k, _ in L.StreamStats._fields_}
        return frames[:min(cnt.value, max_frames)], rf[:min(st.nrefine_fail, len(rf))].tolist(), stats

    def stream_shard(self, cfg: L.Cfg, samples: np.ndarray, lo: int, hi: int, own_lo: int, own_hi: int,
                     start: "L.StreamState | None" = None, meta_received: bool = False, chunk_size: int = 0,
                     until_meta: bool = False, stride: int = 0, max_events: int | None = None):
        """One shard of a sharded stream receive (amod_stream_shard): samples = stream
        samples [lo, hi). Returns (events: list of (StreamEvent copy), payload uint8
        [n, stride], fails: list of (block, pos), ema: (state before own_lo, state at
        own_hi - 1), end: StreamState)."""
        x = np.ascontiguousarray(samples, np.float32)
        assert len(x) == hi - lo
        if not stride:  # rows wide enough for the longest window this shard can cut
            win = int(self._L.amod_estimate_frame_samples(C.byref(cfg), (chunk_size or 4096) + 11))
            stride = payload_stride(cfg, max(win, int(self._L.amod_estimate_frame_samples(C.byref(cfg), 4107))))
        # the receiver demodulates at most one window and fails at most one refinement per
        # 4096-sample block (app.js:749-773), so these bounds never truncate
        nblk = (hi - lo) // 4096 + 1
        max_events = nblk if max_events is None else max_events
        ev = (L.StreamEvent * max(max_events, 1))()
        pay = np.zeros((max(max_events, 1), stride), np.uint8)
        nev, nf = C.c_int64(), C.c_int64()
        max_fails = nblk
        fails = np.zeros(2 * max_fails, np.int64)
        ema = np.zeros(2, np.float64)
        end = L.StreamState()
        with self._lock:
            L.check(self._L.amod_stream_shard(self.ctx, C.byref(cfg), x.ctypes.data, lo, hi, own_lo, own_hi,
                                              C.byref(start) if start is not None else None, int(meta_received),
                                              int(chunk_size), int(until_meta), ev, max_events, C.byref(nev),
                                              pay.ctypes.data, stride, fails.ctypes.data, max_fails, C.byref(nf),
                                              ema.ctypes.data, C.byref(end)), self.ctx)
        if nev.value > max_events or nf.value > max_fails:
            raise RuntimeError(f"stream_shard: {nev.value} windows / {nf.value} failed refinements exceed the "
                               f"buffers ({max_events} / {max_fails})")
        n = nev.value
        events = [L.StreamEvent.from_buffer_copy(ev[i]) for i in range(n)]
        fl = [(int(fails[2 * i]), int(fails[2 * i + 1])) for i in range(nf.value)]
        return events, pay[:n], fl, (float(ema[0]), float(ema[1])), end

    # ------------------------------------------------------------ transmitter
    def transmit_device(self, cfg: L.Cfg, packets_ptr: int, pkt_off_ptr: int, pkt_len_ptr: int, pre_ptr: int,
                        post_ptr: int, nframes: int, out_ptr: int, out_off_ptr: int, stream: int = 0):
        """Enqueue k_tx (GPU modulateOFDM + frame builder) over device-resident packets."""
        L.check(self._L.amod_tx_device(self.ctx, C.byref(cfg), packets_ptr, pkt_off_ptr, pkt_len_ptr, pre_ptr,
                                       post_ptr, int(nframes), out_ptr, out_off_ptr, stream or None), self.ctx)

    def transmit_batch(self, cfg: L.Cfg, packets, kinds):
        """Frames of the given packets (bytes) and builder kinds (TX_LEGACY / TX_META /
        TX_CHUNK, one per packet or one for all) through the GPU transmitter.
        Returns (samples float32, offsets int64, lengths int32), frames back to back."""
        packets = [bytes(p) for p in packets]
        n = len(packets)
        kinds = [kinds] * n if isinstance(kinds, int) else list(kinds)
        plen = np.array([len(p) for p in packets], np.int32)
        poff = np.concatenate([[0], np.cumsum(plen)[:-1]]).astype(np.int64) if n else np.zeros(0, np.int64)
        buf = np.frombuffer(b"".join(packets) or b"\0", np.uint8).copy()
        pre = np.zeros(n, np.int32)
        post = np.zeros(n, np.int32)
        for i, k in enumerate(kinds):
            pre[i], post[i] = tx_silence(cfg, k)
        args = (self.ctx, C.byref(cfg), buf.ctypes.data, int(plen.sum()), poff.ctypes.data, plen.ctypes.data,
                pre.ctypes.data, post.ctypes.data, n)
        with self._lock:
            total = self._L.amod_tx_host(*args, None, None)
            if total < 0:
                raise RuntimeError(f"libamodem error {total}: {L.last_error(self.ctx)}")
            out = np.zeros(max(int(total), 1), np.float32)
            offs = np.zeros(n, np.int64)
            L.check(0 if self._L.amod_tx_host(*args, out.ctypes.data, offs.ctypes.data) == total else -1, self.ctx)
        lens = np.diff(np.append(offs, total)).astype(np.int32)
        return out[:total], offs, lens


class Pipeline:
    """amod_pipe_*: consecutive device decodes alternate between two Demodulators, on the
    pipe's two streams, so batch i + 1's detection overlaps batch i's demodulation.
    Fastest: enqueue a batch's inputs on next_stream(), decode with stream=0, and read its
    results on that stream (e.g. torch.cuda.ExternalStream(next_stream())). With another
    `stream`, decode i's results are ordered on it once decode i + 1 is enqueued, or after
    flush(stream). synchronize() waits on the host. The Demodulators stay the caller's."""

    def next_stream(self) -> int:
        """the hipStream_t (int) the next decode runs on"""
        return int(self._L.amod_pipe_next_stream(self._h) or 0)

    def __init__(self, a: Demodulator, b: Demodulator):
        self._L = a._L
        self._dms = (a, b) # (kept alive while the pipe uses their contexts)
        self._h = None
        h = C.c_void_p()
        L.check(self._L.amod_pipe_open(a.ctx, b.ctx, C.byref(h)), a.ctx)
        self._h = h
        for dm in (a, b):
            if not hasattr(dm, "_pipes"):
                dm._pipes = weakref.WeakSet()
            dm._pipes.add(self)

    def decode_device(self, cfg: L.Cfg, mode: int, samples_ptr: int, offsets_ptr: int, lengths_ptr: int,
                      nframes: int, results_ptr: int, payload_ptr: int, stride: int, stream: int = 0,
                      options: int = 0):
        L.check(self._L.amod_pipe_decode_device(self._h, C.byref(cfg), mode, samples_ptr, offsets_ptr, lengths_ptr,
                                                nframes, results_ptr, payload_ptr, stride, options, stream or None),
                self._dms[0].ctx)

    def flush(self, stream: int = 0):
        L.check(self._L.amod_pipe_flush(self._h, stream or None), self._dms[0].ctx)

    def synchronize(self):
        L.check(self._L.amod_pipe_synchronize(self._h), self._dms[0].ctx)

    def close(self):
        if self._h:
            self._L.amod_pipe_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------ host utilities --
def crc32(data: bytes) -> int:
    data = bytes(data)
    return int(L.load().amod_crc32(data, len(data)))


def num_data_subs(cfg: L.Cfg) -> int:
    """numDataSubs (modem.js:89-93): in-band subcarriers that are not pilots."""
    return int(L.load().amod_num_data_subs(C.byref(cfg)))


def payload_stride(cfg: L.Cfg, max_len: int) -> int:
    return int(L.load().amod_payload_stride(C.byref(cfg), int(max_len)))


def estimate_frame_samples(payload_bytes: int, mod: str = "QPSK", rep: int = 1) -> int:
    cfg = make_cfg(mod, rep)
    return int(L.load().amod_estimate_frame_samples(C.byref(cfg), int(payload_bytes)))


def generate_preamble_symbol1(cfg: L.Cfg | None = None) -> np.ndarray:
    cfg = cfg or make_cfg()
    out = np.zeros(cfg.symbol_len, np.float32)
    L.check(L.load().amod_preamble1(C.byref(cfg), out.ctypes.data))
    return out


def _tx(fn, *args) -> np.ndarray:
    n = fn(*args, None)
    if n < 0:
        raise ValueError("invalid transmit arguments")
    out = np.zeros(max(int(n), 1), np.float32)
    fn(*args, out.ctypes.data)
    return out[:n]


def build_transmit_signal(data: bytes, mod="QPSK", file_name="file", rep=1, cfg=None) -> np.ndarray:
    cfg = cfg or make_cfg(mod, rep)
    data = bytes(data)
    name = (file_name or "file").encode("utf-8")
    return _tx(L.load().amod_tx_legacy, C.byref(cfg), data, len(data), name, len(name))


def build_metadata_frame(total_chunks, total_size, chunk_size, file_name, mod="QPSK", rep=1, cfg=None):
    cfg = cfg or make_cfg(mod, rep)
    name = (file_name or "file").encode("utf-8")
    return _tx(L.load().amod_tx_meta, C.byref(cfg), int(total_chunks), int(total_size), int(chunk_size), name,
               len(name))


def build_data_chunk_frame(data: bytes, seq: int, mod="QPSK", rep=1, cfg=None):
    cfg = cfg or make_cfg(mod, rep)
    data = bytes(data)
    return _tx(L.load().amod_tx_chunk, C.byref(cfg), data, len(data), int(seq))


def generate_test_signal(mod="QPSK", rep=1, cfg=None):
    cfg = cfg or make_cfg(mod, rep)
    return _tx(L.load().amod_tx_test_signal, C.byref(cfg)), bytes(range(16))


def _packet(fn, *args) -> bytes:
    n = fn(*args, None)
    if n < 0:
        raise ValueError("invalid packet arguments")
    out = np.zeros(max(int(n), 1), np.uint8)
    fn(*args, out.ctypes.data)
    return out[:n].tobytes()


def packet_legacy(data: bytes, file_name="file") -> bytes:
    """buildTransmitSignal's packet [nameLen][name][dataLen:4][data][CRC:4] (modem.js:500-521)."""
    data = bytes(data)
    name = (file_name or "file").encode("utf-8")
    return _packet(L.load().amod_packet_legacy, data, len(data), name, len(name))


def packet_meta(total_chunks: int, total_size: int, chunk_size: int, file_name="file") -> bytes:
    """buildMetadataPayload (modem.js:666-692)."""
    name = (file_name or "file").encode("utf-8")
    return _packet(L.load().amod_packet_meta, int(total_chunks), int(total_size), int(chunk_size), name, len(name))


def packet_chunk(data: bytes, seq: int) -> bytes:
    """buildDataChunkPayload (modem.js:694-714)."""
    data = bytes(data)
    return _packet(L.load().amod_packet_chunk, data, len(data), int(seq))


def tx_silence(cfg: L.Cfg, kind: int):
    pre, post = C.c_int32(), C.c_int32()
    L.check(L.load().amod_tx_silence(C.byref(cfg), int(kind), C.byref(pre), C.byref(post)))
    return pre.value, post.value


def synth_legacy_packets(nframes: int, payload_len: int = 1024, name: str = "f.bin", first: int = 0):
    """Packets of the synthetic legacy workload (payload seed 0x9E3779B9 ^ frame index),
    back to back: (bytes uint8, offsets int64, lengths int32)."""
    lib = L.load()
    nm = name.encode()
    total = lib.amod_synth_legacy_packets(nframes, first, payload_len, nm, len(nm), None, None, None)
    buf = np.zeros(max(int(total), 1), np.uint8)
    offs = np.zeros(nframes, np.int64)
    lens = np.zeros(nframes, np.int32)
    lib.amod_synth_legacy_packets(nframes, first, payload_len, nm, len(nm), buf.ctypes.data, offs.ctypes.data,
                                  lens.ctypes.data)
    return buf, offs, lens


def synth_payload(seed: int, length: int) -> bytes:
    out = np.zeros(max(length, 1), np.uint8)
    L.load().amod_synth_payload(seed & 0xFFFFFFFF, int(length), out.ctypes.data)
    return out[:length].tobytes()


def synth_legacy_batch(cfg: L.Cfg, nframes: int, payload_len: int = 1024, name: str = "f.bin", first: int = 0,
                       threads: int = 0, out: np.ndarray | None = None):
    """nframes legacy frames back to back (payload seed 0x9E3779B9 ^ frame index)."""
    lib = L.load()
    nm = name.encode()
    total = lib.amod_synth_legacy_batch(C.byref(cfg), nframes, first, payload_len, nm, len(nm), None, None, None, 0)
    if out is None:
        out = np.empty(int(total), np.float32)
    offs = np.zeros(nframes, np.int64)
    lens = np.zeros(nframes, np.int32)
    lib.amod_synth_legacy_batch(C.byref(cfg), nframes, first, payload_len, nm, len(nm), out.ctypes.data,
                                offs.ctypes.data, lens.ctypes.data, threads)
    return out, offs, lens


# ---------------------------------------------------------------- assembly --
class AssemblerError(Exception):
    """An error the reference's ChunkAssembler throws (name: 'RangeError' / 'TypeError')."""

    def __init__(self, name: str):
        super().__init__(name)
        self.name = name


def _asm_check(rc):
    if rc == L.ASM_RANGE_ERROR:
        raise AssemblerError("RangeError")
    if rc == L.ASM_TYPE_ERROR:
        raise AssemblerError("TypeError")
    if rc < 0:
        raise RuntimeError(f"libamodem assembler error {rc}")
    return rc


class DeviceGroup:
    """Several GPUs from one process (amod_group_*): decode_batch cuts a batch into
    contiguous frame ranges of about equal sample counts, one per device, decoded at once;
    results come back in frame order. devices may repeat (two contexts on one GPU)."""

    def __init__(self, devices):
        self._L = L.load()
        ids = np.ascontiguousarray(devices, np.int32)
        h = C.c_void_p()
        L.check(self._L.amod_group_open(ids.ctypes.data, len(ids), C.byref(h)))
        self._h = h
        self.devices = [int(d) for d in ids]

    def decode_batch(self, samples, offsets, lengths, cfg: L.Cfg, mode: int = L.MODE_RECEIVED, options: int = 0):
        """-> (RESULT_DTYPE records, payload uint8 [n, stride], frames per device)."""
        x = np.ascontiguousarray(samples, np.float32)
        off = np.ascontiguousarray(offsets, np.int64)
        ln = np.ascontiguousarray(lengths, np.int32)
        n = len(off)
        stride = payload_stride(cfg, int(ln.max()) if n else 1)
        rec = np.zeros(n, RESULT_DTYPE)
        pay = np.zeros((n, stride), np.uint8)
        split = np.zeros(len(self.devices), np.int32)
        L.check(self._L.amod_group_decode_host(self._h, C.byref(cfg), mode, x.ctypes.data, len(x), off.ctypes.data,
                                               ln.ctypes.data, n, rec.ctypes.data, pay.ctypes.data, stride, options,
                                               split.ctypes.data))
        return rec, pay, split.tolist()

    def decode_device(self, cfg: L.Cfg, mode: int, shards, options: int = 0):
        """Enqueue every member's decode of its device-resident shard (amod_group_decode_device).
        shards: one dict per member with device pointers samples / offsets / lengths /
        results / payload (ints, e.g. torch .data_ptr()), nframes, payload_stride and an
        optional stream (hipStream_t as int, 0 = the member context's). Returns without
        synchronising (synchronize())."""
        arr = (L.Shard * len(self.devices))()
        for k, sh in enumerate(shards):
            arr[k] = L.Shard(sh.get("samples", 0), sh.get("offsets", 0), sh.get("lengths", 0), sh.get("results", 0),
                             sh.get("payload", 0), int(sh.get("payload_stride", 16)), sh.get("stream", 0) or None,
                             int(sh.get("nframes", 0)), 0)
        L.check(self._L.amod_group_decode_device(self._h, C.byref(cfg), mode, arr, options))

    def synchronize(self):
        L.check(self._L.amod_group_synchronize(self._h))

    def upload(self, samples, offsets, lengths, cfg: L.Cfg) -> "ResidentBatch":
        """Make a host batch resident across the group once (amod_group_upload); decode it
        from HBM as often as needed with ResidentBatch.decode."""
        return ResidentBatch(self, samples, offsets, lengths, cfg)

    def close(self):
        if self._h:
            self._L.amod_group_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResidentBatch:
    """A host batch resident across a DeviceGroup (amod_group_upload: contiguous frame
    ranges of about equal sample counts, one per member); decode() runs every member's
    device-path decode at once and returns records and payload rows in frame order."""

    def __init__(self, group: DeviceGroup, samples, offsets, lengths, cfg: L.Cfg):
        self._L = group._L
        self._group = group  # (the group must outlive its resident batches)
        x = np.ascontiguousarray(samples, np.float32)
        off = np.ascontiguousarray(offsets, np.int64)
        ln = np.ascontiguousarray(lengths, np.int32)
        self.n = len(off)
        self.max_len = int(ln.max()) if self.n else 1
        h = C.c_void_p()
        L.check(self._L.amod_group_upload(group._h, C.byref(cfg), x.ctypes.data, len(x), off.ctypes.data,
                                          ln.ctypes.data, self.n, C.byref(h)))
        self._h = h

    def frames_per_device(self):
        out = np.zeros(len(self._group.devices), np.int32)
        self._L.amod_resident_frames(self._h, out.ctypes.data)
        return out.tolist()

    def decode(self, cfg: L.Cfg, mode: int = L.MODE_RECEIVED, options: int = 0):
        """-> (RESULT_DTYPE records, payload uint8 [n, stride])."""
        stride = payload_stride(cfg, self.max_len)
        rec = np.zeros(self.n, RESULT_DTYPE)
        pay = np.zeros((self.n, stride), np.uint8)
        L.check(self._L.amod_resident_decode(self._h, C.byref(cfg), mode, options, rec.ctypes.data, pay.ctypes.data,
                                             stride))
        return rec, pay

    def close(self):
        if self._h:
            self._L.amod_resident_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StreamingReceiver:
    """app.js StreamingReceiver (706-998) driven live, one audio block per call
    (processAudioBlock, 749-773): DC removal, ring buffer and one state-machine step on
    the host, windows decoded on the GPU (decodeChunkFrame) and handed to the assembler.
    process_audio_block returns the demodulated window's STREAM_FRAME_DTYPE record, or
    None. Fed a recorded stream's blocks, the frames equal Demodulator.stream_receive's."""

    def __init__(self, demodulator: "Demodulator", cfg: L.Cfg, assembler: "ChunkAssembler | None" = None):
        self._L = L.load()
        self._dm = demodulator
        self.cfg = cfg
        self.assembler = assembler if assembler is not None else ChunkAssembler()
        h = C.c_void_p()
        L.check(self._L.amod_live_open(demodulator.ctx, C.byref(cfg), self.assembler._h, C.byref(h)), demodulator.ctx)
        self._h = h

    def process_audio_block(self, samples) -> "np.ndarray | None":
        x = np.ascontiguousarray(samples, np.float32)
        rec = np.zeros(1, STREAM_FRAME_DTYPE)
        has = C.c_int32()
        with self._dm._lock:
            L.check(self._L.amod_live_process_block(self._h, x.ctypes.data, len(x), rec.ctypes.data, C.byref(has)),
                    self._dm.ctx)
        return rec[0] if has.value else None

    def state(self) -> dict:
        st, ls = L.StreamState(), L.LiveStats()
        L.check(self._L.amod_live_state(self._h, C.byref(st), C.byref(ls)))
        out = {k: getattr(st, k) for k, _ in L.StreamState._fields_}
        out.update({k: getattr(ls, k) for k, _ in L.LiveStats._fields_})
        return out

    def refine_fails(self) -> list:
        n = self._L.amod_live_refine_fails(self._h, None, 0)
        buf = np.zeros(max(n, 1), np.int64)
        self._L.amod_live_refine_fails(self._h, buf.ctypes.data, n)
        return buf[:n].tolist()

    def close(self):
        if self._h:
            self._L.amod_live_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ChunkAssembler:
    """app.js ChunkAssembler (597-704) over libamodem's host assembler: same method
    names (snake_case), same state and the same thrown errors. directory: keep the
    chunks as files there (the IndexedDB store's stand-in) instead of in memory."""

    def __init__(self, directory: str | None = None):
        self._L = L.load()
        h = C.c_void_p()
        _asm_check(self._L.amod_asm_open(directory.encode() if directory else None, C.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            self._L.amod_asm_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def handle_metadata_frame(self, total_chunks: int, total_file_size: int, chunk_size: int, file_name: bytes):
        name = bytes(file_name)
        _asm_check(self._L.amod_asm_metadata(self._h, int(total_chunks), int(total_file_size), int(chunk_size), name,
                                             len(name)))

    def handle_data_chunk(self, seq_num: int, data: bytes, crc_valid: bool) -> bool:
        data = bytes(data)
        return _asm_check(self._L.amod_asm_chunk(self._h, int(seq_num), data, len(data), int(bool(crc_valid)))) == 1

    def feed(self, records: np.ndarray, payload: np.ndarray):
        """StreamingReceiver's dispatch over decodeChunkFrame results (RESULT_DTYPE
        records + [n, stride] payload slots), in order."""
        records = np.ascontiguousarray(records)
        payload = np.ascontiguousarray(payload, np.uint8)
        _asm_check(self._L.amod_asm_feed(self._h, records.ctypes.data, payload.ctypes.data, payload.shape[1],
                                         len(records)))

    def state(self) -> dict:
        s = L.AsmState()
        _asm_check(self._L.amod_asm_state(self._h, C.byref(s)))
        return {n: getattr(s, n) for n, _ in L.AsmState._fields_ if n != "reserved"}

    def bitmap(self):
        n = self._L.amod_asm_bitmap(self._h, None, 0)
        out = np.zeros(max(n, 1), np.uint8)
        self._L.amod_asm_bitmap(self._h, out.ctypes.data, n)
        return out[:n]

    def file_name(self) -> bytes:
        n = self._L.amod_asm_name(self._h, None, 0)
        out = np.zeros(max(n, 1), np.uint8)
        self._L.amod_asm_name(self._h, out.ctypes.data, n)
        return out[:n].tobytes()

    def is_complete(self) -> bool:
        return bool(self.state()["complete"])

    def is_received(self, seq: int) -> bool:
        b = self.bitmap()
        return 0 <= seq and (seq >> 3) < len(b) and bool(b[seq >> 3] & (1 << (seq & 7)))

    def get_missing_chunks(self):
        n = self._L.amod_asm_missing(self._h, None, 0)
        out = np.zeros(max(n, 1), np.int32)
        self._L.amod_asm_missing(self._h, out.ctypes.data, n)
        return out[:n].tolist()

    def assemble_file(self) -> bytes:
        n = _asm_check(self._L.amod_asm_file(self._h, None, 0))
        out = np.zeros(max(n, 1), np.uint8)
        _asm_check(self._L.amod_asm_file(self._h, out.ctypes.data, n))
        return out[:n].tobytes()
