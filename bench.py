#!/usr/bin/env python3
"""bench.py — OFDM receive throughput on MI355X (BASELINE.json metric).

One step = one decodeReceivedSignal pass (preprocess, Schmidl-Cox scan, fine timing,
channel estimate, per-symbol FFT/equalise/demap, vote, pack, parse, CRC-32) over the
whole resident batch: BASELINE config C2, 10,000 QPSK frames of 35,874 samples (1 KB
payload) per GPU, synthesised on the GPU by the reference-equivalent transmitter.
Inputs are in HBM before the timed region. Frames are independent, so ranks shard them
(weak scaling, no data-path collective; one RCCL gather of the results afterwards).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--legs ...]

The default run (C2) also carries compact C4 (32k 2 KB chunk windows, decodeChunkFrame)
and C5 (acoustic BPSK rep3 at 10 dB) legs, each with its own roofline and a full-batch
agreement count against the C oracle, plus the streaming-receiver, PCIe, Node-host and
CPU-baseline legs.

--gpus N > 1 without a torch.distributed environment: bench.py starts
`python -m torch.distributed.run --nproc-per-node N` itself (before touching the GPU)
and exits with its status; fewer visible GPUs than N is an error (RCCL needs one device
per rank). AMOD_BENCH_BACKEND=gloo rehearses the N-rank flow with ranks sharing devices.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))
sys.path.insert(0, ROOT)

METRIC = "audio samples/s demodulated + payload MB/s, QPSK 512-FFT, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
SAMPLES_PER_FRAME = 35874     # C2: QPSK 1 KB legacy frame
SAMPLES_PER_FRAME_C3 = 30114  # C3: 16-QAM 1 KB legacy frame
PAYLOAD = 1024
PAYLOAD_C5 = 256
CHUNK = 2048                  # C4: data bytes per chunk frame


def host_threads():
    """(threads, where the number came from): the CPUs this process may run on
    (sched_getaffinity), capped by the cgroup CPU quota (cgroup v2 cpu.max, v1
    cfs_quota_us / cfs_period_us) and by OMP_NUM_THREADS, which the GPU box sets to its
    CPU share (os.cpu_count() shows the whole machine there)."""
    import math
    n = len(os.sched_getaffinity(0))
    src = [f"sched_getaffinity {n}"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        src.append(f"cgroup quota {quota:g}")
        n = min(n, max(1, math.ceil(quota)))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        src.append(f"OMP_NUM_THREADS {omp}")
        n = min(n, int(omp))
    return max(1, n), ", ".join(src)


HOST_THREADS, HOST_THREADS_SOURCE = host_threads()
FLAG_NAMES = {0: "FORCED", 1: "NONFINITE", 2: "BIG", 3: "COARSE", 4: "FINE", 5: "CHANNEL", 6: "PHASE", 7: "DEMAP",
              8: "THRESH", 9: "SPAN", 10: "SOFT", 11: "REPLAY"}


# ------------------------------------------------------------------ launcher --
def launch_plan(gpus: int, env: dict, ndev: int, backend: str):
    """What `bench.py --gpus N` does in this process: ("run", world) when it is a rank
    already (torch.distributed environment) or N == 1; ("spawn", N) to start N ranks;
    ("error", message) when RCCL cannot place N ranks on the visible devices."""
    if "WORLD_SIZE" in env:
        return ("run", int(env["WORLD_SIZE"]))
    if gpus <= 1:
        return ("run", 1)
    if backend != "gloo" and ndev < gpus:
        return ("error", f"--gpus {gpus}: only {ndev} GPU(s) visible; RCCL needs one device per rank "
                         f"(AMOD_BENCH_BACKEND=gloo rehearses {gpus} ranks on shared devices)")
    if backend == "gloo" and ndev < 1:
        return ("error", f"--gpus {gpus}: no GPU visible")
    return ("spawn", gpus)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd).returncode


# ---------------------------------------------------------------- helpers ----
T_START = time.perf_counter()


def progress(msg: str):
    """One line per phase on stderr (long runs show they are alive)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.perf_counter() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def warm_up(step, sync, min_steps, min_s=0.5, max_s=8.0, tol=0.02):
    """At least min_steps steps, then batches of ~50 ms until two consecutive batches'
    per-step times agree within tol and min_s has passed (GPU clocks ramp under load:
    the C2 chain falls from ~0.55 to ~0.46 ms over its first ~50 decodes)."""
    t_start = time.perf_counter()
    n = 0
    for _ in range(min_steps):
        step()
        n += 1
    sync()
    prev, k, dt = None, 4, 0.0
    while True:
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        sync()
        dt = (time.perf_counter() - t0) / k
        n += k
        el = time.perf_counter() - t_start
        if prev is not None and el >= min_s and abs(dt - prev) <= tol * prev:
            break
        if el >= max_s:
            break
        prev = dt
        k = max(4, min(2000, int(0.05 / max(dt, 1e-6))))
    return {"steps": n, "seconds": time.perf_counter() - t_start, "last_ms_per_step": dt * 1e3}


def flag_hist(rec):
    out = {}
    for fl in rec["flags"][rec["flags"] != 0]:
        for b in range(16):
            if int(fl) & (1 << b) and b != 15:
                out[FLAG_NAMES.get(b, str(b))] = out.get(FLAG_NAMES.get(b, str(b)), 0) + 1
    return out


class Env:
    """The rank's process-group and device context."""

    def __init__(self):
        import torch
        import torch.distributed as dist

        import amodem
        from amodem import _lib as L
        self.torch, self.dist, self.amodem, self.L = torch, dist, amodem, L
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # AMOD_BENCH_BACKEND=gloo rehearses the N > 1 flow with several ranks on one GPU
        # (RCCL refuses two ranks per device); the driver's runs use the default, RCCL
        self.backend = os.environ.get("AMOD_BENCH_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        if self.backend == "gloo":
            self.local = self.local % max(1, ndev)
        elif self.local >= ndev:
            raise SystemExit(f"rank {self.rank}: LOCAL_RANK {self.local} but only {ndev} GPU(s) visible")
        self.dev = torch.device("cuda", self.local)
        torch.cuda.set_device(self.dev)
        if self.world > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(self.backend)
        self.lib = L.load()
        self.devices_used = ndev if self.backend == "gloo" else self.world
        self.devices_used = min(self.devices_used, self.world)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, v: float) -> float:
        if self.world == 1:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, vals):
        if self.world == 1:
            return list(vals)
        t = self.torch.tensor(list(vals), dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return [float(v) for v in t.tolist()]


class Workload:
    """One config's synthetic batch on this rank's GPU (built by k_tx, the reference
    transmitter, bit-exact), device-resident, plus its decode step."""

    def __init__(self, env: Env, conf: str, frames: int = 0, snr: float = 20.0, rank=None, device=None):
        # (rank / device: another rank's shard on another device, for the group leg: rank 0
        # alone building every rank's batch)
        torch, amodem, L = env.torch, env.amodem, env.L
        self.env, self.conf, self.snr = env, conf, snr
        C3, C4, C5, C5C = conf == "c3", conf == "c4", conf == "c5", conf == "c5c"
        # c5c: C5's acoustic BPSK rep3 as 256 B data-chunk windows (decodeChunkFrame) in
        # heavy AWGN, where combining the repeats matters (soft_chunk_leg)
        self.chunk = C4 or C5C
        self.noisy = C5 or C5C
        self.cfg = amodem.preset("acoustic", "BPSK", 3) if (C5 or C5C) else \
            amodem.preset("standard", "QAM16" if C3 else "QPSK", 1)
        self.mod = "QAM16" if C3 else ("BPSK" if (C5 or C5C) else "QPSK")
        self.preset = "acoustic" if (C5 or C5C) else "standard"
        F = frames if frames > 0 else (100000 if C3 else (32000 if C4 else 10000))
        self.F = F
        rank = env.rank if rank is None else rank
        self.local = env.local if device is None else int(device)
        dev = env.dev if device is None else torch.device("cuda", self.local)
        self.dev = dev
        self.dm = amodem.Demodulator(self.local)
        if self.chunk:
            # the file's chunks this rank owns: chunk seq = rank * F + i, bytes from xorshift32
            cb = CHUNK if C4 else PAYLOAD_C5
            pre, post = amodem.tx_silence(self.cfg, L.TX_CHUNK)
            # the receiver's window (app.js:853: estimateFrameSamples(chunkSize + 11))
            self.win = int(env.lib.amod_estimate_frame_samples(C.byref(self.cfg), cb + 11))
            spf = pre + self.win + post
            pkts = [amodem.packet_chunk(amodem.synth_payload(0x9E3779B9 ^ (rank * F + i), cb), rank * F + i)
                    for i in range(F)]
            pl = np.array([len(p) for p in pkts], np.int32)
            po = np.concatenate([[0], np.cumsum(pl)[:-1]]).astype(np.int64)
            pk = np.frombuffer(b"".join(pkts), np.uint8).copy()
        else:
            plen = PAYLOAD_C5 if C5 else PAYLOAD
            pk, po, pl = amodem.synth_legacy_packets(F, plen, "f.bin", first=rank * F)
            pre, post = amodem.tx_silence(self.cfg, L.TX_LEGACY)
            spf = SAMPLES_PER_FRAME_C3 if C3 else (
                int(env.lib.amod_tx_frame_samples(C.byref(self.cfg), int(pl[0]), pre, post)) if C5
                else SAMPLES_PER_FRAME)
        self.spf, self.pre, self.pl = spf, pre, pl
        self.offs = np.arange(F, dtype=np.int64) * spf
        self.lens = np.full(F, spf, np.int32)
        self.nsamples = int(self.lens.sum())
        # what one step decodes: whole legacy frames, or the C4 windows (pre1 .. end of the
        # estimated frame, as StreamingReceiver cuts them) in decodeChunkFrame mode
        self.mode = L.MODE_CHUNK if self.chunk else L.MODE_RECEIVED
        self.doffs = self.offs + pre if self.chunk else self.offs
        self.dlens = np.full(F, self.win, np.int32) if self.chunk else self.lens
        self.ndecoded = int(self.dlens.sum())
        self.payload_bytes = CHUNK if C4 else (PAYLOAD_C5 if (C5 or C5C) else PAYLOAD)
        self.packets = (pk, po, pl) if C5C else None  # (the soft leg counts bit errors against them)
        self.xs = torch.empty(self.nsamples + 16, dtype=torch.float32, device=dev)
        d_pk = torch.from_numpy(pk).to(dev)
        d_po, d_pl = torch.from_numpy(po).to(dev), torch.from_numpy(pl).to(dev)
        d_pre = torch.full((F,), pre, dtype=torch.int32, device=dev)
        d_post = torch.full((F,), post, dtype=torch.int32, device=dev)
        d_off = torch.from_numpy(self.offs).to(dev)
        self.d_doff = torch.from_numpy(self.doffs).to(dev)
        self.d_dlen = torch.from_numpy(self.dlens).to(dev)
        self.stream = torch.cuda.current_stream(dev).cuda_stream
        tx_stream = torch.cuda.Stream(dev)  # a real (non-null) stream, so events and kernel share it

        def tx():
            self.dm.transmit_device(self.cfg, d_pk.data_ptr(), d_po.data_ptr(), d_pl.data_ptr(), d_pre.data_ptr(),
                                    d_post.data_ptr(), F, self.xs.data_ptr(), d_off.data_ptr(),
                                    stream=tx_stream.cuda_stream)

        torch.cuda.synchronize(dev)
        tx()
        tx_stream.synchronize()
        tx_ms = []
        for _ in range(3):  # k_tx timed with HIP events on its launch stream
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(tx_stream)
            tx()
            e1.record(tx_stream)
            e1.synchronize()
            tx_ms.append(e0.elapsed_time(e1))
        torch.cuda.synchronize(dev)
        self.tx_ms = sum(tx_ms) / len(tx_ms)
        self.tx_bytes = 4.0 * self.nsamples + float(pl.sum())  # samples written + packet bytes read
        self.sigma = None
        if self.noisy:  # AWGN on the GPU, seeded per rank; power from the first frame's active samples
            x0 = self.xs[: int(self.lens[0])]
            act = x0[x0 != 0]
            self.sigma = float(torch.sqrt((act.double() ** 2).mean() / 10 ** (snr / 10)).item())
            gen = torch.Generator(device=dev)
            gen.manual_seed((0xC5C if C5C else 0xC5) + rank)
            self.xs[: self.nsamples] += torch.randn(self.nsamples, generator=gen, device=dev,
                                                    dtype=torch.float32) * self.sigma
            torch.cuda.synchronize(dev)
        del d_pk, d_po, d_pl, d_pre, d_post, d_off
        self.stride = amodem.payload_stride(self.cfg, int(self.dlens.max()))
        self.d_res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
        self.d_pay = torch.zeros(F * self.stride, dtype=torch.uint8, device=dev)
        self.dm.reserve(self.cfg, F, int(self.dlens.max()))

    def step(self, options=0):
        self.dm.decode_device(self.cfg, self.mode, self.xs.data_ptr(), self.d_doff.data_ptr(), self.d_dlen.data_ptr(),
                              self.F, self.d_res.data_ptr(), self.d_pay.data_ptr(), self.stride, stream=self.stream,
                              options=options)

    def enable_pipeline(self):
        """Consecutive batches through the library's depth-2 pipe (amod_pipe_*, Python
        `Pipeline`) over two contexts, each decoding on its own stream: batch i + 1's
        k_detect runs while batch i's k_demod finishes, so the two kernels' tails and the
        dependent-launch gaps overlap (tools/pipeline_ab.py: C2 0.455 -> 0.425 ms per step,
        C5 1.60 -> 1.47; C4, one k_demod launch, no gain). Result buffers alternate, so
        batch i's rows are intact until batch i + 2."""
        torch, amodem = self.env.torch, self.env.amodem
        self.dm2 = amodem.Demodulator(self.local)
        self.dm2.reserve(self.cfg, self.F, int(self.dlens.max()))
        self.d_res2 = torch.zeros_like(self.d_res)
        self.d_pay2 = torch.zeros_like(self.d_pay)
        self.pipe = self.dm.pipeline(self.dm2)
        self.pi = 0

    def step_ctx(self, k, stream):
        """one decode on context k (0: dm, 1: dm2) into its own result buffers, on `stream`"""
        dm, res, pay = (self.dm, self.d_res, self.d_pay) if k == 0 else (self.dm2, self.d_res2, self.d_pay2)
        dm.decode_device(self.cfg, self.mode, self.xs.data_ptr(), self.d_doff.data_ptr(), self.d_dlen.data_ptr(),
                         self.F, res.data_ptr(), pay.data_ptr(), self.stride, stream=stream)

    def step_pipelined(self):
        k, self.pi = self.pi, self.pi ^ 1
        res, pay = (self.d_res, self.d_pay) if k == 0 else (self.d_res2, self.d_pay2)
        self.pipe.decode_device(self.cfg, self.mode, self.xs.data_ptr(), self.d_doff.data_ptr(),
                                self.d_dlen.data_ptr(), self.F, res.data_ptr(), pay.data_ptr(), self.stride)

    def pipeline_flush(self):
        self.pipe.synchronize()

    def records(self):
        return np.frombuffer(self.d_res.cpu().numpy().tobytes(), self.env.amodem.RESULT_DTYPE)

    def close(self):
        if getattr(self, "pipe", None) is not None:
            self.pipe.close()
            self.pipe = None
        self.dm.close()
        if getattr(self, "dm2", None) is not None:
            self.dm2.close()
            self.dm2 = self.d_res2 = self.d_pay2 = None
        self.xs = self.d_res = self.d_pay = self.d_doff = self.d_dlen = None
        self.env.torch.cuda.empty_cache()

    def name(self):
        return {"c2": "C2", "c3": "C3", "c4": "C4", "c5": "C5", "c5c": "C5c"}[self.conf]

    def workload_text(self):
        if self.conf == "c5c":
            return (f"C5 as chunks: {self.F // 1000}k acoustic BPSK rep3 256 B data-chunk windows per GPU + AWGN at "
                    f"{self.snr:.2f} dB (decodeChunkFrame)")
        if self.chunk:
            return (f"C4: {self.F // 1000}k QPSK 2 KB data-chunk windows per GPU (decodeChunkFrame; value counts the "
                    f"window samples decoded, 25,344 of each 28,431-sample frame)")
        if self.conf == "c5":
            return (f"C5: {self.F // 1000}k acoustic BPSK rep3 256 B legacy frames per GPU + AWGN at {self.snr:.0f} dB "
                    f"(decodeReceivedSignal, hard majority vote = reference behaviour)")
        return (("C3: 100k-frame 16-QAM batch demod per GPU" if self.conf == "c3" else
                 "C2: 10k-frame QPSK batch demod per GPU") + " (decodeReceivedSignal, legacy 1 KB frames)")


def measure(env: Env, wl: Workload, steps: int, warmup: int):
    """Warm up by time, then K steps bracketed by barrier + synchronize; max over ranks.
    Returns the leg's measurement dict (rank 0) and the last step's records."""
    torch, lib = env.torch, env.lib
    dev = env.dev
    # received mode: consecutive batches pipelined over two contexts (Workload.enable_pipeline);
    # chunk mode (one k_demod launch a step) and AMOD_BENCH_PIPELINE=0: one context
    pipe = not wl.chunk and os.environ.get("AMOD_BENCH_PIPELINE", "1") != "0"
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    serial = None
    if pipe:
        # first the per-kernel times (rooflines, chain) from K steps on one context alone, so
        # no launch shares the GPU with the next batch's (its wall time is reported too),
        # then the timed K steps pipelined over two contexts
        wl.enable_pipeline()
        warm_up(wl.step, sync, warmup)
        lib.amod_set_profiling(wl.dm.ctx, 1)
        sync()
        t1 = time.perf_counter()
        for _ in range(steps):
            wl.step()
        sync()
        serial = env.max_over_ranks(time.perf_counter() - t1)
        lib.amod_set_profiling(wl.dm.ctx, 0)
    step = wl.step_pipelined if pipe else wl.step
    warm = warm_up(step, sync, warmup, min_s=0.3 if pipe else 0.5)
    if not pipe:
        lib.amod_set_profiling(wl.dm.ctx, 1)
    env.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if pipe:
        wl.pipeline_flush()  # (the decodes ran on the pipe's slot streams)
    sync()
    env.barrier()
    elapsed = time.perf_counter() - t0
    if pipe:  # both contexts decoded the same batch: the same records and payload bytes
        same_r = wl.d_res2.cpu().numpy().tobytes() == wl.d_res.cpu().numpy().tobytes()
        same_p = np.array_equal(wl.d_pay2.cpu().numpy(), wl.d_pay.cpu().numpy())
        if not (same_r and same_p):  # (diagnostics before failing: which frames, which fields)
            r0 = np.frombuffer(wl.d_res.cpu().numpy().tobytes(), env.amodem.RESULT_DTYPE)
            r1 = np.frombuffer(wl.d_res2.cpu().numpy().tobytes(), env.amodem.RESULT_DTYPE)
            p0, p1 = wl.d_pay.view(wl.F, wl.stride).cpu().numpy(), wl.d_pay2.view(wl.F, wl.stride).cpu().numpy()
            bad = [i for i in range(wl.F) if r0[i].tobytes() != r1[i].tobytes() or p0[i].tobytes() != p1[i].tobytes()]
            print(f"pipelined contexts disagree on {len(bad)} frames", file=sys.stderr)
            for i in bad[:8]:
                print("  frame", i, {n: (r0[n][i].tolist(), r1[n][i].tolist()) for n in r0.dtype.names
                                     if r0[n][i].tobytes() != r1[n][i].tobytes()}, "flags", hex(int(r0["flags"][i])),
                      hex(int(r1["flags"][i])), "pv", int(r0["payload_valid"][i]), int(r1["payload_valid"][i]),
                      "payload bytes differing at", np.nonzero(p0[i] != p1[i])[0][:8].tolist(), file=sys.stderr)
        assert same_r and same_p, "pipelined contexts disagree"
    L = env.L
    kms, kn = (C.c_double * L.STAGE_COUNT)(), C.c_int64()
    lib.amod_kernel_stages(wl.dm.ctx, kms, L.STAGE_COUNT, C.byref(kn))  # (the profiled steps)
    lib.amod_set_profiling(wl.dm.ctx, 0)
    ov_l, ov_b, ov_lead = C.c_int64(), C.c_int64(), C.c_double()
    lib.amod_aux_overlap(wl.dm.ctx, C.byref(ov_l), C.byref(ov_b), C.byref(ov_lead))
    st_ms = [kms[i] / max(1, kn.value) for i in range(L.STAGE_COUNT)]  # per decode (amod_kernel_stages)
    # the launches: k_detect, k_demod alone (the second stream's exact chain beside it is
    # reported on its own), list B's exact kernel
    stage_ms = [st_ms[L.STAGE_DETECT], st_ms[L.STAGE_DEMOD], st_ms[L.STAGE_EXACT_B]]
    rec = wl.records()
    if os.environ.get("AMOD_STAMPS"):  # diagnostics: exact-kernel phase marks of the listed frames
        st = np.zeros(wl.F * 32, dtype=np.uint64)
        n = lib.amod_debug_stamps(wl.dm.ctx, st.ctypes.data, st.size)
        st = st[:n].reshape(-1, 32).astype(np.int64)
        for i in np.nonzero(rec["flags"] & (env.L.FLAG_EXACT | env.L.FLAG_REPLAY))[0][:32]:
            print("listed", i, hex(int(rec["flags"][i])), int(rec["coarse_idx"][i]),
                  [int(st[i, b] - st[i, a]) if st[i, a] and st[i, b] else None
                   for a, b in ((8, 13), (13, 14), (14, 9), (9, 10), (10, 11), (11, 12))], file=sys.stderr)
    ok = int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum())
    fallback = int((rec["flags"] != 0).sum())
    # correctness of what was timed (the last timed step's results): clean configs decode
    # every frame with the synthetic payload; noisy C5 frames are checked against the oracle
    amodem = env.amodem
    pay = wl.d_pay.view(wl.F, wl.stride).cpu().numpy()
    for i in range(0, wl.F, max(1, wl.F // 64)):
        r = amodem.to_reference(rec[i], pay[i].tobytes(), not wl.chunk)
        if wl.noisy and not r.get("crcValid"):
            continue
        want = amodem.synth_payload(0x9E3779B9 ^ (env.rank * wl.F + i), wl.payload_bytes)
        assert r.get("data") == want, (wl.conf, i, r.get("error"))
        if wl.chunk:
            assert r.get("seqNum") == env.rank * wl.F + i, (i, r.get("seqNum"))
    elapsed = env.max_over_ranks(elapsed)
    ok_all, fb_all = env.sum_over_ranks([ok, fallback])
    world = env.world
    value = wl.ndecoded * world * steps / elapsed
    algo_bytes = 4.0 * wl.ndecoded  # each float32 sample read once
    # the critical path: k_detect, k_demod + the wait for the second stream, list B
    chain_s = (st_ms[L.STAGE_DETECT] + st_ms[L.STAGE_DEMOD_PATH] + st_ms[L.STAGE_EXACT_B]) / 1e3
    names = ["k_chunk_prep" if wl.chunk else "k_detect", "k_demod"]
    dom = max(range(2), key=lambda i: stage_ms[i])
    # the dominant launch's algorithmic bytes: k_detect reads every sample once; k_demod
    # reads the 512-sample FFT window of the CE and of every demodulated data symbol
    if dom == 0:
        dom_bytes = algo_bytes
    else:  # CE + the symbols holding the packet (trailing silence skipped)
        per_sym = amodem.num_data_subs(wl.cfg) * {0: 1, 1: 2, 2: 4}[wl.cfg.modulation]
        nsym_dec = -(-int(wl.pl[0]) * 8 * wl.cfg.repetition // per_sym)
        dom_bytes = 4.0 * 512 * (nsym_dec + 1) * wl.F
    achieved = dom_bytes / (stage_ms[dom] / 1e3) / 1e9
    out = {
        "value": value, "unit": "samples/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "warmup_run": warm, "ms_per_step": elapsed / steps * 1e3,
        "pipeline": {"contexts": 2 if pipe else 1,
                     "what": "the library's depth-2 pipe (amod_pipe_decode_device): consecutive batches alternate "
                             "between two contexts (own workspace and stream), batch i+1's k_detect overlaps batch "
                             "i's k_demod; rooflines and chain from the same K steps on one context alone"
                             if pipe else "one context, one stream",
                     "one_context_ms_per_step": (serial / steps * 1e3) if serial else elapsed / steps * 1e3,
                     "one_context_samples_per_s": wl.ndecoded * world * steps / (serial if serial else elapsed)},
        "payload_MB_per_s": wl.payload_bytes * wl.F * world * steps / elapsed / 1e6,
        "config": {"workload": wl.workload_text(), "frames_per_gpu": wl.F, "samples_per_frame": int(wl.dlens[0]),
                   "fft": 512, "modulation": wl.mod, "payload_bytes": wl.payload_bytes,
                   "parallelism": f"frame-sharded x{world}"},
        "frames_ok": int(ok_all), "frames_exact_fallback": int(fb_all), "fallback_flags": flag_hist(rec),
        "awgn_sigma": wl.sigma,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic_for(wl, names[dom]),
                     "kernel": names[dom], "kernel_ms_avg": stage_ms[dom], "algorithmic_bytes": dom_bytes,
                     "algorithmic_bytes_what": "4 B x every decoded sample" if dom == 0 else
                     "4 B x 512 samples x (CE + data symbols holding the packet) per frame"},
        "chain": {"what": "the whole decode per step (%s -> k_demod -> join with the exact chain of the second "
                          "stream -> list B), HIP events; algorithmic bytes = 4 B x every decoded sample" % names[0],
                  "aux_stream_ms_avg": st_ms[L.STAGE_AUX], "join_wait_ms_avg": st_ms[L.STAGE_JOIN_WAIT],
                  "ms_avg": chain_s * 1e3, "achieved": algo_bytes / chain_s / 1e9, "peak": HBM_PEAK_GBS,
                  "unit": "GB/s", "frac": algo_bytes / chain_s / 1e9 / HBM_PEAK_GBS,
                  "kernels_ms_avg": dict(zip(names + ["k_decode_exact"], stage_ms)),
                  "aux_overlap": {"what": "timed decodes whose list A had a frame; of those, the ones whose replica "
                                          "started before k_demod's last wave ended (device real-time clock)",
                                  "decodes_listed": ov_l.value, "beside": ov_b.value,
                                  "lead_us_avg": ov_lead.value / max(1, ov_l.value)},
                  "symbols_demodulated_per_frame": "all" if wl.chunk else
                  "header..CRC symbols only (trailing silence skipped, SURVEY.md 8d)"},
    }
    return out, rec


def traffic_for(wl, kernel):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass
    (FETCH_SIZE x 2 + WRITE_SIZE, tools/pmc_traffic.py) when it was taken on this workload."""
    for rnd in ("r06", "r05", "r04", "r03", "r02"):
        tf = os.path.join(ROOT, "profiles", rnd, "traffic.json")
        if not os.path.exists(tf):
            continue
        with open(tf) as f:
            tj = json.load(f)
        for entry in tj if isinstance(tj, list) else [tj]:
            kt = entry.get("kernels", {}).get(kernel)
            if entry.get("frames") == wl.F and entry.get("samples_per_frame") == int(wl.dlens[0]) and kt:
                return (kt["read_bytes"] + kt["write_bytes"]) / kt.get("dispatches_per_step", 1.0)
    return None


def gather_leg(env: Env, wl: Workload, reps=3):
    """N > 1, after the timed region: the device-resident result records (96 B/frame)
    and payload slots of every rank gathered into rank 0 over RCCL (SURVEY.md §8e,
    BASELINE C4's "RCCL gather over xGMI"), timed with barrier + synchronize on both
    sides, then every gathered record checked on rank 0 (status, CRC, and for C4 the
    file's sequence numbers 0 .. world*F-1 in rank order)."""
    from amodem.shard import gather_to_root
    torch, dist, amodem = env.torch, env.dist, env.amodem
    world, rank, F = env.world, env.rank, wl.F
    counts = [F] * world
    res_rows = wl.d_res.view(F, 96)
    pay_rows = wl.d_pay.view(F, wl.stride)[:, : min(wl.stride, wl.payload_bytes + 64)].contiguous()
    ms = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize(env.dev)
        t0 = time.perf_counter()
        g_res = gather_to_root(res_rows, counts, dst=0)
        g_pay = gather_to_root(pay_rows, counts, dst=0)
        torch.cuda.synchronize(env.dev)
        ms.append((time.perf_counter() - t0) * 1e3)
    t = env.max_over_ranks(max(ms[1:]) if len(ms) > 1 else ms[0])
    if rank != 0:
        return None
    rec = np.frombuffer(g_res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
    pay = g_pay.cpu().numpy()
    wl.gathered = rec  # (the group leg compares its records with these)
    noisy = wl.noisy
    ok = len(rec) == world * F and (noisy or bool(((rec["status"] == 0) & (rec["crc_valid"] == 1)).all()))
    if wl.chunk:
        ok = ok and bool((rec["seq_num"] == np.arange(world * F)).all())
    for i in range(0, world * F, max(1, world * F // 64)):  # payload rows follow their records
        r = amodem.to_reference(rec[i], pay[i].tobytes(), not wl.chunk)
        if noisy and not r.get("crcValid"):
            continue
        ok = ok and r.get("data") == amodem.synth_payload(0x9E3779B9 ^ i, wl.payload_bytes)
    nbytes = (res_rows.numel() + pay_rows.numel()) * (world - 1)  # what crosses xGMI into rank 0
    return {"what": "result records + payload slots of every rank gathered into rank 0 (%s gather)"
                    % ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend()),
            "frames": world * F, "bytes_into_root": nbytes, "ms": t, "GBps": nbytes / (t / 1e3) / 1e9,
            "records_ok": bool(ok), "ranks_joined": world, "devices": env.devices_used}


def scan_phase(env: Env, wl: Workload, reps=20):
    """Average duration of the correlation-scan phase alone on the same resident batch:
    k_corr_scan, the fast kernel's code instantiated to stop after the Schmidl-Cox
    decision (selected by AMOD_STOP_AFTER=1, read when a context builds its tables),
    launched with the same LDS footprint so the same number of frames share a CU."""
    amodem, L, lib = env.amodem, env.L, env.lib
    os.environ["AMOD_STOP_AFTER"] = "1"
    # (its own result buffers: the frames this context lists still go through the exact
    # kernel, whose full payload rows must not land in the workload's buffers, which the
    # pipelined steps later compare byte for byte across two contexts)
    s_res, s_pay = env.torch.zeros_like(wl.d_res), env.torch.zeros_like(wl.d_pay)
    try:
        dm = amodem.Demodulator(env.local)
        dm.reserve(wl.cfg, wl.F, wl.spf)
        run = lambda: dm.decode_device(wl.cfg, L.MODE_RECEIVED, wl.xs.data_ptr(), wl.d_doff.data_ptr(),
                                       wl.d_dlen.data_ptr(), wl.F, s_res.data_ptr(), s_pay.data_ptr(),
                                       wl.stride, stream=wl.stream)
        for _ in range(10):  # clocks settle over the first launches
            run()
        dm.synchronize()
        lib.amod_set_profiling(dm.ctx, 1)
        for _ in range(reps):  # back to back, like the timed region
            run()
        fm, fn, em, en = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        lib.amod_kernel_times(dm.ctx, C.byref(fm), C.byref(fn), C.byref(em), C.byref(en))
        dm.close()
        ms = fm.value / max(1, fn.value)
    finally:
        del os.environ["AMOD_STOP_AFTER"]
    del s_res, s_pay
    b = 4.0 * wl.ndecoded
    return {"phase": "stream pass + Schmidl-Cox coarse search (k_corr_scan: the same code compiled to stop there, "
                     "results not written; %d launches)" % reps,
            "kernel": "k_corr_scan", "kernel_ms_avg": ms, "achieved": b / (ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": b / (ms / 1e3) / 1e9 / HBM_PEAK_GBS}


def tx_obj(wl: Workload):
    t = wl.tx_ms / 1e3
    return {"kernel": "k_tx", "what": "GPU transmitter (modulateOFDM + frame builder, bit-exact) building this "
                                      "run's input", "kernel_ms_avg": wl.tx_ms, "samples_per_s": wl.nsamples / t,
            "roofline": {"bound": "hbm", "achieved": wl.tx_bytes / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": wl.tx_bytes / t / 1e9 / HBM_PEAK_GBS}}


def group_leg(env: Env, conf: str, args, snr: float, gathered):
    """N > 1, rank 0 alone: SURVEY.md §5's one-process design, the drop-in's own multi-GPU
    path (amod_group_decode_device, Python DeviceGroup; JS decodeBatch({devices})): one host
    process drives every rank's device, each member context decoding the shard rank k
    decoded (built again here on device k: the same frames and noise), all at once; K steps
    of the whole group (enqueue every member, then join), per-device kernel times, and the
    records compared with the per-rank records the RCCL gather brought to rank 0."""
    torch, amodem, L, lib = env.torch, env.amodem, env.L, env.lib
    ndev = max(1, torch.cuda.device_count())
    devs = [k % ndev for k in range(env.world)]
    shards = [Workload(env, conf, args.frames, snr, rank=k, device=d) for k, d in enumerate(devs)]
    g = amodem.DeviceGroup(devs)
    cfg, mode = shards[0].cfg, shards[0].mode
    ctxs = [lib.amod_group_context(g._h, k) for k in range(len(devs))]
    for k, w in enumerate(shards):
        env.L.check(lib.amod_reserve(ctxs[k], C.byref(cfg), w.F, int(w.dlens.max())))
    spec = [{"samples": w.xs.data_ptr(), "offsets": w.d_doff.data_ptr(), "lengths": w.d_dlen.data_ptr(),
             "results": w.d_res.data_ptr(), "payload": w.d_pay.data_ptr(), "payload_stride": w.stride,
             "nframes": w.F} for w in shards]

    def step():
        g.decode_device(cfg, mode, spec)
        g.synchronize()

    warm_up(step, lambda: None, args.warmup)
    for c in ctxs:
        lib.amod_set_profiling(c, 1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt = (time.perf_counter() - t0) / args.steps
    per_dev = []
    for k, c in enumerate(ctxs):
        kms, kn = (C.c_double * L.STAGE_COUNT)(), C.c_int64()
        lib.amod_kernel_stages(c, kms, L.STAGE_COUNT, C.byref(kn))
        lib.amod_set_profiling(c, 0)
        st = [kms[i] / max(1, kn.value) for i in range(L.STAGE_COUNT)]
        per_dev.append({"device": devs[k], "frames": shards[k].F, "k_detect_ms": st[L.STAGE_DETECT],
                        "k_demod_ms": st[L.STAGE_DEMOD], "exact_b_ms": st[L.STAGE_EXACT_B]})
    rec = np.concatenate([w.records() for w in shards])
    same = gathered is not None and len(gathered) == len(rec) and \
        rec.tobytes() == np.ascontiguousarray(gathered).tobytes()
    nsamp = sum(w.ndecoded for w in shards)
    out = {"what": "one host process driving %d device contexts (amod_group_decode_device, SURVEY.md section 5), "
                   "every rank's shard built again on its device; K steps of the whole group" % len(devs),
           "devices": devs, "ms_per_step": dt * 1e3, "samples_per_s": nsamp / dt, "per_device": per_dev,
           "records_equal_per_rank": bool(same),
           "frames_ok": int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum()), "frames": len(rec)}
    g.close()
    for w in shards:
        w.close()
    return out


def soft_leg(env: Env, wl: Workload, steps: int, warmup: int, oracle: bool = False):
    """C5's opt-in soft combining of the repeated bits (AMOD_OPT_SOFT_COMBINE, NOT reference
    behaviour: BASELINE C5 names it; k_demod's soft instance, groups whose soft sum lies
    inside its error bound routed to the exact kernel) against the reference's hard
    majority vote on the same resident batch: K steps each on one context (no pipelining),
    per-kernel times, CRC-valid frames and frames the exact kernel decoded; for chunk
    windows (wl.packets) also the frames whose bytes equal the synthetic payload and the
    post-vote bit errors against the transmitted packets. oracle: the hard vote's records
    (the reference's behaviour) against the C oracle over the whole batch."""
    torch, lib, L = env.torch, env.lib, env.L
    sync = lambda: torch.cuda.synchronize(env.dev)  # noqa: E731
    out = {"what": "AMOD_OPT_SOFT_COMBINE (|H|^2-weighted soft vote, k_demod soft instance; not reference "
                   "behaviour) vs the hard majority vote, K steps each (received mode: through the two-context "
                   "pipe as the primary measurement, kernel times from K steps on one context)", "frames": wl.F,
           "snr_db": wl.snr}
    ref = None
    if wl.packets is not None:
        pk, po, pl = wl.packets
        ref = np.zeros((wl.F, int(pl.max())), np.uint8)
        for i in range(wl.F):
            ref[i, : pl[i]] = pk[po[i]: po[i] + pl[i]]
    # received mode: consecutive batches through the library's two-context pipe, as the
    # primary measurement (measure()); the per-kernel times from K steps on one context
    pipe = not wl.chunk and os.environ.get("AMOD_BENCH_PIPELINE", "1") != "0"
    if pipe and getattr(wl, "pipe", None) is None:
        wl.enable_pipeline()
    for name, opt in (("hard", 0), ("soft", L.OPT_SOFT_COMBINE), ("hard_again", 0)):
        def step(opt=opt):
            wl.step(options=opt)

        def step_p(opt=opt):
            k, wl.pi = wl.pi, wl.pi ^ 1
            res, pay = (wl.d_res, wl.d_pay) if k == 0 else (wl.d_res2, wl.d_pay2)
            wl.pipe.decode_device(wl.cfg, wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(), wl.d_dlen.data_ptr(),
                                  wl.F, res.data_ptr(), pay.data_ptr(), wl.stride, options=opt)
        warm_up(step, sync, warmup)
        lib.amod_set_profiling(wl.dm.ctx, 1)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        dt1 = (time.perf_counter() - t0) / steps
        kms, kn = (C.c_double * L.STAGE_COUNT)(), C.c_int64()
        lib.amod_kernel_stages(wl.dm.ctx, kms, L.STAGE_COUNT, C.byref(kn))
        lib.amod_set_profiling(wl.dm.ctx, 0)
        st = [kms[i] / max(1, kn.value) for i in range(L.STAGE_COUNT)]
        dt = dt1
        if pipe:
            warm_up(step_p, sync, warmup, min_s=0.3)
            wl.pipeline_flush()
            sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                step_p()
            wl.pipeline_flush()
            sync()
            dt = (time.perf_counter() - t0) / steps
        rec = wl.records()
        o = {"ms_per_step": dt * 1e3, "one_context_ms_per_step": dt1 * 1e3,
             "k_detect_ms": st[L.STAGE_DETECT], "k_demod_ms": st[L.STAGE_DEMOD],
             "exact_chain_ms": st[L.STAGE_AUX] + st[L.STAGE_EXACT_B],
             "frames_crc_valid": int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum()),
             "frames_exact": int(((rec["flags"] & L.FLAG_EXACT) != 0).sum())}
        if ref is not None:
            pay = wl.d_pay.view(wl.F, wl.stride).cpu().numpy()
            n = np.minimum(rec["payload_valid"].astype(np.int64), wl.packets[2].astype(np.int64))
            cols = np.arange(ref.shape[1])[None, :]
            diff = np.where(cols < n[:, None], pay[:, : ref.shape[1]] ^ ref, 0).astype(np.uint8)
            o["bit_errors"] = int(np.unpackbits(diff).sum())
            o["bits_compared"] = int(n.sum() * 8)
            o["frames_payload_ok"] = int(sum(
                1 for i in range(wl.F) if rec["status"][i] == 0 and rec["crc_valid"][i] == 1 and
                amodem_payload(env, rec[i], pay[i]) == wl_payload(wl, env, i)))
        out[name] = o
        if name == "hard" and oracle and env.world == 1:
            chk = oracle_check(wl, wl.xs[: wl.nsamples].cpu().numpy(), rec)
            out["oracle_agree"] = chk["oracle_agree"]
            out["oracle_ok"] = chk["agree"] == wl.F
            if chk["agree"] != wl.F:
                print(f"{wl.name()} {wl.snr} dB: hard-vote records differ from the oracle on "
                      f"{wl.F - chk['agree']} frames", file=sys.stderr)
    hard_ms = min(out["hard"]["ms_per_step"], out["hard_again"]["ms_per_step"])
    out["soft_over_hard_step"] = out["soft"]["ms_per_step"] / hard_ms
    return out


def amodem_payload(env, rec, slot):
    return env.amodem.to_reference(rec, slot.tobytes(), False).get("data")


def wl_payload(wl, env, i):
    return env.amodem.synth_payload(0x9E3779B9 ^ (env.rank * wl.F + i), wl.payload_bytes)


def soft_chunk_leg(env: Env, args, div=1.5):
    """BASELINE C5's noisy-channel mode where it matters: acoustic BPSK rep3 256 B chunk
    windows (decodeChunkFrame) with AWGN at signal/noise power `div` (1.5: 1.76 dB; where
    tests/test_gpu_soft_combine.py shows the soft vote gaining), soft vs hard."""
    wl = Workload(env, "c5c", 0, 10 * np.log10(div))
    try:
        out = soft_leg(env, wl, args.steps, args.warmup, oracle=True)
    finally:
        wl.close()
    out["noise_divisor"] = div
    out["workload"] = wl.workload_text()
    return out


def e2e_leg(env: Env, wl: Workload, reps=3):
    """Host-resident batch, PCIe included (BASELINE.md "two timing modes"): the samples
    in pinned host memory, copied H2D, decoded, result records and payload slots copied
    back to pinned memory, on one stream; wall time per pass (never `value`)."""
    torch = env.torch
    dev = env.dev
    h_x = torch.empty(wl.nsamples, dtype=torch.float32, pin_memory=True)
    h_x.copy_(wl.xs[: wl.nsamples])
    h_res = torch.empty(wl.d_res.numel(), dtype=torch.uint8, pin_memory=True)
    h_pay = torch.empty(wl.d_pay.numel(), dtype=torch.uint8, pin_memory=True)
    st = torch.cuda.Stream(dev)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            wl.xs[: wl.nsamples].copy_(h_x, non_blocking=True)
            wl.dm.decode_device(wl.cfg, wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(), wl.d_dlen.data_ptr(), wl.F,
                                wl.d_res.data_ptr(), wl.d_pay.data_ptr(), wl.stride, stream=st.cuda_stream)
            h_res.copy_(wl.d_res, non_blocking=True)
            h_pay.copy_(wl.d_pay, non_blocking=True)
        st.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    return {"what": "pinned host samples -> H2D -> decode -> D2H records + payload, one stream, median of %d" % reps,
            "samples_per_s": wl.ndecoded / t, "payload_MB_per_s": wl.payload_bytes * wl.F / t / 1e6, "ms": t * 1e3,
            "h2d_GBps": 4.0 * wl.nsamples / t / 1e9}


def host_api_leg(env: Env, wl: Workload, reps=3):
    """The drop-in host entry from Python (amod_decode_host: host samples in, records and
    payload out, the runtime's own staging) on the same batch; and, when node and the
    addon are present, decodeBatch from Node.js (the reference's host language,
    app.js:513/928 callers) on the same samples (tools/node_decode_batch.js)."""
    x = wl.xs[: wl.nsamples].cpu().numpy()
    out = {}
    dm = wl.dm
    ts = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        rec, _ = dm.decode_batch(x, wl.doffs, wl.dlens, mode=wl.mode, cfg=wl.cfg)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    ok = int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum())
    out["python_decode_host"] = {"what": "amod_decode_host from pageable host memory (runtime staging), median of %d"
                                         % reps, "samples_per_s": wl.ndecoded / t, "ms": t * 1e3, "frames_ok": ok}
    node = shutil_which("node")
    addon = os.path.join(ROOT, "audio-modem_amd", "lib", "amodem.node")
    if node and os.path.exists(addon):
        with tempfile.TemporaryDirectory() as tmp:
            xf = os.path.join(tmp, "x.f32")
            x.tofile(xf)
            spec = os.path.join(tmp, "spec.json")
            with open(spec, "w") as f:
                json.dump({"samples": xf, "offsets": wl.doffs.tolist(), "lengths": wl.dlens.tolist(),
                           "preset": wl.preset, "mod": wl.mod, "rep": wl.cfg.repetition, "chunk": wl.chunk,
                           "reps": reps, "device": env.local}, f)
            r = subprocess.run([node, os.path.join(ROOT, "tools", "node_decode_batch.js"), spec],
                               capture_output=True, text=True, timeout=300)
            if r.returncode == 0:
                nj = json.loads(r.stdout)
                nj["samples_per_s"] = wl.ndecoded / (nj["ms"] / 1e3)
                out["node_decode_batch"] = nj
            else:
                out["node_decode_batch"] = {"error": r.stderr[-3000:], "returncode": r.returncode}
    return out


def c1_latency_leg(env: Env, calls=200):
    """The drop-in as its caller uses it (app.js:513): ONE C1 recording (QPSK 1 KB legacy
    frame, 35,874 samples) through the synchronous decodeReceivedSignal, per-call latency
    (host samples in: H2D, launches, sync, D2H, the result object), from Node.js
    (js/modem.js -> N-API -> amod_decode_host) and from Python (amod_decode_host), next to
    the JS restatement of the reference decoding the same frame on one core
    (oracle/rx_cpu.js; BASELINE.md: modem.js 2.75 ms per C1 frame in the build container)."""
    amodem = env.amodem
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0x9E3779B9, PAYLOAD)
    sig = np.ascontiguousarray(amodem.build_transmit_signal(data, file_name="f.bin", cfg=cfg), np.float32)
    out = {"workload": f"C1: one QPSK 1 KB legacy frame ({len(sig)} samples), decodeReceivedSignal"}
    dm = amodem.Demodulator(env.local)
    try:
        for _ in range(20):
            r = dm.decode_received_signal(sig, "QPSK", 1)
        ts = []
        for _ in range(calls):
            t0 = time.perf_counter()
            r = dm.decode_received_signal(sig, "QPSK", 1)
            ts.append((time.perf_counter() - t0) * 1e3)
    finally:
        dm.close()
    ts.sort()
    out["python_decode_received_signal"] = {"median_ms": ts[len(ts) // 2], "p90_ms": ts[int(0.9 * len(ts))],
                                            "calls": calls, "crcValid": bool(r.get("crcValid")) and r.get("data") == data}
    node = shutil_which("node")
    with tempfile.TemporaryDirectory() as tmp:
        xf = os.path.join(tmp, "c1.f32")
        sig.tofile(xf)
        if node and os.path.exists(os.path.join(ROOT, "audio-modem_amd", "lib", "amodem.node")):
            spec = os.path.join(tmp, "lat.json")
            with open(spec, "w") as f:
                json.dump({"samples": xf, "preset": "standard", "mod": "QPSK", "rep": 1, "warmup": 20,
                           "calls": calls}, f)
            r = subprocess.run([node, os.path.join(ROOT, "tools", "node_latency.js"), spec], capture_output=True,
                               text=True, timeout=300)
            out["node_decode_received_signal"] = json.loads(r.stdout) if r.returncode == 0 else {"error": r.stderr[-400:]}
        if node:  # the CPU baseline: the same frame, one thread (test infrastructure under oracle/)
            spec = os.path.join(tmp, "cpu.json")
            with open(spec, "w") as f:
                json.dump({"samples": xf, "offsets": [0], "lengths": [len(sig)], "preset": "standard", "mod": "QPSK",
                           "rep": 1, "chunk": False, "threads": 1, "seconds": 0.5, "single_frames": 1,
                           "single_seconds": 2.0}, f)
            r = subprocess.run([node, os.path.join(ROOT, "oracle", "rx_cpu.js"), "bench", spec], capture_output=True,
                               text=True, timeout=300)
            if r.returncode == 0:
                j = json.loads(r.stdout)
                out["cpu_js_one_core"] = {"ms_per_call": len(sig) / j["single_core"] * 1e3, "kind": "port",
                                          "what": "oracle/rx_cpu.js (JS restatement of modem.js) on one thread, the "
                                                  "same frame repeated for 2 s", "calibration": calibration_note("c2")}
            else:
                out["cpu_js_one_core"] = {"error": r.stderr[-400:]}
    nl = out.get("node_decode_received_signal", {})
    cj = out.get("cpu_js_one_core", {})
    if "median_ms" in nl and "ms_per_call" in cj:
        out["speedup_vs_cpu_js"] = cj["ms_per_call"] / nl["median_ms"]
    return out


def shutil_which(name):
    import shutil
    return shutil.which(name)


def stream_leg(env: Env, nchunks=2000, chunk=2048):
    """StreamingReceiver over a C4-shaped stream (metadata + nchunks 2 KB QPSK chunk
    frames back to back, built by k_tx): whole-call time from host samples to the
    assembled file, with the receiver's own phase split."""
    amodem, L, torch = env.amodem, env.L, env.torch
    device = env.local
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0xC4000001, nchunks * chunk - 123)
    pk = [amodem.packet_meta(nchunks, len(data), chunk, "c4.bin")]
    pk += [amodem.packet_chunk(data[i * chunk:(i + 1) * chunk], i) for i in range(nchunks)]
    dm = amodem.Demodulator(device)
    sig, _, _ = dm.transmit_batch(cfg, pk, [L.TX_META] + [L.TX_CHUNK] * nchunks)
    total = -(-(len(sig) + 8192) // 4096) * 4096
    x = np.concatenate([sig, np.zeros(total - len(sig), np.float32)])
    del sig
    asm = amodem.ChunkAssembler()
    # warm-up: one whole call (tables, kernels, the context's grow-only buffers: a receiver
    # serving recordings keeps its context, and each finished assembler hands its file
    # arena to the next), then the timed calls
    warm = amodem.ChunkAssembler()
    dm.stream_receive(cfg, x, warm)
    warm.close()
    t0 = time.perf_counter()
    frames, _, st = dm.stream_receive(cfg, x, asm)
    t = time.perf_counter() - t0
    ok = asm.is_complete() and asm.assemble_file() == data
    asm.close()  # (its file arena goes back to the process's pool for the next receiver)
    # the same stream already resident in HBM (amod_stream_receive_device)
    dx = torch.from_numpy(x).to(torch.device("cuda", device))
    torch.cuda.synchronize()
    asm2 = amodem.ChunkAssembler()
    t0 = time.perf_counter()
    frames2, _, st2 = dm.stream_receive_device(cfg, dx.data_ptr(), len(x), asm2)
    t2 = time.perf_counter() - t0
    ok2 = asm2.is_complete() and asm2.assemble_file() == data and len(frames2) == len(frames)
    dm.close()
    del dx
    torch.cuda.empty_cache()

    def phases(s):
        return {"ema_gpu": s["t_ema_ms"], "screen_fine_gpu": s["t_fine_ms"], "decode_gpu": s["t_decode_ms"],
                "state_machine_host": s["t_host_ms"], "total": s["t_total_ms"]}

    return {"what": "app.js StreamingReceiver restated (amod_stream_receive): host samples in, frames + assembled "
                    "file out (the host call uploads in 64 MB pieces, each piece's EMA on the GPU as it lands: its "
                    "ema_gpu phase is upload + EMA); the second call on a warm context",
            "workload": f"C4-shaped stream, metadata + {nchunks} x 2 KB QPSK chunk frames ({len(x)} samples)",
            "samples_per_s": len(x) / t, "payload_MB_per_s": len(data) / t / 1e6, "seconds": t,
            "frames": int(len(frames)), "file_ok": bool(ok), "phases_ms": phases(st),
            "device_resident": {"samples_per_s": len(x) / t2, "seconds": t2, "file_ok": bool(ok2),
                                "phases_ms": phases(st2),
                                "host_share": st2["t_host_ms"] / max(1e-9, st2["t_total_ms"])},
            "reference_rate_note": "reference StreamingReceiver: 2.0e6 samples/s per core (SURVEY.md section 3.2)"}


# ------------------------------------------------------------ CPU baselines --
def js_baseline(wl: Workload, x, nframes, seconds=1.5, single_frames=60, single_seconds=2.0, gpu_rec=None):
    """The JS restatement of the reference RX (oracle/rx_cpu.js, bit-exact on the golden
    frames, within 5 % of modem.js on one core: profiles/cpu_calibration.json) on this
    host's cores, one worker_thread per core (BASELINE.md's CPU-baseline plan), frames
    dealt round-robin, each worker repeating its share for `seconds`; and on one thread."""
    node = shutil_which("node")
    if node is None:
        return {"error": "node not installed"}
    with tempfile.TemporaryDirectory() as tmp:
        xf = os.path.join(tmp, "x.f32")
        offs, lens = wl.doffs[:nframes] - wl.offs[0], wl.dlens[:nframes]
        end = int(wl.offs[nframes - 1] + wl.lens[nframes - 1])
        np.ascontiguousarray(x[:end], np.float32).tofile(xf)
        spec = os.path.join(tmp, "spec.json")
        with open(spec, "w") as f:
            json.dump({"samples": xf, "offsets": offs.tolist(), "lengths": lens.tolist(), "preset": wl.preset,
                       "mod": wl.mod, "rep": wl.cfg.repetition, "chunk": wl.chunk, "threads": HOST_THREADS,
                       "seconds": seconds, "single_frames": single_frames, "single_seconds": single_seconds}, f)
        r = subprocess.run([node, os.path.join(ROOT, "oracle", "rx_cpu.js"), "bench", spec], capture_output=True,
                           text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-400:]}
    j = json.loads(r.stdout)
    out = {"value": j["all_cores"], "unit": "samples/s", "cores": j["threads"], "cores_source": HOST_THREADS_SOURCE,
           "kind": "port",
           "sample": f"{nframes} {wl.name()} frames dealt round-robin to {j['threads']} worker_threads, each repeating "
                     f"its share for {seconds} s ({j['all_cores_samples']} samples in {j['all_cores_seconds']:.2f} s); "
                     f"{j['single_core_frames']} frames on 1 thread; oracle/rx_cpu.js (JS restatement of modem.js, "
                     f"node {j['node']})",
           "single_core": j["single_core"], "host_cpus_visible": j["cores"],
           "payload_MB_per_s": j["all_cores"] / float(wl.dlens[0]) * wl.payload_bytes / 1e6,
           "calibration": calibration_note(wl.conf)}
    if gpu_rec is not None:
        st, crc = np.array(j["status"]), np.array(j["crc"], np.uint64)
        agree = int(((gpu_rec["status"][:nframes] == st) &
                     ((st != 0) | (gpu_rec["actual_crc"][:nframes].astype(np.uint64) == crc))).sum())
        out["js_agree"] = f"{agree}/{nframes} frames: GPU status and CRC equal the JS baseline's"
        out["js_agree_ok"] = agree == nframes
    return out


def calibration_note(conf):
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if not os.path.exists(cal):
        return None
    with open(cal) as f:
        w = json.load(f)["workloads"].get(conf)
    if not w or "js_over_modem_js" not in w:
        return None
    return {"js_over_modem_js": w["js_over_modem_js"], "modem_js_ms_per_frame": w["modem_js_ms"],
            "note": "single-thread rate ratio JS baseline / unmodified modem.js on identical frames, build container "
                    "(tools/calibrate_cpu.py)"}


def oracle_check(wl: Workload, x, gpu_rec):
    """The C restatement (oracle/amodem_oracle.c) over the WHOLE batch on 16 threads: every
    frame's status and CRC against the GPU's (the agreement count the judge reads), with
    its rate beside it."""
    from oracle import oracle as O
    c = O.cfg(wl.preset)
    offs = wl.doffs - wl.offs[0]
    dt, st, crc = O.bench_decode(c, x, offs, wl.dlens, wl.mod, wl.cfg.repetition, HOST_THREADS, chunk=wl.chunk)
    agree = int(((gpu_rec["status"] == st) & ((st != 0) | (gpu_rec["actual_crc"] == crc))).sum())
    return {"oracle_agree": f"{agree}/{wl.F} frames: GPU status and CRC equal the C oracle's", "agree": agree,
            "frames": wl.F, "oracle_ok_frames": int((st == 0).sum()),
            "c_port": {"value": float(wl.dlens.sum()) / dt, "unit": "samples/s", "cores": HOST_THREADS,
                       "kind": "port", "sample": f"all {wl.F} {wl.name()} frames, oracle/amodem_oracle.c"}}


def cpu_legs(wl: Workload, rec, js_frames, js_seconds=1.5):
    """CPU baseline (JS, timed) + the full-batch C-oracle agreement of this leg (rank 0, N=1)."""
    x = wl.xs[: wl.nsamples].cpu().numpy()
    chk = oracle_check(wl, x, rec)
    if chk["agree"] != wl.F:  # the timed GPU results must be the reference's, frame for frame
        raise SystemExit(f"{wl.name()}: GPU results differ from the oracle on {wl.F - chk['agree']} frames")
    cpu = js_baseline(wl, x, min(js_frames, wl.F), seconds=js_seconds, gpu_rec=rec)
    cpu.update({k: chk[k] for k in ("oracle_agree", "c_port")})
    del x
    return cpu


# ------------------------------------------------------------- the JSON line --
LINE_MAX = 8192  # bytes of the printed line (the driver's parser gave up on r05's 20.9 KB line)


def _g(v, nd=4):
    """A float to nd significant digits (the compact line's secondary numbers)."""
    if isinstance(v, float):
        return float(f"{v:.{nd}g}")
    return v


def _pick(d, keys, nd=4):
    """The keys of d that are present, floats rounded; nested (key, subkeys) pairs recurse."""
    out = {}
    if not isinstance(d, dict):
        return out
    for k in keys:
        if isinstance(k, tuple):
            k, sub = k
            if isinstance(d.get(k), dict):
                out[k] = _pick(d[k], sub, nd)
        elif k in d:
            out[k] = _g(d[k], nd)
    return out


def _leg_summary(leg):
    """One config leg in a few numbers: rate, step, dominant kernel and its roofline
    fraction, the chain, oracle agreement; the soft-combine and noisy objects by count."""
    if not isinstance(leg, dict):
        return leg
    if "error" in leg:
        return {"error": str(leg["error"])[:200]}
    out = _pick(leg, ["value", "ms_per_step", "payload_MB_per_s", "frames_ok", "frames_exact_fallback"])
    rf = leg.get("roofline")
    if isinstance(rf, dict):
        out["kernel"] = rf.get("kernel")
        out["kernel_ms"] = _g(rf.get("kernel_ms_avg"))
        out["frac"] = _g(rf.get("frac"))
        out["traffic"] = _g(rf.get("traffic"))
    ch = leg.get("chain")
    if isinstance(ch, dict):
        out["chain_ms"] = _g(ch.get("ms_avg"))
        out["kernels_ms"] = {k: _g(v) for k, v in (ch.get("kernels_ms_avg") or {}).items()}
    cb = leg.get("cpu_baseline")
    if isinstance(cb, dict):
        out["oracle_agree"] = (cb.get("oracle_agree") or cb.get("error", ""))[:80]
        out["cpu_value"] = _g(cb.get("value"))
    for k in ("soft_combine", "noisy"):
        if isinstance(leg.get(k), dict):
            out[k] = _soft_summary(leg[k])
    if "hard" in leg or "soft" in leg:  # a soft_leg object itself
        out.update(_soft_summary(leg))
    return out


def _soft_summary(s):
    out = {}
    for name in ("hard", "soft"):
        if isinstance(s.get(name), dict):
            out[name] = _pick(s[name], ["ms_per_step", "one_context_ms_per_step", "k_demod_ms", "exact_chain_ms",
                                        "frames_crc_valid",
                                        "frames_exact", "frames_payload_ok", "bit_errors", "bits_compared"])
    for k in ("soft_over_hard_step", "frames", "snr_db", "noise_divisor", "oracle_agree", "oracle_ok"):
        if k in s:
            out[k] = _g(s[k]) if not isinstance(s[k], str) else s[k][:80]
    return out


def compact_line(full: dict, full_path=None) -> dict:
    """The one stdout line the driver parses: the contract's keys and the whole roofline /
    cpu_baseline objects (long prose cut), then one-number summaries of every other
    object; `full` (written beside, at full_path) keeps everything. Bounded to LINE_MAX
    bytes (tests/test_bench_line.py)."""
    out = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    if isinstance(full.get("config"), dict):
        out["config"] = dict(full["config"])
    if isinstance(full.get("roofline"), dict):
        rf = {k: v for k, v in full["roofline"].items() if k != "algorithmic_bytes_what"}
        rf["per_unit"] = full["roofline"].get("algorithmic_bytes_what", "")[:80]
        out["roofline"] = rf
    cb = full.get("cpu_baseline")
    if isinstance(cb, dict):
        c = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample", "single_core", "oracle_agree",
                                "js_agree_ok", "error") if k in cb}
        if "sample" in c:
            c["sample"] = str(c["sample"])[:240]
        if isinstance(cb.get("c_port"), dict):
            c["c_port_value"] = cb["c_port"].get("value")
        if isinstance(cb.get("calibration"), dict):
            c["js_over_modem_js"] = _g(cb["calibration"].get("js_over_modem_js"))
        out["cpu_baseline"] = c
    out.update(_pick(full, ["payload_MB_per_s", "frames_ok", "frames_exact_fallback", "devices"]))
    out.update(_pick(full, [("pipeline", ["contexts", "one_context_ms_per_step"]),
                            ("scan_roofline", ["kernel", "kernel_ms_avg", "frac"]),
                            ("graph", ["ms_per_step", "frames_ok", "error"]),
                            ("e2e", ["samples_per_s", "ms"]),
                            ("gather", ["frames", "ms", "GBps", "records_ok", "ranks_joined", "devices"]),
                            ("group", ["ms_per_step", "samples_per_s", "records_equal_per_rank", "frames_ok",
                                       "frames"])]))
    ch = full.get("chain")
    if isinstance(ch, dict):
        out["chain"] = {"ms_avg": _g(ch.get("ms_avg")), "frac": _g(ch.get("frac")),
                        "kernels_ms": {k: _g(v) for k, v in (ch.get("kernels_ms_avg") or {}).items()}}
    tx = full.get("tx")
    if isinstance(tx, dict):
        out["tx"] = {"kernel_ms_avg": _g(tx.get("kernel_ms_avg")),
                     "frac": _g((tx.get("roofline") or {}).get("frac"))}
    ha = full.get("host_api")
    if isinstance(ha, dict):
        h = {}
        if isinstance(ha.get("python_decode_host"), dict):
            h["python_ms"] = _g(ha["python_decode_host"].get("ms"))
        nb = ha.get("node_decode_batch")
        if isinstance(nb, dict):
            h["node_ms"] = _g(nb.get("ms")) if "ms" in nb else str(nb.get("error", ""))[:120]
            if isinstance(nb.get("resident"), dict):
                h["node_resident_ms"] = _g(nb["resident"].get("ms"))
        out["host_api"] = h
    st = full.get("stream")
    if isinstance(st, dict):
        s = _pick(st, ["samples_per_s", "payload_MB_per_s", "frames", "file_ok"])
        s["phases_ms"] = {k: _g(v) for k, v in (st.get("phases_ms") or {}).items()}
        dr = st.get("device_resident")
        if isinstance(dr, dict):
            s["device_resident"] = _pick(dr, ["samples_per_s", "file_ok", "host_share"])
            s["device_resident"]["phases_ms"] = {k: _g(v) for k, v in (dr.get("phases_ms") or {}).items()}
        out["stream"] = s
    legs = full.get("legs")
    if isinstance(legs, dict):
        L = {}
        for name, leg in legs.items():
            if name == "c1_latency" and isinstance(leg, dict):
                L[name] = {"python_ms": _g((leg.get("python_decode_received_signal") or {}).get("median_ms")),
                           "node_ms": _g((leg.get("node_decode_received_signal") or {}).get("median_ms")),
                           "cpu_js_ms": _g((leg.get("cpu_js_one_core") or {}).get("ms_per_call")),
                           "speedup_vs_cpu_js": _g(leg.get("speedup_vs_cpu_js"))}
            else:
                L[name] = _leg_summary(leg)
        out["legs"] = L
    if full_path:
        out["full"] = full_path
    line = json.dumps(out, separators=(",", ":"))
    if len(line) > LINE_MAX:  # (never expected: drop the summaries, keep the contract)
        for k in ("legs", "stream", "host_api", "group", "gather", "graph", "e2e", "scan_roofline", "tx"):
            out.pop(k, None)
            if len(json.dumps(out, separators=(",", ":"))) <= LINE_MAX:
                break
        out["truncated"] = True
    return out


def write_full(full: dict):
    """The whole result object beside the line: $AMOD_BENCH_FULL, else
    gpurun_out/bench_full.json under the run's tree. Returns the path (relative to the
    tree when inside it), or None when it could not be written."""
    path = os.environ.get("AMOD_BENCH_FULL") or os.path.join(ROOT, "gpurun_out", "bench_full.json")
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
    except OSError as e:
        print(f"bench.py: could not write {path}: {e}", file=sys.stderr)
        return None
    ap = os.path.abspath(path)
    return os.path.relpath(ap, ROOT) if ap.startswith(ROOT + os.sep) else ap


# --------------------------------------------------------------------- main --
def graph_leg(env: Env, wl: Workload, steps: int):
    """The same decode captured once into a hipGraph (amod_reserve was called; include/
    amodem.h) and replayed `steps` times: the step time without the per-launch host work
    (the dependent kernels' GPU-side gaps remain), on one context: compare it with
    pipeline.one_context_ms_per_step. (AMOD_BENCH_GRAPH_PIPE=1 captures each context's
    decode into its own graph and alternates the replays over the two streams, as the
    eager steps do: 0.456 ms per C2 step against 0.441 on one context and 0.425 eager
    pipelined. This runtime ran the two graphs' replays one after the other.) After the
    timed replays one replay's records are checked like the eager steps'."""
    torch = env.torch
    try:
        nctx = 2 if getattr(wl, "dm2", None) is not None and os.environ.get("AMOD_BENCH_GRAPH_PIPE") == "1" else 1
        graphs, streams = [], []
        torch.cuda.synchronize(env.dev)
        for k in range(nctx):
            g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream(env.dev)
            with torch.cuda.stream(s):
                wl.step_ctx(k, s.cuda_stream)  # (one eager decode on the capture stream first)
                s.synchronize()
                with torch.cuda.graph(g, stream=s):
                    wl.step_ctx(k, s.cuda_stream)
            graphs.append(g)
            streams.append(s)
        torch.cuda.synchronize(env.dev)
        it = [0]

        def replay():
            k = it[0] % nctx
            it[0] += 1
            with torch.cuda.stream(streams[k]):
                graphs[k].replay()

        warm_up(replay, lambda: torch.cuda.synchronize(env.dev), 5)  # (clocks, as for the eager steps)
        torch.cuda.synchronize(env.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            replay()
        torch.cuda.synchronize(env.dev)
        dt = (time.perf_counter() - t0) / steps
        wl.d_res.zero_()
        with torch.cuda.stream(streams[0]):
            graphs[0].replay()
        torch.cuda.synchronize(env.dev)
        rec = wl.records()
        ok = int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum())
        return {"what": "the decode captured into a hipGraph per context (%d), replays alternating over the "
                        "contexts' streams as the eager steps do (host launch work removed; the kernels' GPU-side "
                        "dependency gaps remain)" % nctx,
                "ms_per_step": dt * 1e3, "samples_per_s": wl.ndecoded / dt, "frames_ok": ok, "steps": steps,
                "contexts": nctx}
    except Exception as e:  # (reported, never fatal: the eager line above is the metric)
        return {"error": repr(e)[:300]}


def run_leg(env: Env, conf: str, args, frames=0, snr=20.0, primary=False):
    progress(f"{conf}: synthesising the batch")
    wl = Workload(env, conf, frames, snr)
    progress(f"{conf}: {wl.F} frames x {int(wl.dlens[0])} samples resident; measuring")
    extra = {}
    if primary and conf != "c4":
        extra["scan_roofline"] = scan_phase(env, wl)
    out, rec = measure(env, wl, args.steps, args.warmup)
    if primary and env.world == 1:  # right after the eager steps, while the clocks are up
        out["graph"] = graph_leg(env, wl, args.steps)
    out["tx"] = tx_obj(wl)
    if conf == "c5" and env.world == 1:
        progress(f"{conf}: soft combining vs the hard vote")
        out["soft_combine"] = soft_leg(env, wl, args.steps, args.warmup)
    if env.world > 1:
        out["gather"] = gather_leg(env, wl)
        if primary and env.rank == 0 and os.environ.get("AMOD_BENCH_GROUP", "1") != "0":
            progress(f"{conf}: group leg (rank 0 drives every device from one process)")
            out["group"] = group_leg(env, conf, args, snr, getattr(wl, "gathered", None))
        env.barrier()
    if primary and not args.no_e2e:
        out["e2e"] = e2e_leg(env, wl)
    # the host entries (Python amod_decode_host, Node decodeBatch) on the batches a host can
    # hold in one Float32Array comfortably (C3's 12 GB is device-path only)
    if not args.no_e2e and conf != "c3" and env.rank == 0 and env.world == 1:
        progress(f"{conf}: host API legs (amod_decode_host from Python, decodeBatch from Node)")
        out["host_api"] = host_api_leg(env, wl)
    if env.rank == 0 and env.world == 1 and args.cpu_frames >= 0:
        progress(f"{conf}: CPU legs (C oracle over the whole batch, JS baseline on worker_threads)")
        js_frames = args.cpu_frames or (640 if conf != "c5" else 192)
        out["cpu_baseline"] = cpu_legs(wl, rec, js_frames, js_seconds=1.5 if primary else 1.0)
    out.update(extra)
    wl.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: 10k QPSK 1 KB frames per GPU (the metric's config); c3: 100k 16-QAM 1 KB frames; "
                         "c4: 32k QPSK 2 KB data-chunk windows (decodeChunkFrame); c5: 10k acoustic BPSK rep3 "
                         "256 B frames + AWGN (--snr)")
    ap.add_argument("--legs", default="auto",
                    help="extra legs after the primary one: comma list of c3,c4,c5 (c5 at 10 dB), 'none'; "
                         "auto = c3,c4,c5 with --config c2")
    ap.add_argument("--snr", type=float, default=20.0, help="c5: AWGN SNR in dB (active-sample power)")
    ap.add_argument("--soft", action="store_true", help="(kept for old command lines: every c5 leg times "
                    "AMOD_OPT_SOFT_COMBINE against the hard vote)")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per GPU (0: the config's, C2 10,000 / C3 100,000 / C4 32,000)")
    ap.add_argument("--stream-chunks", type=int, default=-1,
                    help="C4-shaped stream for the streaming-receiver leg (0 = skip; default 32000 with c2)")
    ap.add_argument("--cpu-frames", type=int, default=0, help="CPU-baseline sample (0 = auto, -1 = skip)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive and host-API legs")
    args = ap.parse_args()

    backend = os.environ.get("AMOD_BENCH_BACKEND", "nccl")
    ndev = 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        import torch  # device_count does not initialise the GPU on this image
        ndev = torch.cuda.device_count()
    kind, val = launch_plan(args.gpus, dict(os.environ), ndev, backend)
    if kind == "error":
        print(f"bench.py: {val}", file=sys.stderr)
        sys.exit(2)
    if kind == "spawn":
        sys.exit(spawn_ranks(val, sys.argv[1:]))

    env = Env()
    if args.gpus > 1 and env.world != args.gpus and env.rank == 0:
        print(f"bench.py: --gpus {args.gpus} but {env.world} rank(s) joined; reporting n_gpus={env.world}",
              file=sys.stderr)
    if args.stream_chunks < 0:
        args.stream_chunks = 32000 if args.config == "c2" else 0
    legs = [] if args.legs == "none" else (
        (["c3", "c4", "c5"] if args.config == "c2" else []) if args.legs == "auto" else args.legs.split(","))
    # the streaming receiver first (its host phases idle the GPU; rank 0 only)
    if args.stream_chunks > 0 and env.rank == 0:
        progress(f"streaming receiver over {args.stream_chunks} chunks")
    stream_res = stream_leg(env, args.stream_chunks) if (args.stream_chunks > 0 and env.rank == 0) else None
    env.barrier()
    prim = run_leg(env, args.config, args, frames=args.frames, snr=args.snr, primary=True)
    lat = None
    if env.rank == 0 and env.world == 1 and not args.no_e2e:
        progress("c1_latency: one frame through the synchronous drop-in")
        lat = c1_latency_leg(env)
    extra = {}
    for lg in legs:
        name = lg if lg != "c5" else "c5_10db"
        extra[name] = run_leg(env, lg, args, snr=10.0 if lg == "c5" else args.snr)
    if "c5" in legs and env.world == 1:
        # soft combining at 7 dB, about the lowest SNR at which the reference still detects
        # the preambles (it fails at <= 6 dB)
        progress("c5 at 7 dB: soft combining vs the hard vote")
        wl7 = Workload(env, "c5", 0, 7.0)
        extra["c5_soft_7db"] = soft_leg(env, wl7, args.steps, args.warmup, oracle=True)
        wl7.close()
        progress("c5 chunk windows at 1.76 dB: soft combining vs the hard vote")
        extra["c5_soft_chunk"] = soft_chunk_leg(env, args)
    if env.rank == 0:
        out = {"metric": METRIC}
        out.update({k: prim[k] for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step")})
        out.update({"higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                    "data": "synthetic (reference-equivalent TX on the GPU, xorshift32 payloads)"})
        for k, v in prim.items():
            if k not in out:
                out[k] = v
        out["devices"] = env.devices_used
        out["stream"] = stream_res
        out["legs"] = extra
        if lat is not None:
            out["legs"]["c1_latency"] = lat
        path = write_full(out)
        print(json.dumps(compact_line(out, path), separators=(",", ":")), flush=True)
    if env.world > 1:
        env.dist.destroy_process_group()


if __name__ == "__main__":
    main()
