#!/usr/bin/env python3
"""bench.py — OFDM receive throughput on MI355X (BASELINE.json metric).

One step = one decodeReceivedSignal pass (preprocess, Schmidl-Cox scan, fine
timing, channel estimate, per-symbol FFT/equalise/demap, vote, pack, parse,
CRC-32) over the whole resident batch: BASELINE config C2, 10,000 QPSK frames of
35,874 samples (1 KB payload) per GPU, synthesised with the reference-equivalent
transmitter. Inputs are in HBM before the timed region. Frames are independent,
so ranks shard them (weak scaling, no data-path collective).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]
  (c4: decodeChunkFrame over 2 KB data-chunk windows, 32,000 per GPU = the 500 MB
  file of BASELINE C4 across 8 GPUs)
  (N > 1: torch.distributed.run, one process per GPU; RCCL for the barrier, the
  max-over-ranks time and, after the timed region, the gather of results into rank 0)
"""
import argparse
import ctypes as C
import json
import os
import sys
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
CHUNK = 2048                  # C4: data bytes per chunk frame


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: 10k QPSK 1 KB frames per GPU (the metric's config); c3: 100k 16-QAM 1 KB frames; "
                         "c4: 32k QPSK 2 KB data-chunk windows (decodeChunkFrame); c5: 10k acoustic BPSK rep3 "
                         "256 B frames + AWGN (--snr)")
    ap.add_argument("--snr", type=float, default=20.0, help="c5: AWGN SNR in dB (active-sample power)")
    ap.add_argument("--soft", action="store_true", help="c5: also decode once with AMOD_OPT_SOFT_COMBINE")
    ap.add_argument("--frames", type=int, default=0,
                    help="frames per GPU (0: the config's, C2 10,000 / C3 100,000 / C4 32,000)")
    ap.add_argument("--stream-chunks", type=int, default=-1,
                    help="C4-shaped stream for the streaming-receiver leg (0 = skip; default 2000 with c2)")
    ap.add_argument("--cpu-frames", type=int, default=0, help="CPU-baseline sample (0 = auto, -1 = skip)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive leg")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import amodem
    from amodem import _lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AMOD_BENCH_BACKEND=gloo rehearses the N > 1 flow with several ranks on one GPU
    # (RCCL refuses two ranks per device); the driver's runs use the default, RCCL
    backend = os.environ.get("AMOD_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    C3, C4, C5 = args.config == "c3", args.config == "c4", args.config == "c5"
    if args.stream_chunks < 0:
        args.stream_chunks = 2000 if args.config == "c2" else 0
    cfg = amodem.preset("acoustic", "BPSK", 3) if C5 else amodem.preset("standard", "QAM16" if C3 else "QPSK", 1)
    F = args.frames if args.frames > 0 else (100000 if C3 else (32000 if C4 else 10000))
    dm = amodem.Demodulator(local)
    # ---- synthetic input, built on the GPU by k_tx (the reference transmitter, bit-exact)
    # from the workload's packets; the timed region is device-resident
    if C4:
        # the file's chunks this rank owns: chunk seq = rank * F + i, bytes from xorshift32
        pre, post = amodem.tx_silence(cfg, L.TX_CHUNK)
        win = amodem.estimate_frame_samples(CHUNK + 11, "QPSK", 1)  # the receiver's window (app.js:853)
        spf = pre + win + post
        chunks = [amodem.synth_payload(0x9E3779B9 ^ (rank * F + i), CHUNK) for i in range(F)]
        pkts = [amodem.packet_chunk(chunks[i], rank * F + i) for i in range(F)]
        pl = np.array([len(p) for p in pkts], np.int32)
        po = np.concatenate([[0], np.cumsum(pl)[:-1]]).astype(np.int64)
        pk = np.frombuffer(b"".join(pkts), np.uint8).copy()
    else:
        plen = PAYLOAD_C5 if C5 else PAYLOAD
        pk, po, pl = amodem.synth_legacy_packets(F, plen, "f.bin", first=rank * F)
        pre, post = amodem.tx_silence(cfg, L.TX_LEGACY)
        spf = SAMPLES_PER_FRAME_C3 if C3 else (int(lib_frame_samples(amodem, L, cfg, int(pl[0]), pre, post)) if C5
                                               else SAMPLES_PER_FRAME)
    offs = (np.arange(F, dtype=np.int64) * spf)
    lens = np.full(F, spf, np.int32)
    nsamples = int(lens.sum())
    # what one step decodes: whole legacy frames, or the C4 windows (pre1 .. end of the
    # estimated frame, as StreamingReceiver cuts them) in decodeChunkFrame mode
    mode = L.MODE_CHUNK if C4 else L.MODE_RECEIVED
    doffs = offs + pre if C4 else offs
    dlens = np.full(F, win, np.int32) if C4 else lens
    ndecoded = int(dlens.sum())
    payload_bytes = CHUNK if C4 else (PAYLOAD_C5 if C5 else PAYLOAD)
    xs = torch.empty(nsamples + 16, dtype=torch.float32, device=dev)
    d_pk = torch.from_numpy(pk).to(dev)
    d_po, d_pl = torch.from_numpy(po).to(dev), torch.from_numpy(pl).to(dev)
    d_pre = torch.full((F,), pre, dtype=torch.int32, device=dev)
    d_post = torch.full((F,), post, dtype=torch.int32, device=dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_doff = torch.from_numpy(doffs).to(dev)
    d_dlen = torch.from_numpy(dlens).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    tx_stream = torch.cuda.Stream(dev)  # a real (non-null) stream, so events and kernel share it

    def tx():
        dm.transmit_device(cfg, d_pk.data_ptr(), d_po.data_ptr(), d_pl.data_ptr(), d_pre.data_ptr(),
                           d_post.data_ptr(), F, xs.data_ptr(), d_off.data_ptr(), stream=tx_stream.cuda_stream)

    torch.cuda.synchronize(dev)
    tx()
    tx_stream.synchronize()
    tx_ms = []
    for _ in range(5):  # k_tx timed with HIP events on its launch stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(tx_stream)
        tx()
        e1.record(tx_stream)
        e1.synchronize()
        tx_ms.append(e0.elapsed_time(e1))
    torch.cuda.synchronize(dev)
    tx_avg_ms = sum(tx_ms) / len(tx_ms)
    sigma = None
    if C5:  # AWGN on the GPU, seeded per rank; power from the first frame's active samples
        x0 = xs[: int(lens[0])]
        act = x0[x0 != 0]
        sigma = float(torch.sqrt((act.double() ** 2).mean() / 10 ** (args.snr / 10)).item())
        gen = torch.Generator(device=dev)
        gen.manual_seed(0xC5 + rank)
        xs[:nsamples] += torch.randn(nsamples, generator=gen, device=dev, dtype=torch.float32) * sigma
        torch.cuda.synchronize(dev)
    stride = amodem.payload_stride(cfg, int(dlens.max()))
    d_res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    d_pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)

    dm.reserve(cfg, F, int(dlens.max()))

    def step():
        dm.decode_device(cfg, mode, xs.data_ptr(), d_doff.data_ptr(), d_dlen.data_ptr(), F,
                         d_res.data_ptr(), d_pay.data_ptr(), stride, stream=stream)

    lib = L.load()
    stream_res = stream_leg(amodem, L, local, args.stream_chunks) if (args.stream_chunks > 0 and rank == 0) else None
    # correlation-scan phase alone (k_corr_scan), measured before the timed region
    # (decodeChunkFrame has no scan: the window starts at pre1)
    scan = None if C4 else scan_phase(amodem, L, lib, cfg, local, xs, d_doff, d_dlen, F, d_res, d_pay, stride,
                                      stream, spf)
    # the W untimed warm-up steps right before the timed ones (after the legs above, whose
    # host phases leave the GPU idle)
    for _ in range(args.warmup):
        step()
    lib.amod_set_profiling(dm.ctx, 1)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    kms, kn = (C.c_double * 3)(), C.c_int64()
    lib.amod_kernel_breakdown(dm.ctx, kms, C.byref(kn))
    lib.amod_set_profiling(dm.ctx, 0)
    stage_ms = [kms[i] / max(1, kn.value) for i in range(3)]  # per decode: detect, demod, exact
    # correctness of what was timed (the last timed step's results): every frame decodes, CRC valid,
    # payload exact
    rec = np.frombuffer(d_res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
    ok = int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum())
    fallback = int((rec["flags"] != 0).sum())
    fallback_flags = {}
    for fl in rec["flags"][rec["flags"] != 0]:
        for b in range(16):
            if int(fl) & (1 << b) and b != 15:
                fallback_flags[FLAG_NAMES.get(b, str(b))] = fallback_flags.get(FLAG_NAMES.get(b, str(b)), 0) + 1
    if os.environ.get("AMOD_STAMPS"):  # diagnostics: exact-kernel phase marks of the listed frames
        st = np.zeros(F * 32, dtype=np.uint64)
        n = L.load().amod_debug_stamps(dm.ctx, st.ctypes.data, st.size)
        st = st[:n].reshape(-1, 32).astype(np.int64)
        for i in np.nonzero(rec["flags"] & (L.FLAG_EXACT | L.FLAG_REPLAY))[0][:32]:
            print("listed", i, hex(int(rec["flags"][i])), int(rec["coarse_idx"][i]),
                  [int(st[i, b] - st[i, a]) if st[i, a] and st[i, b] else None
                   for a, b in ((8, 13), (13, 14), (14, 9), (9, 10), (10, 11), (11, 12))], file=sys.stderr)
    pay = d_pay.view(F, stride).cpu().numpy()
    for i in range(0, F, max(1, F // 16)):
        r = amodem.to_reference(rec[i], pay[i].tobytes(), not C4)
        if C5 and not r.get("crcValid"):
            continue  # noisy frames: checked against the oracle in the cpu_baseline leg
        assert r.get("data") == amodem.synth_payload(0x9E3779B9 ^ (rank * F + i), payload_bytes), (i, r.get("error"))
        if C4:
            assert r.get("seqNum") == rank * F + i, (i, r.get("seqNum"))

    e2e = None
    if not args.no_e2e:
        e2e = e2e_leg(torch, dm, cfg, mode, xs, nsamples, d_doff, d_dlen, F, d_res, d_pay, stride, dev, ndecoded,
                      payload_bytes)

    gather = None
    if world > 1:
        gather = gather_leg(amodem, dist, torch, dev, rank, world, F, stride, d_res, d_pay, C4, payload_bytes)

    t = torch.tensor([elapsed, float(ok), float(fallback)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        ok, fallback = int(tsum[0].item()), int(tsum[1].item())

    if rank == 0:
        total_samples = ndecoded * world * args.steps
        value = total_samples / elapsed
        payload_mbps = payload_bytes * F * world * args.steps / elapsed / 1e6
        algo_bytes = 4.0 * ndecoded  # each float32 sample read once
        chain_s = sum(stage_ms[:2]) / 1e3
        names = ["k_chunk_prep" if C4 else "k_detect", "k_demod"]
        dom = max(range(2), key=lambda i: stage_ms[i])
        # the dominant launch's algorithmic bytes: k_detect reads every sample once; k_demod
        # reads the 512-sample FFT window of the CE and of every demodulated data symbol
        spf_dec = int(dlens[0])
        if dom == 0:
            dom_bytes = algo_bytes
        else:  # CE + the symbols holding the packet (trailing silence skipped)
            per_sym = amodem.num_data_subs(cfg) * {0: 1, 1: 2, 2: 4}[cfg.modulation]
            nsym_dec = -(-int(pl[0]) * 8 * cfg.repetition // per_sym)
            dom_bytes = 4.0 * 512 * (nsym_dec + 1) * F
        achieved = dom_bytes / (stage_ms[dom] / 1e3) / 1e9
        traffic = None
        # HBM bytes per launch of the dominant kernel from the committed PMC pass
        # (FETCH_SIZE x 2 + WRITE_SIZE, tools/traffic.py) when it was taken on this workload
        tf = os.path.join(ROOT, "profiles", "r02", "traffic.json")
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            kt = tj.get("kernels", {}).get(names[dom])
            if tj.get("frames") == F and tj.get("samples_per_frame") == spf and kt:
                traffic = (kt["read_bytes"] + kt["write_bytes"]) / kt.get("dispatches_per_step", 1.0)
        mod = "QAM16" if C3 else ("BPSK" if C5 else "QPSK")
        name = "C3" if C3 else ("C4" if C4 else ("C5" if C5 else "C2"))
        cpu, tx_cpu, d2h = None, None, None
        if args.cpu_frames >= 0:
            # the CPU legs need the samples on the host: copy back the sample's frames
            per_thread = 100 if C5 else 1000
            ncpu = args.cpu_frames if args.cpu_frames > 0 else min(F, per_thread * min(16, os.cpu_count() or 1))
            t0 = time.perf_counter()
            xh = xs[: ncpu * spf].cpu().numpy()
            d2h = 4.0 * ncpu * spf / (time.perf_counter() - t0) / 1e9
            cpu = cpu_baseline(xh, doffs[:ncpu], dlens[:ncpu], mod, name, chunk=C4, payload=payload_bytes,
                               preset="acoustic" if C5 else "standard", rep=cfg.repetition, gpu_rec=rec[:ncpu])
            tx_cpu = None if C4 else tx_cpu_baseline(amodem, cfg, min(ncpu, 4000), spf, payload_bytes)
        tx_bytes = 4.0 * nsamples + float(pl.sum())  # samples written + packet bytes read
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference-equivalent TX, xorshift32 payloads)",
            "config": {"workload": ("C4: 32k QPSK 2 KB data-chunk windows per GPU (decodeChunkFrame; value counts "
                                    "the window samples decoded, 25,344 of each 28,431-sample frame)" if C4 else
                                    ("C5: 10k acoustic BPSK rep3 256 B legacy frames per GPU + AWGN at %.0f dB "
                                     "(decodeReceivedSignal, hard majority vote = reference behaviour)" % args.snr
                                     if C5 else
                                     ("C3: 100k-frame 16-QAM batch demod per GPU" if C3 else
                                      "C2: 10k-frame QPSK batch demod per GPU") +
                                     " (decodeReceivedSignal, legacy 1 KB frames)")),
                       "frames_per_gpu": F, "samples_per_frame": int(dlens[0]), "fft": 512,
                       "modulation": mod, "payload_bytes": payload_bytes, "parallelism": f"frame-sharded x{world}"},
            "payload_MB_per_s": payload_mbps,
            "frames_ok": ok,
            "frames_exact_fallback": fallback,
            "fallback_flags": fallback_flags,
            "awgn_sigma": sigma,
            "d2h_GBps": d2h,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": names[dom], "kernel_ms_avg": stage_ms[dom],
                         "algorithmic_bytes": dom_bytes},
            "chain": {"what": "the whole fast path per step (%s -> k_demod), HIP events on "
                              "the launch stream; algorithmic bytes = 4 B x every decoded sample" % names[0],
                      "ms_avg": chain_s * 1e3, "achieved": algo_bytes / chain_s / 1e9, "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": algo_bytes / chain_s / 1e9 / HBM_PEAK_GBS,
                      "kernels_ms_avg": dict(zip(names + ["k_decode_exact"], stage_ms)),
                      "symbols_demodulated_per_frame": "header..CRC symbols only (C2: 21 of 36; trailing "
                                                       "silence skipped, SURVEY.md 8d)" if not C4 else "all"},
            "soft_combine": soft_leg(amodem, L, dm, cfg, mode, xs, d_doff, d_dlen, F, d_res, d_pay, stride, stream,
                                     rec) if (C5 and args.soft) else None,
            "cpu_baseline": cpu,
            "scan_roofline": None if scan is None else {
                "phase": "stream pass + Schmidl-Cox coarse search ("
                         "k_corr_scan: the same code compiled to stop there, results not written; 20 launches)",
                "kernel": "k_corr_scan", "kernel_ms_avg": scan, "achieved": algo_bytes / (scan / 1e3) / 1e9,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": algo_bytes / (scan / 1e3) / 1e9 / HBM_PEAK_GBS},
            "tx": {"kernel": "k_tx", "what": "GPU transmitter (modulateOFDM + buildTransmitSignal, bit-exact) "
                                             "building this run's input", "kernel_ms_avg": tx_avg_ms,
                   "samples_per_s": nsamples / (tx_avg_ms / 1e3),
                   "roofline": {"bound": "hbm", "achieved": tx_bytes / (tx_avg_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": tx_bytes / (tx_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS},
                   "cpu_baseline": tx_cpu},
            "stream": stream_res,
            "e2e": e2e,
            "gather": gather,
        }
        print(json.dumps(out), flush=True)
    dm.close()
    if world > 1:
        dist.destroy_process_group()


FLAG_NAMES = {0: "FORCED", 1: "NONFINITE", 2: "BIG", 3: "COARSE", 4: "FINE", 5: "CHANNEL", 6: "PHASE", 7: "DEMAP",
              8: "THRESH", 9: "SPAN", 10: "SOFT", 11: "REPLAY"}
PAYLOAD_C5 = 256


def lib_frame_samples(amodem, L, cfg, pkt_len, pre, post):
    import ctypes as C
    return L.load().amod_tx_frame_samples(C.byref(cfg), pkt_len, pre, post)


def soft_leg(amodem, L, dm, cfg, mode, xs, d_off, d_len, F, d_res, d_pay, stride, stream, hard_rec):
    """C5's opt-in soft combining of the repeated bits (AMOD_OPT_SOFT_COMBINE, NOT reference
    behaviour: the exact kernel demodulates after the fast detection), one timed pass."""
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dm.decode_device(cfg, mode, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F, d_res.data_ptr(),
                     d_pay.data_ptr(), stride, stream=stream, options=L.OPT_SOFT_COMBINE)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    rec = np.frombuffer(d_res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
    ok_soft = int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum())
    ok_hard = int(((hard_rec["status"] == 0) & (hard_rec["crc_valid"] == 1)).sum())
    return {"what": "AMOD_OPT_SOFT_COMBINE (|H|^2-weighted soft vote; not reference behaviour)", "ms": t * 1e3,
            "frames_crc_valid_soft": ok_soft, "frames_crc_valid_hard": ok_hard}


def e2e_leg(torch, dm, cfg, mode, xs, nsamples, d_off, d_len, F, d_res, d_pay, stride, dev, ndecoded, payload_bytes,
            reps=3):
    """Host-resident batch, PCIe included (BASELINE.md "two timing modes"): the samples
    in pinned host memory, copied H2D, decoded, result records and payload slots copied
    back to pinned memory, on one stream; wall time per pass (never `value`)."""
    h_x = torch.empty(nsamples, dtype=torch.float32, pin_memory=True)
    h_x.copy_(xs[:nsamples])
    h_res = torch.empty(d_res.numel(), dtype=torch.uint8, pin_memory=True)
    h_pay = torch.empty(d_pay.numel(), dtype=torch.uint8, pin_memory=True)
    st = torch.cuda.Stream(dev)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            xs[:nsamples].copy_(h_x, non_blocking=True)
            dm.decode_device(cfg, mode, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F, d_res.data_ptr(),
                             d_pay.data_ptr(), stride, stream=st.cuda_stream)
            h_res.copy_(d_res, non_blocking=True)
            h_pay.copy_(d_pay, non_blocking=True)
        st.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    return {"what": "pinned host samples -> H2D -> decode -> D2H records + payload, one stream, median of %d" % reps,
            "samples_per_s": ndecoded / t, "payload_MB_per_s": payload_bytes * F / t / 1e6, "ms": t * 1e3,
            "h2d_GBps": 4.0 * nsamples / t / 1e9}


def gather_leg(amodem, dist, torch, dev, rank, world, F, stride, d_res, d_pay, chunk_mode, payload_bytes, reps=3):
    """N > 1, after the timed region: the device-resident result records (96 B/frame)
    and payload slots of every rank gathered into rank 0 over RCCL (SURVEY.md §8e,
    BASELINE C4's "RCCL gather over xGMI"), timed with barrier + synchronize on both
    sides, then every gathered record checked on rank 0 (status, CRC, and for C4 the
    file's sequence numbers 0 .. world*F-1 in rank order)."""
    from amodem.shard import gather_to_root

    counts = [F] * world
    res_rows = d_res.view(F, 96)
    pay_rows = d_pay.view(F, stride)[:, : min(stride, payload_bytes + 64)].contiguous()  # data bytes + header slack
    ms = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g_res = gather_to_root(res_rows, counts, dst=0)
        g_pay = gather_to_root(pay_rows, counts, dst=0)
        torch.cuda.synchronize(dev)
        ms.append((time.perf_counter() - t0) * 1e3)
    tmax = torch.tensor([max(ms[1:]) if len(ms) > 1 else ms[0]], dtype=torch.float64, device=dev)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    if rank != 0:
        return None
    rec = np.frombuffer(g_res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
    pay = g_pay.cpu().numpy()
    ok = bool(((rec["status"] == 0) & (rec["crc_valid"] == 1)).all()) and len(rec) == world * F
    if chunk_mode:
        ok = ok and bool((rec["seq_num"] == np.arange(world * F)).all())
    for i in range(0, world * F, max(1, world * F // 64)):  # payload rows follow their records
        r = amodem.to_reference(rec[i], pay[i].tobytes(), not chunk_mode)
        ok = ok and r.get("data") == amodem.synth_payload(0x9E3779B9 ^ i, payload_bytes)
    nbytes = (res_rows.numel() + pay_rows.numel()) * (world - 1)  # what crosses xGMI into rank 0
    t = float(tmax.item())
    return {"what": "result records + payload slots of every rank gathered into rank 0 (%s gather)"
                    % ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend()),
            "frames": world * F, "bytes_into_root": nbytes, "ms": t, "GBps": nbytes / (t / 1e3) / 1e9,
            "records_ok": ok}


def scan_phase(amodem, L, lib, cfg, local, xs, d_off, d_len, F, d_res, d_pay, stride, stream, spf, reps=20):
    """Average duration of the correlation-scan phase alone on the same resident batch:
    k_corr_scan, the fast kernel's code instantiated to stop after the Schmidl-Cox
    decision (selected by AMOD_STOP_AFTER=1, read when a context builds its tables),
    launched with the same LDS footprint so the same number of frames share a CU."""
    os.environ["AMOD_STOP_AFTER"] = "1"
    try:
        dm = amodem.Demodulator(local)
        dm.reserve(cfg, F, spf)
        run = lambda: dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                                       d_res.data_ptr(), d_pay.data_ptr(), stride, stream=stream)
        for _ in range(10):  # clocks settle over the first launches
            run()
        dm.synchronize()
        lib.amod_set_profiling(dm.ctx, 1)
        for _ in range(reps):  # back to back, like the timed region
            run()
        fm, fn, em, en = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        lib.amod_kernel_times(dm.ctx, C.byref(fm), C.byref(fn), C.byref(em), C.byref(en))
        dm.close()
        return fm.value / max(1, fn.value)
    finally:
        del os.environ["AMOD_STOP_AFTER"]


def stream_leg(amodem, L, device, nchunks=2000, chunk=2048):
    """StreamingReceiver over a C4-shaped stream (metadata + nchunks 2 KB QPSK chunk
    frames back to back, built by k_tx): whole-call time from host samples to the
    assembled file, with the receiver's own phase split."""
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0xC4000001, nchunks * chunk - 123)
    pk = [amodem.packet_meta(nchunks, len(data), chunk, "c4.bin")]
    pk += [amodem.packet_chunk(data[i * chunk:(i + 1) * chunk], i) for i in range(nchunks)]
    dm = amodem.Demodulator(device)
    sig, _, _ = dm.transmit_batch(cfg, pk, [L.TX_META] + [L.TX_CHUNK] * nchunks)
    total = -(-(len(sig) + 8192) // 4096) * 4096
    x = np.concatenate([sig, np.zeros(total - len(sig), np.float32)])
    asm = amodem.ChunkAssembler()
    dm.stream_receive(cfg, x[: 64 * 4096], amodem.ChunkAssembler())  # warm-up (tables, kernels)
    t0 = time.perf_counter()
    frames, _, st = dm.stream_receive(cfg, x, asm)
    t = time.perf_counter() - t0
    ok = asm.is_complete() and asm.assemble_file() == data
    # the same stream already resident in HBM (amod_stream_receive_device)
    import torch
    dx = torch.from_numpy(x).to(torch.device("cuda", device))
    torch.cuda.synchronize()
    asm2 = amodem.ChunkAssembler()
    t0 = time.perf_counter()
    frames2, _, st2 = dm.stream_receive_device(cfg, dx.data_ptr(), len(x), asm2)
    t2 = time.perf_counter() - t0
    ok2 = asm2.is_complete() and asm2.assemble_file() == data and len(frames2) == len(frames)
    dm.close()
    return {"what": "app.js StreamingReceiver restated (amod_stream_receive): host samples in, frames + assembled file out",
            "workload": f"C4-shaped stream, metadata + {nchunks} x 2 KB QPSK chunk frames ({len(x)} samples)",
            "samples_per_s": len(x) / t, "payload_MB_per_s": len(data) / t / 1e6, "seconds": t,
            "frames": int(len(frames)), "file_ok": bool(ok),
            "phases_ms": {"ema_gpu": st["t_ema_ms"], "screen_fine_gpu": st["t_fine_ms"], "decode_gpu": st["t_decode_ms"],
                          "state_machine_host": st["t_host_ms"], "total": st["t_total_ms"]},
            "device_resident": {"samples_per_s": len(x) / t2, "seconds": t2, "file_ok": bool(ok2),
                                "phases_ms": {"ema_gpu": st2["t_ema_ms"], "screen_fine_gpu": st2["t_fine_ms"],
                                              "decode_gpu": st2["t_decode_ms"], "state_machine_host": st2["t_host_ms"],
                                              "total": st2["t_total_ms"]}},
            "reference_rate_note": "reference StreamingReceiver: 2.0e6 samples/s per core (SURVEY.md section 3.2)"}


def cpu_baseline(x, offs, lens, mod, name, chunk=False, payload=PAYLOAD, preset="standard", rep=1, gpu_rec=None):
    """The C restatement of the reference RX (oracle/, kind 'port') on this host's cores
    over a bounded sample of the same frames: all cores (16 threads, repeated to ~1 s of
    wall time, ~16 s of CPU work) and one core (~2 s). profiles/cpu_calibration.json
    (tools/calibrate_cpu.py, build container) holds the measured speed ratio of this port
    to the reference modem.js on one core; dividing by it gives the modem.js-equivalent
    rates reported beside the port's own."""
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    c = O.cfg(preset)
    t, reps = 0.0, 0
    agree = None
    while t < 1.0 and reps < 8:
        dt, st, crc = O.bench_decode(c, x, offs, lens, mod, rep, threads, chunk=chunk)
        if gpu_rec is None:
            assert (st == 0).all()
        else:  # noisy frames: the GPU's outcomes must be the reference's (the oracle's)
            agree = int(((gpu_rec["status"] == st) & ((st != 0) | (gpu_rec["actual_crc"] == crc))).sum())
        t += dt
        reps += 1
    samples = float(lens.sum()) * reps
    n1 = min(len(offs), 1000 if rep == 1 else 160)  # one core: ~2 s
    t1, st, _ = O.bench_decode(c, x, offs[:n1], lens[:n1], mod, rep, 1, chunk=chunk)
    assert gpu_rec is not None or (st == 0).all()
    single = float(lens[:n1].sum()) / t1
    out = {"value": samples / t, "unit": "samples/s", "cores": threads, "kind": "port",
           "sample": f"{len(offs)} {name} frames x {reps} passes ({int(samples)} samples) on {threads} threads; "
                     f"{n1} frames on 1 thread; oracle/amodem_oracle.c{' (decodeChunkFrame)' if chunk else ''}",
           "payload_MB_per_s": payload * len(offs) * reps / t / 1e6, "seconds": t + t1,
           "single_core": single}
    if agree is not None:
        out["oracle_agree"] = f"{agree}/{len(offs)} frames: GPU status and CRC equal the C oracle's"
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    key = {"C2": "c2", "C3": "c3", "C4": "c4", "C5": "c5"}.get(name)
    if os.path.exists(cal) and key:
        with open(cal) as f:
            r = json.load(f)["workloads"][key]["ratio_oracle_over_modem_js"]
        out["port_over_modem_js"] = r
        out["modem_js_equivalent"] = {"single_core": single / r, "all_cores": samples / t / r,
                                      "note": "port rates / the port-to-modem.js ratio measured in the build "
                                              "container (profiles/cpu_calibration.json)"}
    return out


def tx_cpu_baseline(amodem, cfg, nframes, spf, payload=PAYLOAD):
    """The host C++ builders (libamodem's amod_synth_legacy_batch, the same arithmetic
    as the reference TX) on this host's cores over nframes frames."""
    threads = min(16, os.cpu_count() or 1)
    out = np.empty(nframes * spf, np.float32)
    t0 = time.perf_counter()
    amodem.synth_legacy_batch(cfg, nframes, payload_len=payload, name="f.bin", threads=threads, out=out)
    t = time.perf_counter() - t0
    return {"value": nframes * spf / t, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{nframes} frames, libamodem host builders, {threads} threads", "seconds": t}


if __name__ == "__main__":
    main()
