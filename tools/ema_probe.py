#!/usr/bin/env python3
"""Diagnostics: the streaming receiver's DC-removal pass (k_ema_*) on the bench's C4-shaped
stream, device-resident, with the warm-up length from AMOD_EMA_WARM: EMA time, chunks the
fix pass recomputed, and whether the assembled file is right.
  AMOD_EMA_WARM=4 python tools/ema_probe.py [nchunks]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32000
    env = bench.Env()
    amodem, L = env.amodem, env.L
    cfg = amodem.preset("standard", "QPSK", 1)
    data = amodem.synth_payload(0xC4000001, n * 2048 - 123)
    pk = [amodem.packet_meta(n, len(data), 2048, "c4.bin")] + \
         [amodem.packet_chunk(data[i * 2048:(i + 1) * 2048], i) for i in range(n)]
    dm = amodem.Demodulator(env.local)
    sig, _, _ = dm.transmit_batch(cfg, pk, [L.TX_META] + [L.TX_CHUNK] * n)
    total = -(-(len(sig) + 8192) // 4096) * 4096
    x = np.concatenate([sig, np.zeros(total - len(sig), np.float32)])
    dx = torch.from_numpy(x).to(env.dev)
    torch.cuda.synchronize()
    out = []
    for rep in range(3):
        asm = amodem.ChunkAssembler()
        t0 = time.perf_counter()
        frames, _, st = dm.stream_receive_device(cfg, dx.data_ptr(), len(x), asm)
        t = time.perf_counter() - t0
        out.append({"seconds": t, "t_ema_ms": st["t_ema_ms"], "fixed": st["ema_chunks_fixed"],
                    "t_fine_ms": st["t_fine_ms"], "t_host_ms": st["t_host_ms"], "t_decode_ms": st["t_decode_ms"],
                    "file_ok": asm.is_complete() and asm.assemble_file() == data, "frames": len(frames)})
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"warm": os.environ.get("AMOD_EMA_WARM", "16"), "chunks": n, "runs": out}))


if __name__ == "__main__":
    main()
