#!/usr/bin/env python3
"""Diagnostics: k_detect / k_demod times on the C2 workload for several k_demod grid
sizes (AMOD_DEMOD_BPC = blocks per CU; unset = the occupancy query)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    import torch
    import amodem
    from amodem import _lib as L
    F = int(os.environ.get("FRAMES", "10000"))
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, F, threads=16)
    dev = torch.device("cuda", 0)
    xs = torch.empty(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off, d_len = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
    stride = amodem.payload_stride(cfg, int(lens.max()))
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    lib = L.load()
    for bpc in os.environ.get("BPCS", "0,1,2,3,4,5,6,8").split(","):
        if bpc == "0":
            os.environ.pop("AMOD_DEMOD_BPC", None)
        else:
            os.environ["AMOD_DEMOD_BPC"] = bpc
        dm = amodem.Demodulator(0)
        dm.reserve(cfg, F, int(lens.max()))
        run = lambda: dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                                       res.data_ptr(), pay.data_ptr(), stride)
        os.environ["AMOD_DEMOD_DIAG"] = "1"
        run()
        os.environ.pop("AMOD_DEMOD_DIAG")
        dm.synchronize()
        rec = amodem.RESULT_DTYPE
        import numpy as np
        r = np.frombuffer(res.cpu().numpy().tobytes(), rec)
        ok = int(((r["status"] == 0) & (r["crc_valid"] == 1)).sum())
        lib.amod_set_profiling(dm.ctx, 1)
        for _ in range(10):
            run()
        ms, n = (C.c_double * 3)(), C.c_int64()
        lib.amod_kernel_breakdown(dm.ctx, ms, C.byref(n))
        print(f"bpc={bpc:>2}  detect {ms[0] / n.value:.4f} ms  demod {ms[1] / n.value:.4f} ms  exact {ms[2] / n.value:.4f}"
              f"  ok {ok}/{F}", flush=True)
        dm.close()


if __name__ == "__main__":
    main()
