#!/usr/bin/env python3
"""Experiments only: interleaved A/B of libamodem.so builds on bench workloads, per stage.

  python tools/ab_demod.py LIB_A LIB_B [...]      (AB_CONFS=c2,c4 by default)

The inputs come from bench.Workload (k_tx on the GPU, device-resident); every library
gets its own context per workload and the launch rounds alternate between libraries
(A B A B ...), so clock drift hits every variant alike. Prints per variant and workload
the median k_detect / k_demod / chain time (amod_kernel_stages, HIP events) and whether
the last decode's records are all OK (AB_CHECK=0 skips the check: diagnostic builds
that remove work produce wrong results on purpose)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    env = bench.Env()
    L, amodem = env.L, env.amodem
    confs = os.environ.get("AB_CONFS", "c2,c4").split(",")
    rounds = int(os.environ.get("AB_ROUNDS", "12"))
    check = os.environ.get("AB_CHECK", "1") != "0"
    libs = []
    for path in sys.argv[1:]:
        lib = C.CDLL(os.path.abspath(path))
        for name, (rt, args) in L.SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = rt, args
        libs.append((os.path.basename(os.path.dirname(os.path.abspath(path))), lib))
    for conf in confs:
        wl = bench.Workload(env, conf, snr=10.0)
        runs = []
        for vname, lib in libs:
            h = C.c_void_p()
            L.check(lib.amod_open(env.local, C.byref(h)))
            L.check(lib.amod_reserve(h, C.byref(wl.cfg), wl.F, int(wl.dlens.max())))

            def run(lib=lib, h=h):
                L.check(lib.amod_decode_device(h, C.byref(wl.cfg), wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(),
                                               wl.d_dlen.data_ptr(), wl.F, wl.d_res.data_ptr(), wl.d_pay.data_ptr(),
                                               wl.stride, 0, C.c_void_p(wl.stream)))
            runs.append((vname, lib, h, run))
        for _ in range(30):  # warm-up (clock ramp)
            for _, _, _, run in runs:
                run()
        env.torch.cuda.synchronize(env.dev)
        t = {v: [] for v, *_ in runs}
        ok = {}
        for _ in range(rounds):
            for vname, lib, h, run in runs:
                lib.amod_set_profiling(h, 1)
                for _ in range(3):
                    run()
                kms, kn = (C.c_double * L.STAGE_COUNT)(), C.c_int64()
                lib.amod_kernel_stages(h, kms, L.STAGE_COUNT, C.byref(kn))
                lib.amod_set_profiling(h, 0)
                st = [kms[i] / max(1, kn.value) for i in range(L.STAGE_COUNT)]
                t[vname].append((st[L.STAGE_DETECT], st[L.STAGE_DEMOD],
                                 st[L.STAGE_DETECT] + st[L.STAGE_DEMOD_PATH] + st[L.STAGE_EXACT_B]))
                if check and vname not in ok:
                    env.torch.cuda.synchronize(env.dev)
                    rec = wl.records()
                    ok[vname] = int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum())
        for vname, *_ in runs:
            a = np.median(np.array(t[vname]), axis=0)
            print(f"{conf} {vname:24s} detect {a[0]:.4f}  demod {a[1]:.4f}  chain {a[2]:.4f} ms"
                  + (f"  ok {ok[vname]}/{wl.F}" if check else ""), flush=True)
        for _, lib, h, _ in runs:
            lib.amod_close(h)
        wl.close()


if __name__ == "__main__":
    main()
