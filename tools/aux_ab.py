#!/usr/bin/env python3
"""Experiments only: interleaved A/B of context variants (AMOD_* knobs, read when a
context opens) on the bench workloads, in ONE process.

  python tools/aux_ab.py 'hi:AMOD_AUX_PRIORITY=1' 'lo:AMOD_AUX_PRIORITY=0' ...

Per workload (AB_CONFS, default c2,c4,c5 with c5 at 10 dB) every variant gets its own
context; rounds alternate between variants. Per variant: the median wall time of a
3-decode burst (host clock, synchronised; profiling off) and the median per-decode stage
times with profiling on (k_detect, k_demod, aux stream, chain), plus the overlap count."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    env = bench.Env()
    L, lib = env.L, env.lib
    confs = os.environ.get("AB_CONFS", "c2,c4,c5").split(",")
    rounds = int(os.environ.get("AB_ROUNDS", "12"))
    variants = []
    for spec in sys.argv[1:]:
        name, _, kv = spec.partition(":")
        variants.append((name, dict(p.split("=", 1) for p in kv.split(",") if p)))
    for conf in confs:
        wl = bench.Workload(env, conf, snr=10.0)
        runs = []
        for vname, kv in variants:
            old = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            h = C.c_void_p()
            L.check(lib.amod_open(env.local, C.byref(h)))
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            L.check(lib.amod_reserve(h, C.byref(wl.cfg), wl.F, int(wl.dlens.max())))

            def run(h=h, st=None):
                L.check(lib.amod_decode_device(h, C.byref(wl.cfg), wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(),
                                               wl.d_dlen.data_ptr(), wl.F, wl.d_res.data_ptr(), wl.d_pay.data_ptr(),
                                               wl.stride, 0, C.c_void_p(st if st is not None else wl.stream)))
            if os.environ.get("AB_GRAPH"):  # the decode captured once, replayed
                torch = env.torch
                gs = torch.cuda.Stream(env.dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(gs):
                    run(st=gs.cuda_stream)
                    gs.synchronize()
                    with torch.cuda.graph(g, stream=gs):
                        run(st=gs.cuda_stream)
                torch.cuda.synchronize(env.dev)
                keep = (g, gs)

                def run(g=g, keep=keep):
                    g.replay()
            runs.append((vname, h, run))
        for _ in range(40):
            for _, _, run in runs:
                run()
        env.torch.cuda.synchronize(env.dev)
        wall = {v: [] for v, *_ in runs}
        st = {v: [] for v, *_ in runs}
        ov = {v: [0, 0] for v, *_ in runs}
        for _ in range(rounds):
            for vname, h, run in runs:
                env.torch.cuda.synchronize(env.dev)
                t0 = time.perf_counter()
                for _ in range(3):
                    run()
                env.torch.cuda.synchronize(env.dev)
                wall[vname].append((time.perf_counter() - t0) / 3 * 1e3)
                lib.amod_set_profiling(h, 1)
                for _ in range(3):
                    run()
                kms, kn = (C.c_double * L.STAGE_COUNT)(), C.c_int64()
                lib.amod_kernel_stages(h, kms, L.STAGE_COUNT, C.byref(kn))
                lib.amod_set_profiling(h, 0)
                a, b, lead = C.c_int64(), C.c_int64(), C.c_double()
                lib.amod_aux_overlap(h, C.byref(a), C.byref(b), C.byref(lead))
                ov[vname][0] += a.value
                ov[vname][1] += b.value
                n = max(1, kn.value)
                st[vname].append([kms[L.STAGE_DETECT] / n, kms[L.STAGE_DEMOD] / n, kms[L.STAGE_AUX] / n,
                                  (kms[L.STAGE_DETECT] + kms[L.STAGE_DEMOD_PATH] + kms[L.STAGE_EXACT_B]) / n])
        for vname, *_ in runs:
            s = np.median(np.array(st[vname]), axis=0)
            print(f"{conf} {vname:10s} wall {np.median(wall[vname]):.4f} ms  detect {s[0]:.4f} demod {s[1]:.4f} "
                  f"aux {s[2]:.4f} chain {s[3]:.4f}  listed {ov[vname][0]} beside {ov[vname][1]}", flush=True)
        for _, h, _ in runs:
            lib.amod_close(h)
        wl.close()


if __name__ == "__main__":
    main()
