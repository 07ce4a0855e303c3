#!/usr/bin/env python3
"""Experiments only: consecutive batches pipelined over two contexts (each its own
workspace, result buffers and stream) against one context, on bench workloads. A batch
is the same resident input every step; step i goes to context i % 2 on that context's
stream, so batch i + 1's k_detect can start while batch i's k_demod runs (the two
kernels' tails and the dependent-launch gaps overlap). Modes: one (one context), two
(two torch streams, no events), pipe_slot / pipe_cur (the library's amod_pipe_* on its slot
streams / ordered after torch's current stream), ev_pipe (the pipe's event
protocol by hand on torch streams). Prints ms per step for each mode,
medians of AB_ROUNDS rounds of AB_STEPS steps, interleaved, and checks every record.
  AB_CONFS=c2,c4,c5 python tools/pipeline_ab.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    env = bench.Env()
    torch, amodem = env.torch, env.amodem
    confs = os.environ.get("AB_CONFS", "c2,c4,c5").split(",")
    rounds = int(os.environ.get("AB_ROUNDS", "10"))
    steps = int(os.environ.get("AB_STEPS", "20"))
    for conf in confs:
        wl = bench.Workload(env, conf, snr=10.0)
        dm2 = amodem.Demodulator(env.local)
        dm2.reserve(wl.cfg, wl.F, int(wl.dlens.max()))
        s1 = torch.cuda.Stream(env.dev)
        s2 = torch.cuda.Stream(env.dev)
        res2 = torch.zeros_like(wl.d_res)
        pay2 = torch.zeros_like(wl.d_pay)

        def dec(dm, res, pay, st):
            dm.decode_device(wl.cfg, wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(), wl.d_dlen.data_ptr(), wl.F,
                             res.data_ptr(), pay.data_ptr(), wl.stride, stream=st.cuda_stream)

        def one(n):
            for _ in range(n):
                dec(wl.dm, wl.d_res, wl.d_pay, s1)

        def two(n):
            for i in range(n):
                if i % 2 == 0:
                    dec(wl.dm, wl.d_res, wl.d_pay, s1)
                else:
                    dec(dm2, res2, pay2, s2)

        # the library's pipe (amod_pipe_*): S = the current stream / the pipe's own stream
        pipe = wl.dm.pipeline(dm2)
        cur = torch.cuda.current_stream(env.dev).cuda_stream
        ring = [(wl.d_res, wl.d_pay), (res2, pay2)]

        def lib_pipe(n, s):
            for i in range(n):
                r, p = ring[i % 2]
                pipe.decode_device(wl.cfg, wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(), wl.d_dlen.data_ptr(),
                                   wl.F, r.data_ptr(), p.data_ptr(), wl.stride, stream=s)
            pipe.flush(s)

        # the pipe's protocol by hand on torch streams and events (S = the current stream)
        ev_in = torch.cuda.Event()
        ev_done = [torch.cuda.Event(), torch.cuda.Event()]

        def ev_pipe(n):
            S = torch.cuda.current_stream(env.dev)
            for i in range(n):
                k = i % 2
                ev_in.record(S)
                (s1 if k == 0 else s2).wait_event(ev_in)
                dec(wl.dm if k == 0 else dm2, *ring[k], s1 if k == 0 else s2)
                ev_done[k].record(s1 if k == 0 else s2)
                if i > 0:
                    S.wait_event(ev_done[k ^ 1])
            S.wait_event(ev_done[(n - 1) % 2])

        modes = (("one", one), ("two", two), ("pipe_slot", lambda n: lib_pipe(n, 0)),
                 ("pipe_cur", lambda n: lib_pipe(n, cur)), ("ev_pipe", ev_pipe))
        for _, f in modes:  # warm-up (clock ramp)
            for _ in range(30):
                f(2)
        torch.cuda.synchronize(env.dev)
        t = {m: [] for m, _ in modes}
        for _ in range(rounds):
            for name, f in modes:
                torch.cuda.synchronize(env.dev)
                t0 = time.perf_counter()
                f(steps)
                torch.cuda.synchronize(env.dev)
                t[name].append((time.perf_counter() - t0) / steps * 1e3)
        ok = []
        for res in (wl.d_res, res2):
            rec = np.frombuffer(res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
            ok.append(int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum()))
        print(f"{conf} " + "  ".join(f"{m} {np.median(v):.4f}" for m, v in t.items()) +
              f" ms/step   ok {ok[0]}/{ok[1]} of {wl.F}", flush=True)
        pipe.close()
        dm2.close()
        wl.close()


if __name__ == "__main__":
    main()
