"""Experiments only: the same resident batch decoded repeatedly on two contexts (as the
bench's pipelined steps do); prints the frames whose records or payload rows differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import bench
    env = bench.Env()
    conf = sys.argv[1] if len(sys.argv) > 1 else "c5"
    snr = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    opts = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    wl = bench.Workload(env, conf, 0, snr)
    wl.enable_pipeline()
    torch = env.torch
    outs = []
    watch = [int(v) for v in os.environ.get("DET_WATCH", "").split(",") if v]
    def show(tag, res):
        if not watch:
            return
        r = np.frombuffer(res.cpu().numpy().tobytes(), env.amodem.RESULT_DTYPE)
        print(tag, [(i, hex(int(r["flags"][i])), int(r["payload_valid"][i]), int(r["status"][i])) for i in watch],
              flush=True)
    if os.environ.get("DET_PROF"):  # the bench's serial steps first: profiled, on dm alone
        env.lib.amod_set_profiling(wl.dm.ctx, int(os.environ.get("DET_PROFILING", "1")))
        for k in range(int(os.environ["DET_PROF"])):
            wl.step()
            torch.cuda.synchronize()
            show(f"serial {k}", wl.d_res)
        env.lib.amod_set_profiling(wl.dm.ctx, 0)
    if os.environ.get("DET_SHOWPIPE"):
        for k in range(8):
            wl.step_pipelined()
            torch.cuda.synchronize()
            show(f"pipe {k}", wl.d_res if k % 2 == 0 else wl.d_res2)
    if os.environ.get("DET_PIPE"):  # the bench's pipelined steps (both contexts concurrently)
        for _ in range(int(os.environ["DET_PIPE"])):
            wl.step_pipelined()
        wl.pipeline_flush()
        torch.cuda.synchronize()
        r0 = np.frombuffer(wl.d_res.cpu().numpy().tobytes(), env.amodem.RESULT_DTYPE).copy()
        r1 = np.frombuffer(wl.d_res2.cpu().numpy().tobytes(), env.amodem.RESULT_DTYPE).copy()
        p0 = wl.d_pay.view(wl.F, wl.stride).cpu().numpy()
        p1 = wl.d_pay2.view(wl.F, wl.stride).cpu().numpy()
        bad = [i for i in range(wl.F) if r1[i].tobytes() != r0[i].tobytes() or p1[i].tobytes() != p0[i].tobytes()]
        print(f"pipelined: {len(bad)} frames differ", flush=True)
        for i in bad[:8]:
            fields = [n for n in r0.dtype.names if r1[n][i] != r0[n][i]]
            dpay = np.nonzero(p1[i] != p0[i])[0]
            print("  frame", i, "fields", {n: (r0[n][i].item(), r1[n][i].item()) for n in fields}, "flags",
                  hex(int(r0["flags"][i])), hex(int(r1["flags"][i])), "pv", int(r0["payload_valid"][i]),
                  int(r1["payload_valid"][i]), "payload bytes differ", len(dpay), dpay[:6].tolist())
        wl.close()
        return
    for it in range(6):
        wl.step_ctx(it % 2, wl.stream) if opts == 0 else None
        if opts:
            dm = wl.dm if it % 2 == 0 else wl.dm2
            res, pay = (wl.d_res, wl.d_pay) if it % 2 == 0 else (wl.d_res2, wl.d_pay2)
            dm.decode_device(wl.cfg, wl.mode, wl.xs.data_ptr(), wl.d_doff.data_ptr(), wl.d_dlen.data_ptr(), wl.F,
                             res.data_ptr(), pay.data_ptr(), wl.stride, stream=wl.stream, options=opts)
        torch.cuda.synchronize()
        res, pay = (wl.d_res, wl.d_pay) if it % 2 == 0 else (wl.d_res2, wl.d_pay2)
        outs.append((np.frombuffer(res.cpu().numpy().tobytes(), env.amodem.RESULT_DTYPE).copy(),
                     pay.view(wl.F, wl.stride).cpu().numpy().copy()))
    r0, p0 = outs[0]
    for k, (r, p) in enumerate(outs[1:], 1):
        bad = [i for i in range(wl.F) if r[i].tobytes() != r0[i].tobytes() or p[i].tobytes() != p0[i].tobytes()]
        print(f"decode {k} vs 0: {len(bad)} frames differ", flush=True)
        for i in bad[:6]:
            fields = [n for n in r.dtype.names if r[n][i] != r0[n][i]]
            dpay = np.nonzero(p[i] != p0[i])[0]
            print("  frame", i, "fields", {n: (int(r0[n][i]) if r.dtype[n].kind != 'f' else float(r0[n][i]),
                                               int(r[n][i]) if r.dtype[n].kind != 'f' else float(r[n][i]))
                                           for n in fields}, "payload bytes differ", len(dpay), dpay[:4].tolist())
    wl.close()


if __name__ == "__main__":
    main()
