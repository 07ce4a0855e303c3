#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh directory into the committed profile files:
kernel_stats.csv (rocprofv3 --stats of the C2 bench), per_dispatch_us.txt (the fast-path
kernels' durations, dispatch by dispatch), counters.txt (per-kernel means of every PMC
counter), traffic.json (FETCH_SIZE x 2 and WRITE_SIZE per launch against the
algorithmic bytes of bench.json, per kernel and for the chain).

usage: python tools/profile_summary.py gpurun_out/r03/c2 profiles/r03/c2
(a step is one k_detect launch, or one k_chunk_prep launch in chunk mode; traffic.json
entries of several workloads are merged into profiles/<round>/traffic.json by
tools/profile_merge.py)
"""
import collections
import csv
import json
import os
import re
import shutil
import sys


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][-48:]


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "ktrace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for f in ("bench.json", "bench_under_rocprof.json", "bench_c5_20db.json", "bench_c5_10db.json",
              "bench_stream_under_rocprof.json"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    if os.path.exists(os.path.join(src, "ktrace_stream", "run_kernel_stats.csv")):
        shutil.copy(os.path.join(src, "ktrace_stream", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats_stream.csv"))
    if os.path.exists(os.path.join(src, "ktrace_c5", "run_kernel_stats.csv")):
        shutil.copy(os.path.join(src, "ktrace_c5", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats_c5_10db.csv"))
    # per-dispatch durations of the fast path kernels
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, "ktrace", "run_kernel_trace.csv"))):
        k = short(r["Kernel_Name"])
        if k in ("k_detect", "k_demod", "k_decode_exact", "k_corr_scan", "k_chunk_prep"):
            per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    with open(os.path.join(dst, "per_dispatch_us.txt"), "w") as fo:
        for k, v in per.items():
            s = sorted(v)
            fo.write("%s n=%d mean=%.1f median=%.1f min=%.1f max=%.1f\n  %s\n" % (
                k, len(v), sum(v) / len(v), s[len(s) // 2], s[0], s[-1], " ".join("%.1f" % x for x in v)))
    # counters
    all_c = {}
    for sub in ("fetch", "write", "sq", "sq2"):
        for k, d in counters(os.path.join(src, sub, "run_counter_collection.csv")).items():
            for c, v in d.items():
                all_c.setdefault(k, {})[c] = (sum(v) / len(v), len(v), sum(v))
    with open(os.path.join(dst, "counters.txt"), "w") as fo:
        fo.write("per-kernel mean over dispatches (rocprofv3 --pmc, one pass per counter group; "
                 "SQ counters summed over the chip)\n")
        for k in sorted(all_c):
            if not k.startswith("k_"):
                continue
            fo.write("%s\n" % k)
            for c, (m, n, _) in sorted(all_c[k].items()):
                fo.write("    %-24s %18.1f   (%d dispatches)\n" % (c, m, n))
    # traffic vs algorithmic bytes (FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE
    # reports half the bytes of a wide coalesced stream: x2, MI355X_MICROARCH.md)
    bench = json.load(open(os.path.join(src, "bench.json")))
    frames = bench["config"]["frames_per_gpu"]
    spf = bench["config"]["samples_per_frame"]
    alg_chain = 4.0 * frames * spf
    alg = {"k_detect": alg_chain, "k_corr_scan": alg_chain}
    rf = bench.get("roofline", {})
    if rf.get("kernel") == "k_demod":
        alg["k_demod"] = rf["algorithmic_bytes"]
    step_k = "k_detect" if "k_detect" in all_c else "k_chunk_prep"
    out = {"workload": bench["config"]["workload"], "frames": frames, "samples_per_frame": spf,
           "note": "FETCH_SIZE x 2 (gfx950 half-count of wide streaming reads) and WRITE_SIZE, KiB -> bytes, per launch",
           "kernels": {}}
    # per step: a kernel's bytes over all its dispatches / the steps (k_detect dispatches) of
    # the pass; k_demod runs twice a step (the main launch and the detection-replay list
    # launch, usually empty), k_decode_exact three times
    tot_r = tot_w = 0.0
    steps_f = all_c.get(step_k, {}).get("FETCH_SIZE", (0, 1, 0))[1]
    steps_w = all_c.get(step_k, {}).get("WRITE_SIZE", (0, 1, 0))[1]
    out["note"] = ("FETCH_SIZE x 2 (gfx950 half-count of wide streaming reads) and WRITE_SIZE, KiB -> bytes, per step "
                   "(all of a kernel's dispatches in the pass / its %s dispatches)" % step_k)
    for k in ("k_detect", "k_chunk_prep", "k_demod", "k_decode_exact", "k_corr_scan"):
        c = all_c.get(k, {})
        if "FETCH_SIZE" not in c:
            continue
        steps_k_f = steps_f if k != "k_corr_scan" else c["FETCH_SIZE"][1]
        steps_k_w = steps_w if k != "k_corr_scan" else c.get("WRITE_SIZE", (0, 1, 0))[1]
        rd = 2 * 1024 * c["FETCH_SIZE"][2] / max(1, steps_k_f)
        wr = 1024 * c.get("WRITE_SIZE", (0.0, 0, 0.0))[2] / max(1, steps_k_w)
        e = {"read_bytes": rd, "write_bytes": wr, "dispatches_per_step": c["FETCH_SIZE"][1] / max(1, steps_k_f)}
        if k in alg:
            e["algorithmic_bytes"] = alg[k]
            e["read_over_algorithmic"] = rd / alg[k]
        out["kernels"][k] = e
        if k in ("k_detect", "k_chunk_prep", "k_demod", "k_decode_exact"):
            tot_r += rd
            tot_w += wr
    out["chain"] = {"read_bytes": tot_r, "write_bytes": tot_w, "algorithmic_bytes": alg_chain,
                    "read_over_algorithmic": tot_r / alg_chain}
    json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))
    print(open(os.path.join(dst, "per_dispatch_us.txt")).read()[:2000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
