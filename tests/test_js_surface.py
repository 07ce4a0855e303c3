"""The JavaScript surface (audio-modem_amd/js/modem.js over the N-API addon) against
the reference's golden vectors: same names, return shapes, values and error strings
as modem.js. CPU tests cover the host-side functions (no GPU call); the `gpu`
tests decode the golden frames through decodeReceivedSignal / decodeChunkFrame /
decodeBatch and compare with the reference's result objects."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import ROOT, frames, kat, loopback, sha

NODE = shutil.which("node")
DRIVER = os.path.join(ROOT, "tests", "js", "surface_driver.js")
ADDON = os.path.join(ROOT, "audio-modem_amd", "lib", "amodem.node")
MISSING = NODE is None or not os.path.exists(ADDON)


@pytest.fixture(autouse=True)
def _surface_present(request):
    # CPU tests skip without node / the addon; a GPU test never passes by skipping: both
    # travel with the image and the in-tree build, so their absence on the box is a failure
    if MISSING:
        if request.node.get_closest_marker("gpu"):
            pytest.fail("node or audio-modem_amd/lib/amodem.node missing on the GPU box")
        pytest.skip("node or amodem.node missing")

GLOBALS = ["fft", "OFDM_CONFIGS", "OFDM", "setOFDMConfig", "Constellations", "generatePreambleSymbol1",
           "buildTransmitSignal", "decodeReceivedSignal", "FRAME_META", "FRAME_DATA", "buildMetadataFrame",
           "buildDataChunkFrame", "decodeChunkFrame", "estimateFrameSamples", "generateSweepTone",
           "generateTestSignal", "analyzeLoopback"]


def run(jobs, tmp_path, timeout=600, env=None):
    for i, j in enumerate(jobs):
        j.setdefault("id", str(i))
    p = tmp_path / "jobs.json"
    p.write_text(json.dumps(jobs))
    out = subprocess.run([NODE, DRIVER, str(p)], capture_output=True, text=True, timeout=timeout,
                         env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout)


def ok(res, key):
    r = res[key]
    assert "ok" in r, r
    return r["ok"]


def test_exports(tmp_path):
    names = ok(run([{"op": "exports", "id": "e"}], tmp_path), "e")
    for g in GLOBALS + ["decodeBatch", "uploadBatch", "DeviceBatch"]:
        assert g in names, g


def test_fft_bit_exact(tmp_path):
    vecs = kat()["fft"]
    res = run([{"op": "fft", "re": v["inRe"], "im": v["inIm"], "id": v["label"]} for v in vecs], tmp_path)
    for v in vecs:
        re, im = ok(res, v["label"])
        assert re == v["fftRe"] and im == v["fftIm"], v["label"]


def test_crc32(tmp_path):
    vecs = kat()["crc32"]
    res = run([{"op": "crc32", "hex": v["hex"], "id": v["label"]} for v in vecs], tmp_path)
    for v in vecs:
        assert ok(res, v["label"]) == v["crc"]


def test_estimate_frame_samples_and_config(tmp_path):
    jobs = []
    for cfg, c in kat()["configs"].items():
        jobs.append({"op": "ofdm", "config": cfg, "id": f"ofdm_{cfg}"})
        jobs.append({"op": "preamble1", "config": cfg, "id": f"pre1_{cfg}"})
        for i, e in enumerate(c["estimateFrameSamples"]):
            jobs.append({"op": "estimate", "config": cfg, "payload": e["payload"], "mod": e["mod"], "rep": e["rep"],
                         "id": f"{cfg}_{i}"})
    jobs.append({"op": "ofdm", "config": "no-such-config", "id": "fallback"})
    res = run(jobs, tmp_path)
    for cfg, c in kat()["configs"].items():
        o = ok(res, f"ofdm_{cfg}")
        for k in ("FFT_SIZE", "CP_LEN", "SYMBOL_LEN", "SAMPLE_RATE", "SUB_START", "SUB_END", "PILOTS"):
            assert o["cfg"][k] == c[k], (cfg, k)
        assert o["nds"] == c["numDataSubs"]
        assert ok(res, f"pre1_{cfg}")["sha"] == sha(np.asarray(c["pre1"], np.float32))
        for i, e in enumerate(c["estimateFrameSamples"]):
            assert ok(res, f"{cfg}_{i}") == e["samples"], (cfg, e)
    assert ok(res, "fallback")["cfg"]["CP_LEN"] == 64  # unknown name -> standard (modem.js:96)


def test_constellations(tmp_path):
    jobs = [{"op": "constellations", "mod": m, "id": m} for m in ("BPSK", "QPSK", "QAM16")]
    jobs.append({"op": "estimate", "payload": 1, "mod": "PSK8", "rep": 1, "id": "bad"})
    res = run(jobs, tmp_path)
    for m in ("BPSK", "QPSK", "QAM16"):
        c = ok(res, m)
        assert c["bps"] == kat()["constellations"][m]["bps"]
        assert c["points"] == kat()["constellations"][m]["points"]
    assert res["bad"]["throw"] == "TypeError"


def test_sweep_tone(tmp_path):
    vecs = kat()["sweepTone"]
    res = run([{"op": "sweep", "args": v["args"], "id": str(i)} for i, v in enumerate(vecs)], tmp_path)
    for i, v in enumerate(vecs):
        r = ok(res, str(i))
        assert r["n"] == v["n"] and r["sha"] == v["sha"], v["args"]


def test_transmit_builders(tmp_path):
    from oracle import oracle as O
    jobs = []
    for i, t in enumerate(kat()["txInfo"]):
        data = O.payload(0x9E3779B9 ^ 7, t["len"]).tobytes()
        jobs.append({"op": "tx_legacy", "config": t["config"], "hex": data.hex(), "mod": t["mod"], "rep": t["rep"],
                     "name": t["name"], "id": f"info{i}"})
    cases = [f for f in frames() if f["tx"]["kind"] in ("legacy", "meta", "chunk", "test")]
    for f in cases:
        tx = f["tx"]
        j = {"config": f["config"], "mod": tx["mod"], "rep": tx["rep"], "id": f["name"]}
        if tx["kind"] == "legacy":
            j.update(op="tx_legacy", hex=O.payload(tx["seed"], tx["len"]).tobytes().hex(), name=tx["name"])
        elif tx["kind"] == "meta":
            j.update(op="tx_meta", chunks=tx["totalChunks"], size=tx["totalFileSize"], chunkSize=tx["chunkSize"],
                     name=tx["name"])
        elif tx["kind"] == "chunk":
            j.update(op="tx_chunk", hex=O.payload(tx["seed"], tx["len"]).tobytes().hex(), seq=tx["seq"])
        else:
            j.update(op="tx_test")
        jobs.append(j)
    res = run(jobs, tmp_path)
    for i, t in enumerate(kat()["txInfo"]):
        r = ok(res, f"info{i}")
        assert r["signal"]["sha"] == t["sha"] and r["signal"]["n"] == t["n"]
        for k in ("numSymbols", "bitsPerSymbol", "totalBits", "dataLen"):
            assert r[k] == t[k], (t, k)
    for f in cases:
        r = ok(res, f["name"])
        sig = r["signal"] if f["tx"]["kind"] in ("legacy", "test") else r
        assert sig["n"] == f["txLen"] and sig["sha"] == f["txSha"], f["name"]
        if f["tx"]["kind"] == "test":
            assert r["testData"] == {"hex": bytes(range(16)).hex()}


def test_analyze_loopback_needs_gpu(tmp_path):
    # the receive core runs on the GPU only: with no device it must throw, never run a CPU copy
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = tmp_path / "lb.js"
    p.write_text("process.env.AMODEM_NO_GLOBALS='1';const M=require(%r);"
                 "try{M.analyzeLoopback(new Float32Array(10),'QPSK',1,new Uint8Array(16));process.exit(3)}"
                 "catch(e){process.exit(e instanceof Error?0:4)}" % os.path.join(ROOT, "audio-modem_amd", "js", "modem.js"))
    assert subprocess.run([NODE, str(p)], timeout=120).returncode == 0


def test_loopback_golden_signals_rebuild():
    """The loopback fixtures' recipes rebuild the reference's exact input signals."""
    from oracle import oracle as O
    for c in loopback():
        x = O.build_case(c)
        assert len(x) == c["n"] and sha(x.astype(np.float32)) == c["sigSha"], c["name"]


# --------------------------------------------------------------- GPU decode --
def _norm(v):
    """golden JSON and driver output share the {hex} convention; strip nothing else"""
    return v


@pytest.mark.gpu
def test_decode_golden_frames_through_js(tmp_path):
    from oracle import oracle as O
    jobs = []
    for f in frames():
        x = np.ascontiguousarray(O.build_case(f), np.float32)
        fn = tmp_path / f"{f['name']}.f32"
        x.tofile(fn)
        jobs.append({"op": "decode" if f["rx"] == "legacy" else "decode_chunk", "config": f["config"],
                     "file": str(fn), "mod": f["mod"], "rep": f["rep"], "id": f["name"]})
    res = run(jobs, tmp_path)
    for f in frames():
        assert ok(res, f["name"]) == f["result"], f["name"]


@pytest.mark.gpu
def test_decode_batch_through_js(tmp_path):
    from oracle import oracle as O
    sel = [f for f in frames() if f["config"] == "standard" and f["rx"] == "legacy" and f["mod"] == "QPSK"
           and f["rep"] == 1]
    xs = [np.ascontiguousarray(O.build_case(f), np.float32) for f in sel]
    offs = np.cumsum([0] + [len(x) for x in xs[:-1]]).tolist()
    fn = tmp_path / "batch.f32"
    np.concatenate(xs).astype(np.float32).tofile(fn)
    res = run([{"op": "decode_batch", "config": "standard", "file": str(fn), "offsets": offs,
                "lengths": [len(x) for x in xs], "mod": "QPSK", "rep": 1, "id": "b"},
               {"op": "decode_batch", "config": "standard", "file": str(fn), "offsets": offs,
                "lengths": [len(x) for x in xs], "mod": "QPSK", "rep": 1, "share": True, "id": "s"}], tmp_path)
    got = ok(res, "b")
    assert got["results"] == [f["result"] for f in sel]
    assert got["ownData"]  # every `data` a fresh Uint8Array, as bytes.slice (modem.js:636,837)
    shared = ok(res, "s")  # shareBuffers: the same results, views of one payload buffer
    assert shared["results"] == got["results"] and not shared["ownData"]
    assert got["progress"][-1] == len(sel) and got["prefixes_final"]


@pytest.mark.gpu
def test_decode_batch_progress_through_js(tmp_path):
    """decodeBatch formats each uploaded piece's frames while the library decodes the rest
    (amod_decode_host_progress, a napi threadsafe callback): with 16 KB upload pieces (the
    runtime's AMOD_UP_PIECE test knob) the frames come back in many steps; every onProgress
    prefix is already final and the results equal the golden ones, plain and shared."""
    from oracle import oracle as O
    sel = [f for f in frames() if f["config"] == "standard" and f["rx"] == "legacy" and f["mod"] == "QPSK"
           and f["rep"] == 1]
    xs = [np.ascontiguousarray(O.build_case(f), np.float32) for f in sel]
    offs = np.cumsum([0] + [len(x) for x in xs[:-1]]).tolist()
    fn = tmp_path / "batch.f32"
    np.concatenate(xs).astype(np.float32).tofile(fn)
    job = {"op": "decode_batch", "config": "standard", "file": str(fn), "offsets": offs,
           "lengths": [len(x) for x in xs], "mod": "QPSK", "rep": 1}
    res = run([dict(job, id="b"), dict(job, id="s", share=True)], tmp_path, env={"AMOD_UP_PIECE": "4096"})
    for key in ("b", "s"):
        got = ok(res, key)
        assert got["results"] == [f["result"] for f in sel], key
        pr = got["progress"]
        assert len(pr) > 1 and pr[-1] == len(sel) and all(a < b for a, b in zip(pr, pr[1:])), pr
        assert got["prefixes_final"], key


@pytest.mark.gpu
def test_decode_batch_progress_throws(tmp_path):
    """An onProgress that throws (it runs from the library's progress callback, where no
    caller could catch it) rejects decodeBatch's promise with that error, is not called
    again, and leaves the addon usable: the next decodeBatch resolves normally."""
    from oracle import oracle as O
    sel = [f for f in frames() if f["config"] == "standard" and f["rx"] == "legacy" and f["mod"] == "QPSK"
           and f["rep"] == 1]
    xs = [np.ascontiguousarray(O.build_case(f), np.float32) for f in sel]
    offs = np.cumsum([0] + [len(x) for x in xs[:-1]]).tolist()
    fn = tmp_path / "batch.f32"
    np.concatenate(xs).astype(np.float32).tofile(fn)
    job = {"op": "decode_batch_throw", "config": "standard", "file": str(fn), "offsets": offs,
           "lengths": [len(x) for x in xs], "mod": "QPSK", "rep": 1}
    res = run([dict(job, id="t")], tmp_path, env={"AMOD_UP_PIECE": "4096"})
    got = ok(res, "t")
    assert got["rejected"] == "onProgress boom" and got["calls"] == 1, got
    assert got["again"] == len(sel), got


@pytest.mark.gpu
def test_resident_batch_through_js(tmp_path):
    """uploadBatch (amod_group_upload) makes the batch resident on two GPU contexts
    (device 0 twice on the one-GPU box) once; decodeBatch(DeviceBatch) decodes it from
    HBM (amod_resident_decode), twice: the reference result objects in frame order."""
    from oracle import oracle as O
    sel = [f for f in frames() if f["config"] == "standard" and f["rx"] == "legacy" and f["mod"] == "QPSK"
           and f["rep"] == 1]
    xs = [np.ascontiguousarray(O.build_case(f), np.float32) for f in sel]
    offs = np.cumsum([0] + [len(x) for x in xs[:-1]]).tolist()
    fn = tmp_path / "batch.f32"
    np.concatenate(xs).astype(np.float32).tofile(fn)
    res = run([{"op": "decode_resident", "config": "standard", "file": str(fn), "offsets": offs,
                "lengths": [len(x) for x in xs], "mod": "QPSK", "rep": 1, "devices": 2, "id": "r"}], tmp_path,
              env={"AMODEM_GROUP_DEVICES": "0,0"})
    got = ok(res, "r")
    want = [f["result"] for f in sel]
    assert got["isDeviceBatch"] and sum(got["framesPerDevice"]) == len(sel)
    assert got["first"] == want and got["second"] == want  # (the second with free() called while in flight)
    assert got["afterFree"] and "freed" in got["afterFree"]


@pytest.mark.gpu
def test_resident_batch_concurrent_decodes(tmp_path):
    """two decodeBatch(DeviceBatch) promises in flight on one resident batch,
    with different modulations (different payload strides; the batch was reserved for
    QPSK, so the other is the narrower BPSK), run on the libuv pool at
    once; amod_resident_decode serialises them, so each equals the same decode alone."""
    from oracle import oracle as O
    sel = [f for f in frames() if f["config"] == "standard" and f["rx"] == "legacy" and f["mod"] == "QPSK"
           and f["rep"] == 1]
    xs = [np.ascontiguousarray(O.build_case(f), np.float32) for f in sel]
    offs = np.cumsum([0] + [len(x) for x in xs[:-1]]).tolist()
    fn = tmp_path / "batch.f32"
    np.concatenate(xs).astype(np.float32).tofile(fn)
    res = run([{"op": "decode_resident_concurrent", "config": "standard", "file": str(fn), "offsets": offs,
                "lengths": [len(x) for x in xs], "mod": "QPSK", "mods": ["QPSK", "BPSK", "QPSK"], "rep": 1,
                "devices": 2, "id": "c"}], tmp_path, env={"AMODEM_GROUP_DEVICES": "0,0"})
    got = ok(res, "c")
    assert got["same"]
    assert got["first"] == [f["result"] for f in sel]


def _lb_num(v):
    return float(v["num"]) if isinstance(v, dict) else float(v)


def _gold_num(v):
    return float(v) if isinstance(v, str) else v


@pytest.mark.gpu
def test_analyze_loopback_golden(tmp_path):
    """analyzeLoopback (modem.js:975-1082) on the reference's own loopback results:
    detection (Schmidl-Cox, then the cross-correlation fallback), correlation, the
    CE magnitudes, pilot SNR, BER against the 16-byte test pattern and quality."""
    from oracle import oracle as O
    jobs = []
    for c in loopback():
        fn = tmp_path / f"{c['name']}.f32"
        np.ascontiguousarray(O.build_case(c), np.float32).tofile(fn)
        jobs.append({"op": "loopback", "config": c["config"], "file": str(fn), "mod": c["mod"], "rep": c["rep"],
                     "testData": list(range(16)), "id": c["name"]})
    res = run(jobs, tmp_path)
    for c in loopback():
        g = c["result"]
        r = ok(res, c["name"])
        assert r["detected"] == g["detected"] and r["quality"] == g["quality"], (c["name"], r, g)
        assert r["ber"] == g["ber"], c["name"]
        # fp64 replica of the reference arithmetic: equal to the last few ulps
        assert _lb_num(r["correlation"]) == pytest.approx(_gold_num(g["correlation"]), rel=1e-12, abs=1e-15), c["name"]
        assert _lb_num(r["snrEstimate"]) == pytest.approx(_gold_num(g["snrEstimate"]), rel=1e-9, abs=1e-9), c["name"]
        got = [_lb_num(v) for v in r["channelMagnitude"]]
        exp = [_gold_num(v) for v in g["channelMagnitude"]]
        assert got == pytest.approx(exp, rel=1e-12, abs=1e-12), c["name"]


def _asm_scenarios():
    from helpers import GOLDEN
    with open(os.path.join(GOLDEN, "assembler.json")) as f:
        return json.load(f)["scenarios"]


@pytest.mark.parametrize("store", ["memory", "files"])
def test_chunk_assembler_through_js(store, tmp_path):
    """app.js ChunkAssembler's methods, getters and thrown errors through the JS class,
    on every golden scenario the reference produced (tests/golden/assembler.json)."""
    import amodem
    scen = _asm_scenarios()
    jobs = []
    for name, sc in sorted(scen.items()):
        ops = []
        for op in sc["ops"]:
            op = dict(op)
            if op["op"] == "chunk":
                op["hex"] = amodem.synth_payload(op["seed"], op["len"]).hex()
            ops.append(op)
        d = tmp_path / name
        if store == "files":
            d.mkdir()
        jobs.append({"op": "asm", "ops": ops, "id": name, **({"directory": str(d)} if store == "files" else {})})
    res = run(jobs, tmp_path)
    for name, sc in scen.items():
        got = ok(res, name)
        assert len(got) == len(sc["steps"]), name
        for g, step in zip(got, sc["steps"]):
            w = step["state"]
            assert g["error"] == step["error"], (name, g)
            assert g["file"] == step["file"], name
            for k in ("totalChunks", "totalFileSize", "chunkSize", "receivedCount", "crcErrors", "complete"):
                assert g[k] == w[k], (name, k)
            assert g["fileName"] == (w["fileName"] or ""), name
            if w["bitmap"] is not None:
                assert g["bitmap"][:64] == w["bitmap"], name
                assert len(g["bitmap"]) == w["bitmapLen"], name
            else:
                assert g["bitmap"] is None, name
            if w["missing"] is not None:
                assert g["missing"] == w["missing"], name
                miss = set(w["missing"])
                assert g["received"] == [i not in miss for i in range(w["totalChunks"])], name


def test_chunk_assembler_close(tmp_path):
    """ChunkAssembler handles are numbers released by close() (or at exit), not napi
    externals: a closed handle throws TypeError, a second close is a no-op, 3000
    open/close cycles run, and assemblers left open do not crash the exit (Node 12's
    weak references on externals did)."""
    r = ok(run([{"op": "asm_close", "id": "c", "cycles": 3000, "leftOpen": 50}], tmp_path), "c")
    assert r == {"before": 2, "after": "TypeError", "chunk": "TypeError", "again": None, "cycles": 3000}


@pytest.mark.gpu
def test_receive_stream_through_js(tmp_path):
    """receiveStream (StreamingReceiver over a recorded stream) from JS on the golden
    streams: every window, its decode outcome, the failed refinements, the counters and
    the assembled file equal what the reference receiver did (tests/golden/stream.json)."""
    from test_gpu_stream import build_stream, streams
    jobs, want = [], {}
    for sp in streams():
        _, x, _ = build_stream(sp)
        p = tmp_path / f"{sp['name']}.f32"
        x.astype(np.float32).tofile(p)
        jobs.append({"op": "stream", "file": str(p), "mod": sp["mod"], "rep": sp["rep"], "config": sp["config"],
                     "id": sp["name"]})
        want[sp["name"]] = sp
    res = run(jobs, tmp_path)
    for name, sp in want.items():
        g = ok(res, name)
        got = [{"pos": f["preambleGlobalPos"], "end": f["expectedFrameEnd"], "len": f["length"],
                **({"error": f["result"]["error"]} if "error" in f["result"] else
                   {k: v for k, v in f["result"].items() if k in ("frameType", "crcValid", "seqNum", "dataLen",
                                                                   "totalChunks", "chunkSize")})}
               for f in g["frames"]]
        exp = [{k: v for k, v in w.items() if k != "fileName"} for w in sp["frames"]]
        assert got == exp, name
        assert g["refineFail"] == sp["refineFail"], name
        assert (g["framesDecoded"], g["frameErrors"]) == (sp["framesDecoded"], sp["frameErrors"]), name
        a = sp["assembler"]
        assert [g["asm"][k] for k in ("totalChunks", "totalFileSize", "chunkSize", "receivedCount", "crcErrors",
                                      "complete", "fileName")] == [a[k] for k in ("totalChunks", "totalFileSize",
                                                                                 "chunkSize", "receivedCount",
                                                                                 "crcErrors", "complete",
                                                                                 "fileName")], name
        if sp["offered"] is not None:
            assert g["file"] == sp["offered"]["sha256"], name


@pytest.mark.gpu
def test_live_receiver_through_js(tmp_path):
    """StreamingReceiver.processAudioBlock from JS, one 4096-sample block per call (the
    reference's audio callback, app.js:1108-1112), on the golden streams: the windows,
    outcomes, counters, final scan position and assembled file equal the reference's."""
    from test_gpu_stream import build_stream, streams
    jobs, want = [], {}
    for sp in streams():
        _, x, _ = build_stream(sp)
        p = tmp_path / f"{sp['name']}.f32"
        x.astype(np.float32).tofile(p)
        jobs.append({"op": "live", "file": str(p), "mod": sp["mod"], "rep": sp["rep"], "config": sp["config"],
                     "id": sp["name"]})
        want[sp["name"]] = sp
    res = run(jobs, tmp_path)
    for name, sp in want.items():
        g = ok(res, name)
        got = [{"pos": f["preambleGlobalPos"], "end": f["expectedFrameEnd"], "len": f["length"],
                **({"error": f["result"]["error"]} if "error" in f["result"] else
                   {k: v for k, v in f["result"].items() if k in ("frameType", "crcValid", "seqNum", "dataLen",
                                                                   "totalChunks", "chunkSize")})}
               for f in g["frames"]]
        assert got == [{k: v for k, v in w.items() if k != "fileName"} for w in sp["frames"]], name
        assert (g["framesDecoded"], g["frameErrors"]) == (sp["framesDecoded"], sp["frameErrors"]), name
        assert (g["state"], g["acScanPos"]) == (sp["final"]["state"], sp["final"]["acScanPos"]), name
        assert g["totalWritten"] == sp["n"], name
        # assembler closed first: its handle throws, the receiver on it keeps working
        assert g["afterAsmClose"] == {"asm": "TypeError", "rxState": g["state"], "rxBlock": None}, name
        assert g["afterRxClose"] == {"rx": "TypeError", "again": None}, name
        a = sp["assembler"]
        assert [g["asm"][k] for k in ("totalChunks", "totalFileSize", "chunkSize", "receivedCount", "crcErrors",
                                      "complete", "fileName")] == [a[k] for k in ("totalChunks", "totalFileSize",
                                                                                 "chunkSize", "receivedCount",
                                                                                 "crcErrors", "complete",
                                                                                 "fileName")], name
        if sp["offered"] is not None:
            assert g["file"] == sp["offered"]["sha256"], name


@pytest.mark.gpu
def test_decode_batch_devices_through_js(tmp_path):
    """decodeBatch(..., {devices: 2}) splits the batch over two GPU contexts
    (amod_group_decode_host; on the one-GPU box both on device 0 via AMODEM_GROUP_DEVICES):
    the reference result objects, in frame order, as with one device."""
    from oracle import oracle as O
    sel = [f for f in frames() if f["config"] == "standard" and f["rx"] == "legacy" and f["rep"] == 1
           and f["mod"] in ("QPSK", "BPSK")]
    xs = [np.ascontiguousarray(O.build_case(f), np.float32) for f in sel]
    offs = np.cumsum([0] + [len(x) for x in xs[:-1]]).tolist()
    fn = tmp_path / "batch.f32"
    np.concatenate(xs).astype(np.float32).tofile(fn)
    groups = {}
    for f in sel:
        groups.setdefault(f["mod"], []).append(sel.index(f))
    jobs = []
    for mod, idx in groups.items():
        jobs.append({"op": "decode_batch", "config": "standard", "file": str(fn), "offsets": [offs[i] for i in idx],
                     "lengths": [len(xs[i]) for i in idx], "mod": mod, "rep": 1, "devices": 2, "id": mod})
    res = run(jobs, tmp_path, env={"AMODEM_GROUP_DEVICES": "0,0"})
    for mod, idx in groups.items():
        assert ok(res, mod)["results"] == [sel[i]["result"] for i in idx], mod
