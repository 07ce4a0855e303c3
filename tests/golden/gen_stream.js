#!/usr/bin/env node
// Golden-vector generator for the streaming receiver (test infrastructure, runs ONLY
// in the build container). Loads the UNMODIFIED reference modem.js and app.js with
// vm.runInThisContext behind minimal DOM / IndexedDB stand-ins, builds chunked-file
// audio streams with the reference's own transmit builders from recipes, and feeds
// them to the reference StreamingReceiver (app.js:706-998) in 4096-sample blocks
// (the ScriptProcessor size, app.js:1103), letting its async work finish between
// blocks as a real-time audio callback would. Recorded per stream: the SHA-256 of
// the stream (rebuilt bit-exactly by the product TX + oracle post-ops), every
// demodulated frame window (preambleGlobalPos, expectedFrameEnd) with the
// decodeChunkFrame result, failed refinements, the receiver counters and the file
// it offers for download. Only recipes and outputs are written.
//
// Usage: node tests/golden/gen_stream.js [/root/reference]
'use strict';
const vm = require('vm');
const fs = require('fs');
const path = require('path');
const util = require('util');
const crypto = require('crypto');

const REF = process.argv[2] || '/root/reference';
global.TextEncoder = util.TextEncoder;
global.TextDecoder = util.TextDecoder;
const el = () => ({ addEventListener() {}, style: {}, classList: { add() {}, remove() {}, toggle() {} },
  appendChild() {}, setAttribute() {}, getContext: () => null, textContent: '', innerHTML: '', value: '' });
global.document = { addEventListener() {}, getElementById: () => null, createElement: el,
  querySelectorAll: () => [], querySelector: () => null, body: el() };
global.window = global;
function fakeIndexedDB() {
  const dbs = {};
  const later = (f) => setImmediate(f);
  return {
    open(name) {
      const req = {};
      later(() => {
        let db = dbs[name];
        const fresh = !db;
        if (fresh) {
          const stores = {};
          db = dbs[name] = {
            objectStoreNames: { contains: (n) => n in stores },
            createObjectStore(n, opts) { stores[n] = { keyPath: opts.keyPath, map: new Map() }; },
            close() {},
            transaction(n) {
              const st = stores[n];
              const tx = {};
              tx.objectStore = () => ({
                clear() { st.map.clear(); },
                put(obj) { st.map.set(obj[st.keyPath], { seqNum: obj.seqNum, data: new Uint8Array(obj.data) }); },
                get(key) { const r = {}; later(() => { r.result = st.map.get(key); if (r.onsuccess) r.onsuccess(); }); return r; },
              });
              later(() => { if (tx.oncomplete) tx.oncomplete(); });
              return tx;
            },
          };
        }
        req.result = db;
        if (fresh && req.onupgradeneeded) req.onupgradeneeded({ target: { result: db } });
        if (req.onsuccess) req.onsuccess({ target: { result: db } });
      });
      return req;
    },
  };
}
global.indexedDB = fakeIndexedDB();

vm.runInThisContext(fs.readFileSync(path.join(REF, 'modem.js'), 'utf8'), { filename: 'modem.js' });
vm.runInThisContext(fs.readFileSync(path.join(REF, 'app.js'), 'utf8'), { filename: 'app.js' });
// UI hooks the receiver calls: silenced; the offered download is captured
let offered = null;
global.addLog = () => {};
global.updateStreamingUI = () => {};
global.drawChunkBitmap = () => {};
global.updateProgress = () => {};
global.offerDownload = (data, name) => { offered = { data, name }; };
const StreamingReceiverRef = vm.runInThisContext('StreamingReceiver');
const RECV = vm.runInThisContext('RECV_STATE');

// ---- recipes (same as gen_golden.js; restated by oracle/oracle.py apply_post)
function xs32(s) { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s; }
function payloadBytes(seed, len) {
  const out = new Uint8Array(len);
  let s = seed >>> 0;
  for (let i = 0; i < len; i++) { if ((i & 3) === 0) s = xs32(s); out[i] = (s >>> (8 * (i & 3))) & 0xff; }
  return out;
}
function addNoise(sig, snrDb, seed) {
  let p = 0, cnt = 0;
  for (let i = 0; i < sig.length; i++) { const v = sig[i]; if (v !== 0) { p += v * v; cnt++; } }
  p = cnt > 0 ? p / cnt : 0;
  let div = 1; for (let k = 0; k < snrDb / 10; k++) div *= 10;
  const sigma = Math.sqrt(p / div);
  let s = seed >>> 0;
  const out = new Float32Array(sig.length);
  for (let i = 0; i < sig.length; i++) {
    let g = 0;
    for (let j = 0; j < 12; j++) { s = xs32(s); g += s / 4294967296; }
    g -= 6;
    out[i] = Math.fround(sig[i] + sigma * g);
  }
  return out;
}
function applyPost(sig, post) {
  for (const op of post || []) {
    if (op.op === 'noise') sig = addNoise(sig, op.snr, op.seed);
    else if (op.op === 'dc') { const o = new Float32Array(sig.length); for (let i = 0; i < sig.length; i++) o[i] = Math.fround(sig[i] + op.dc); sig = o; }
    else if (op.op === 'gain') { const o = new Float32Array(sig.length); for (let i = 0; i < sig.length; i++) o[i] = Math.fround(sig[i] * op.gain); sig = o; }
    else throw new Error('bad post op');
  }
  return sig;
}

// stream = lead zeros + frames (metadata / data chunks of one file) + tail zeros,
// zero-padded to whole 4096-sample blocks, then the post ops over everything
function buildStream(sp) {
  setOFDMConfig(sp.config);
  const file = payloadBytes(sp.fileSeed, sp.fileLen);
  const nch = Math.ceil(sp.fileLen / sp.chunkSize);
  const parts = [new Float32Array(sp.lead || 0)];
  for (const f of sp.frames) {
    let s;
    if (f.kind === 'meta') s = buildMetadataFrame(nch, sp.fileLen, sp.chunkSize, sp.fileName, sp.mod, sp.rep);
    else s = buildDataChunkFrame(file.slice(f.seq * sp.chunkSize, (f.seq + 1) * sp.chunkSize), f.seq, sp.mod, sp.rep);
    if (f.corrupt) { s = Float32Array.from(s); for (let i = f.corrupt.start; i < f.corrupt.end; i++) s[i] = Math.fround(f.corrupt.value); }
    parts.push(s);
    if (f.gap) parts.push(new Float32Array(f.gap));
  }
  parts.push(new Float32Array(sp.tail || 0));
  let n = parts.reduce((a, p) => a + p.length, 0);
  const total = Math.ceil(n / 4096) * 4096;
  const sig = new Float32Array(total);
  let off = 0;
  for (const p of parts) { sig.set(p, off); off += p.length; }
  return { sig: applyPost(sig, sp.post), file };
}

async function runReceiver(sp, sig) {
  setOFDMConfig(sp.config);
  offered = null;
  const rx = new StreamingReceiverRef(sp.mod, sp.rep);
  const frames = [], refineFail = [];
  const origDemod = rx._demodulateFrame.bind(rx);
  rx._demodulateFrame = function () { frames.push({ pos: this.preambleGlobalPos, end: this.expectedFrameEnd }); return origDemod(); };
  const origRefine = rx._refineAndCollect.bind(rx);
  rx._refineAndCollect = function () {
    const pos = this.preambleGlobalPos;
    origRefine();
    if (this.state === RECV.IDLE) refineFail.push(pos);
  };
  const origDecode = global.decodeChunkFrame;
  global.decodeChunkFrame = (x, m, r) => {
    const res = origDecode(x, m, r);
    const rec = frames[frames.length - 1];
    rec.len = x.length;
    if (res.error) rec.error = res.error;
    else {
      rec.frameType = res.frameType; rec.crcValid = res.crcValid;
      if (res.frameType === FRAME_DATA) { rec.seqNum = res.seqNum; rec.dataLen = res.dataLen; }
      else { rec.totalChunks = res.totalChunks; rec.chunkSize = res.chunkSize; rec.fileName = res.fileName; }
    }
    return res;
  };
  const settle = async () => { for (let k = 0; k < 4; k++) await new Promise((r) => setImmediate(r)); };
  for (let b = 0; b < sig.length; b += 4096) {
    rx.processAudioBlock(sig.subarray(b, b + 4096));
    await settle();
    while (rx.state === RECV.DEMODULATING) await settle();
  }
  for (let k = 0; k < 200 && offered === null && rx.assembler.isComplete() && rx.assembler.totalChunks > 0; k++) await settle();
  global.decodeChunkFrame = origDecode;
  const a = rx.assembler;
  return {
    frames, refineFail, framesDecoded: rx.framesDecoded, frameErrors: rx.frameErrors,
    assembler: { totalChunks: a.totalChunks, totalFileSize: a.totalFileSize, chunkSize: a.chunkSize, fileName: a.fileName,
      receivedCount: a.receivedCount, crcErrors: a.crcErrors, complete: a.isComplete() },
    offered: offered ? { name: offered.name, size: offered.data.length,
      sha256: crypto.createHash('sha256').update(Buffer.from(offered.data)).digest('hex') } : null,
    final: { state: rx.state, acScanPos: rx.acScanPos },
  };
}

const chunks = (n, extra) => Array.from({ length: n }, (_, i) => Object.assign({ kind: 'chunk', seq: i }, (extra || {})[i] || {}));
const STREAMS = [
  { name: 'qpsk_clean', config: 'standard', mod: 'QPSK', rep: 1, chunkSize: 2048, fileSeed: 0x51, fileLen: 8 * 2048 - 300,
    fileName: 'clean.bin', lead: 0, tail: 8192, frames: [{ kind: 'meta' }, ...chunks(8)] },
  { name: 'qpsk_dc_gain_lead', config: 'standard', mod: 'QPSK', rep: 1, chunkSize: 2048, fileSeed: 0x52, fileLen: 5 * 2048,
    fileName: 'dc.bin', lead: 7777, tail: 8192, frames: [{ kind: 'meta' }, ...chunks(5, { 2: { gap: 3000 } })],
    post: [{ op: 'gain', gain: 0.5 }, { op: 'dc', dc: 0.1 }] },
  { name: 'qam16_noise20', config: 'standard', mod: 'QAM16', rep: 1, chunkSize: 2048, fileSeed: 0x53, fileLen: 6 * 2048 - 1,
    fileName: 'noisy.bin', lead: 2000, tail: 8192, frames: [{ kind: 'meta' }, ...chunks(6)],
    post: [{ op: 'noise', snr: 20, seed: 0x5eed }] },
  { name: 'qpsk_corrupt_retransmit', config: 'standard', mod: 'QPSK', rep: 1, chunkSize: 1024, fileSeed: 0x54, fileLen: 5 * 1024,
    fileName: 'retx.bin', lead: 0, tail: 8192,
    frames: [{ kind: 'meta' }, ...chunks(5, { 2: { corrupt: { start: 2205 + 1728 + 600, end: 2205 + 1728 + 900, value: 0.6 } } }),
      { kind: 'chunk', seq: 2 }, { kind: 'chunk', seq: 3 }] },
  { name: 'acoustic_bpsk3', config: 'acoustic', mod: 'BPSK', rep: 3, chunkSize: 128, fileSeed: 0x55, fileLen: 3 * 128 - 20,
    fileName: 'ac.bin', lead: 500, tail: 12288, frames: [{ kind: 'meta' }, ...chunks(3)] },
  { name: 'narrowband_qpsk', config: 'narrowband', mod: 'QPSK', rep: 1, chunkSize: 64, fileSeed: 0x56, fileLen: 3 * 64,
    fileName: 'nb.bin', lead: 0, tail: 12288, frames: [{ kind: 'meta' }, ...chunks(3)] },
  { name: 'no_metadata', config: 'standard', mod: 'QPSK', rep: 1, chunkSize: 2048, fileSeed: 0x57, fileLen: 2 * 2048,
    fileName: 'nometa.bin', lead: 0, tail: 8192, frames: chunks(2) },
];

(async () => {
  const out = { generator: 'tests/golden/gen_stream.js', reference: 'app.js StreamingReceiver (706-998), 4096-sample blocks', streams: [] };
  for (const sp of STREAMS) {
    const { sig, file } = buildStream(sp);
    const res = await runReceiver(sp, sig);
    const sha = crypto.createHash('sha256').update(Buffer.from(sig.buffer, sig.byteOffset, sig.byteLength)).digest('hex');
    const fileSha = crypto.createHash('sha256').update(Buffer.from(file)).digest('hex');
    const rec = Object.assign({}, sp, { recipe: sp.frames, n: sig.length, sha256: sha, fileSha256: fileSha }, res);
    out.streams.push(rec);
    console.log(sp.name, sig.length, 'frames', res.frames.length, 'decoded', res.framesDecoded, 'errors', res.frameErrors,
      'offered', res.offered && res.offered.sha256 === fileSha, 'refineFail', res.refineFail.length);
  }
  fs.writeFileSync(path.join(__dirname, 'stream.json'), JSON.stringify(out));
})();
