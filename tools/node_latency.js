#!/usr/bin/env node
// The drop-in as app.js calls it (app.js:513): one recording, synchronous
// decodeReceivedSignal from the JS surface (audio-modem_amd/js/modem.js -> N-API ->
// amod_decode_host: H2D, launches, sync, D2H, result object), timed per call
// (bench.py c1_latency leg). Usage: node tools/node_latency.js <spec.json>
// spec: {samples: <float32 file of one frame>, preset, mod, rep, warmup, calls}
'use strict';
const fs = require('fs');
const path = require('path');
const modem = require(path.join(__dirname, '..', 'audio-modem_amd', 'js', 'modem.js'));

const spec = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const buf = fs.readFileSync(spec.samples);
const sig = new Float32Array(buf.buffer.slice(buf.byteOffset, buf.byteOffset + buf.length - (buf.length % 4)));
modem.setOFDMConfig(spec.preset);
let res = null;
for (let i = 0; i < (spec.warmup || 20); i++) res = modem.decodeReceivedSignal(sig, spec.mod, spec.rep);
const ms = [];
for (let i = 0; i < (spec.calls || 200); i++) {
  const t0 = process.hrtime.bigint();
  res = modem.decodeReceivedSignal(sig, spec.mod, spec.rep);
  ms.push(Number(process.hrtime.bigint() - t0) / 1e6);
}
ms.sort((a, b) => a - b);
const q = (p) => ms[Math.min(ms.length - 1, Math.floor(p * ms.length))];
process.stdout.write(JSON.stringify({
  what: `decodeReceivedSignal(one ${sig.length}-sample recording) from node ${process.version}, synchronous, ` +
    `${ms.length} calls after ${spec.warmup || 20} warm-up calls`,
  median_ms: q(0.5), p10_ms: q(0.1), p90_ms: q(0.9), min_ms: ms[0], calls: ms.length,
  crcValid: res.crcValid === true, preambleIdx: res.preambleIdx, dataLen: res.dataLen,
}));
