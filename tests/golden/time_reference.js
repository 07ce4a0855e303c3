#!/usr/bin/env node
// CPU-baseline calibration (runs ONLY in the build container, like gen_golden.js): times
// the UNMODIFIED reference /root/reference/modem.js (vm.runInThisContext, single thread)
// on the bench workloads' frames, built by the reference's own transmitter from the
// same xorshift32 payloads the product's synthetic inputs use. Prints JSON: per
// workload the median milliseconds per frame over `reps` passes.
// Usage: node tests/golden/time_reference.js [frames] [reps] [/root/reference/modem.js]
'use strict';
const vm = require('vm');
const fs = require('fs');
const NF = +(process.argv[2] || 40), REPS = +(process.argv[3] || 7);
const REF = process.argv[4] || '/root/reference/modem.js';
vm.runInThisContext(fs.readFileSync(REF, 'utf8'), { filename: 'modem.js' });

function xs32(s) { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; return s >>> 0; }
function payloadBytes(seed, len) {
  const out = new Uint8Array(len);
  let s = seed >>> 0;
  for (let i = 0; i < len; i++) {
    if ((i & 3) === 0) s = xs32(s);
    out[i] = (s >>> (8 * (i & 3))) & 0xff;
  }
  return out;
}
function median(a) { const b = a.slice().sort((x, y) => x - y); return b[b.length >> 1]; }

function timeIt(frames, decode, check) {
  for (const f of frames.slice(0, 3)) check(decode(f)); // warm-up + correctness
  const per = [];
  for (let r = 0; r < REPS; r++) {
    const t0 = process.hrtime.bigint();
    for (const f of frames) decode(f);
    per.push(Number(process.hrtime.bigint() - t0) / 1e6 / frames.length);
  }
  return median(per);
}

const out = {};
// C1/C2: legacy QPSK 1 KB frames (decodeReceivedSignal)
setOFDMConfig('standard');
let frames = [];
for (let i = 0; i < NF; i++) frames.push(buildTransmitSignal(payloadBytes((0x9E3779B9 ^ i) >>> 0, 1024), 'QPSK', 'f.bin', 1).signal);
out.c2 = { samples: frames[0].length, ms: timeIt(frames, f => decodeReceivedSignal(f, 'QPSK', 1), r => { if (!r.crcValid) throw new Error('c2'); }) };
// C3: legacy 16-QAM 1 KB frames
frames = [];
for (let i = 0; i < NF; i++) frames.push(buildTransmitSignal(payloadBytes((0x9E3779B9 ^ i) >>> 0, 1024), 'QAM16', 'f.bin', 1).signal);
out.c3 = { samples: frames[0].length, ms: timeIt(frames, f => decodeReceivedSignal(f, 'QAM16', 1), r => { if (!r.crcValid) throw new Error('c3'); }) };
// C4: 2 KB data-chunk windows from pre1 (decodeChunkFrame), as StreamingReceiver cuts them
frames = [];
const pre = Math.round(OFDM.SAMPLE_RATE * 0.05);
const win = estimateFrameSamples(2048 + 11, 'QPSK', 1);
for (let i = 0; i < NF; i++) {
  const f = buildDataChunkFrame(payloadBytes((0x9E3779B9 ^ i) >>> 0, 2048), i, 'QPSK', 1);
  frames.push(f.slice(pre, pre + win));
}
out.c4 = { samples: win, ms: timeIt(frames, f => decodeChunkFrame(f, 'QPSK', 1), r => { if (!r.crcValid) throw new Error('c4'); }) };
// C5: acoustic BPSK rep3 256 B frames (clean)
setOFDMConfig('acoustic');
frames = [];
for (let i = 0; i < Math.min(NF, 16); i++) frames.push(buildTransmitSignal(payloadBytes((0x9E3779B9 ^ i) >>> 0, 256), 'BPSK', 'f.bin', 3).signal);
out.c5 = { samples: frames[0].length, ms: timeIt(frames, f => decodeReceivedSignal(f, 'BPSK', 3), r => { if (!r.crcValid) throw new Error('c5'); }) };
out.node = process.version;
out.frames = NF;
out.reps = REPS;
console.log(JSON.stringify(out));
