#!/usr/bin/env node
// Single-thread timing of the receive path on identical frames (build container only,
// since it loads the unmodified reference): the reference modem.js (vm.runInThisContext)
// and the JS CPU baseline oracle/rx_cpu.js, interleaved pass by pass so machine drift hits
// both alike. Prints JSON {ref_ms, js_ms} per frame (medians over reps).
// Usage: node tools/time_rx.js <spec.json> [reps] [/root/reference/modem.js]
// spec: {samples, offsets, lengths, preset, mod, rep, chunk} as for rx_cpu.js
'use strict';
const fs = require('fs');
const path = require('path');
const vm = require('vm');
const js = require(path.join(__dirname, '..', 'oracle', 'rx_cpu.js'));

const spec = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const REPS = +(process.argv[3] || 9);
vm.runInThisContext(fs.readFileSync(process.argv[4] || '/root/reference/modem.js', 'utf8'), { filename: 'modem.js' });
setOFDMConfig(spec.preset);

const all = new Float32Array(fs.readFileSync(spec.samples).buffer.slice(0));
const frames = spec.offsets.map((o, i) => all.slice(o, o + spec.lengths[i]));
const cfg = js.configFor(spec.preset);
const ref = (f) => (spec.chunk ? decodeChunkFrame(f, spec.mod, spec.rep) : decodeReceivedSignal(f, spec.mod, spec.rep));
const mine = (f) => (spec.chunk ? js.decodeChunk(cfg, f, spec.mod, spec.rep) : js.decodeReceived(cfg, f, spec.mod, spec.rep));

function pass(fn) {
  const t0 = process.hrtime.bigint();
  for (const f of frames) fn(f);
  return Number(process.hrtime.bigint() - t0) / 1e6 / frames.length;
}
for (const f of frames.slice(0, 4)) {
  const a = ref(f), b = mine(f);
  if (a.actualCRC !== b.actualCRC || a.error !== b.error) throw new Error('outcomes differ');
}
pass(ref); pass(mine); // warm-up passes
const tr = [], tj = [];
for (let r = 0; r < REPS; r++) { tr.push(pass(ref)); tj.push(pass(mine)); }
const med = (a) => a.slice().sort((x, y) => x - y)[a.length >> 1];
console.log(JSON.stringify({ ref_ms: med(tr), js_ms: med(tj), frames: frames.length, reps: REPS, node: process.version }));
