#!/usr/bin/env node
// The Node.js host path of the drop-in (bench.py host_api leg): decodeBatch from the JS
// surface (audio-modem_amd/js/modem.js, N-API -> amod_decode_host), as app.js's callers
// (app.js:513, 928) would drive the engine with a whole batch, timed end to end (host
// Float32Array in, reference-shaped result objects out), and the native call alone.
// Usage: node tools/node_decode_batch.js <spec.json>
// spec: {samples: <float32 file>, offsets, lengths, preset, mod, rep, chunk, reps, device}
'use strict';
const fs = require('fs');
const path = require('path');
const modem = require(path.join(__dirname, '..', 'audio-modem_amd', 'js', 'modem.js'));

// a float32 file of any size into one Float32Array (a Node 12 Buffer stops at 2^31 - 1
// bytes, so fs.readFileSync cannot take a C4 shard or a C5 batch): 1 GB pieces read
// through views of the array's own buffer
function readF32(file) {
  const size = fs.statSync(file).size;
  const nb = size - (size % 4); // (no 32-bit bitwise ops on sizes past 2^31)
  const x = new Float32Array(nb / 4);
  const fd = fs.openSync(file, 'r');
  try {
    for (let pos = 0; pos < nb;) {
      const n = Math.min(1 << 30, nb - pos);
      const v = new Uint8Array(x.buffer, pos, n);
      for (let got = 0; got < n;) {
        const r = fs.readSync(fd, v, got, n - got, pos + got);
        if (r <= 0) throw new Error(`short read of ${file} at ${pos + got}`);
        got += r;
      }
      pos += n;
    }
  } finally {
    fs.closeSync(fd);
  }
  return x;
}

async function main() {
  const spec = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
  const say = (m) => process.stderr.write(`[node_decode_batch] ${m}\n`); // (progress: a crash names its step)
  const x = readF32(spec.samples);
  say(`read ${x.length} samples`);
  const offs = Float64Array.from(spec.offsets), lens = Int32Array.from(spec.lengths);
  modem.setOFDMConfig(spec.preset);
  const opts = { device: spec.device | 0, devices: 1, mode: spec.chunk ? 'chunk' : 'received' };
  const reps = spec.reps || 3;
  const med = (a) => a.slice().sort((p, q) => p - q)[a.length >> 1];
  const whole = [], nat = [];
  let res = null;
  say('decodeBatch');
  for (let r = 0; r <= reps; r++) {
    const t0 = process.hrtime.bigint();
    res = await modem.decodeBatch(x, offs, lens, spec.mod, spec.rep, opts);
    const t1 = process.hrtime.bigint();
    if (r) whole.push(Number(t1 - t0) / 1e6);
  }
  // the N-API call alone (records + payload ArrayBuffers, no per-frame result objects)
  const cfg = {
    fft_size: 512, cp_len: modem.OFDM.CP_LEN, symbol_len: modem.OFDM.SYMBOL_LEN, sample_rate: 44100,
    sub_start: modem.OFDM.SUB_START, sub_end: modem.OFDM.SUB_END, pilots: modem.OFDM.PILOTS.slice(),
    modulation: { BPSK: 0, QPSK: 1, QAM16: 2 }[spec.mod], repetition: spec.rep,
  };
  say('native.decodeAsync');
  const lib = [];
  for (let r = 0; r <= reps; r++) {
    const t0 = process.hrtime.bigint();
    const o = await modem.native.decodeAsync(x, offs, lens, cfg, spec.chunk ? 1 : 0, 0, spec.device | 0, 1);
    const t1 = process.hrtime.bigint();
    if (r) { nat.push(Number(t1 - t0) / 1e6); lib.push(o.nativeMs); }
  }
  // the batch made resident once (uploadBatch), then decodeBatch(DeviceBatch) from HBM:
  // launches, the D2H of records + payload rows and the result objects, no upload
  say('uploadBatch');
  const t0u = process.hrtime.bigint();
  const dbatch = modem.uploadBatch(x, offs, lens, spec.mod, spec.rep, { devices: 1 });
  const upload_ms = Number(process.hrtime.bigint() - t0u) / 1e6;
  say('decodeBatch(DeviceBatch)');
  const resd = [];
  let rres = null;
  for (let r = 0; r <= reps; r++) {
    const t0 = process.hrtime.bigint();
    rres = await modem.decodeBatch(dbatch, null, null, spec.mod, spec.rep, { mode: opts.mode });
    const t1 = process.hrtime.bigint();
    if (r) resd.push(Number(t1 - t0) / 1e6);
  }
  dbatch.free();
  const ok = res.filter((r) => r.crcValid === true).length;
  process.stdout.write(JSON.stringify({
    what: `decodeBatch(${lens.length} frames) from node ${process.version}: host Float32Array -> N-API -> ` +
      'amod_decode_host -> result objects (fresh data arrays, as the reference), median of ' + reps,
    ms: med(whole), native_call_ms: med(nat), library_call_ms: med(lib), frames: lens.length, frames_crc_valid: ok,
    resident: {
      what: 'uploadBatch once, then decodeBatch(DeviceBatch): amod_resident_decode from HBM + D2H + result objects',
      upload_ms, ms: med(resd), frames_crc_valid: rres.filter((r) => r.crcValid === true).length,
    },
  }));
}

main().catch((e) => { process.stderr.write(String(e && e.stack || e)); process.exit(1); });
