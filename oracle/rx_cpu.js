'use strict';
// rx_cpu.js — CPU BASELINE / TEST INFRASTRUCTURE ONLY (like everything under oracle/):
// a plain-JavaScript restatement of the reference receive chain, the CPU path
// BASELINE.md ("CPU-baseline plan") asks to time on the GPU box's host cores with one
// worker_thread per core. The reference source never travels to the GPU box, so this
// file stands in for it there; it is pinned bit-exactly to the golden fixtures
// (tests/test_cpu_js_baseline.py) and its single-core speed is calibrated against the
// unmodified modem.js in the build container (tools/calibrate_cpu.py).
//
// It restates, in IEEE double with the reference's operation order:
//   preprocessSignal      modem.js:213-232    detectPreamble  modem.js:286-319
//   fine cross-corr       modem.js:566-588    estimateChannel modem.js:421-440
//   fft / ifft            modem.js:6-66       demodulateOFDM  modem.js:365-418
//   constellations/demap  modem.js:107-150    majorityVote    modem.js:487-495
//   bitsToBytes / crc32   modem.js:443-476    templates       modem.js:153-208
//   decodeReceivedSignal  modem.js:557-654    decodeChunkFrame modem.js:770-803
//   meta / chunk parsers  modem.js:805-849
// The per-decode work is the reference's: templates are rebuilt on every decode and
// every symbol gets fresh spectra, as modem.js does, so the timing represents it.
//
// Usage (the bench's cpu_baseline leg and the tests drive it through a JSON spec):
//   node oracle/rx_cpu.js decode <spec.json>  -> JSON results, reference-shaped
//   node oracle/rx_cpu.js bench  <spec.json>  -> JSON rates (single core, all cores)
// spec: {samples: <float32 file>, offsets: [...], lengths: [...], preset, mod, rep,
//        chunk: bool, threads, seconds}

const fs = require('fs');
const os = require('os');
const util = require('util');

const PRESETS = {
  standard: { cp: 64, s0: 12, s1: 232, pilots: [15, 29, 43, 57, 71, 85, 99, 113, 127, 141, 155, 169, 183, 197, 211, 225] },
  acoustic: { cp: 128, s0: 23, s1: 93, pilots: [25, 35, 45, 55, 65, 75, 85] },
  narrowband: { cp: 256, s0: 35, s1: 58, pilots: [37, 45, 53] },
};
const N = 512;

function configFor(name) { // setOFDMConfig: unknown names mean 'standard' (modem.js:95-98)
  const p = PRESETS[name] || PRESETS.standard;
  return { cp: p.cp, sym: N + p.cp, s0: p.s0, s1: p.s1, pilots: p.pilots };
}

// ------------------------------------------------------------------- points --
const BPS = { BPSK: 1, QPSK: 2, QAM16: 4 };
function pointsOf(mod) { // initConstellation (modem.js:107-131)
  if (mod === 'BPSK') return [[1, 0], [-1, 0]];
  if (mod === 'QPSK') {
    const a = 1 / Math.SQRT2;
    return [[a, a], [-a, a], [-a, -a], [a, -a]];
  }
  if (mod !== 'QAM16') throw new TypeError(`unknown modulation ${mod}`);
  const grid = [];
  let e = 0;
  for (let i = 0; i < 16; i++) {
    const r = i >> 2, c = i & 3;
    const x = 2 * (c ^ (c >> 1)) - 3, y = 2 * (r ^ (r >> 1)) - 3;
    grid.push([x, y]);
    e += x * x + y * y;
  }
  const g = 1 / Math.sqrt(e / 16);
  return grid.map((p) => [p[0] * g, p[1] * g]);
}

// ----------------------------------------------------------------- transform --
// radix-2 decimation in time after a bit-reversal permutation; every stage restarts the
// twiddle recurrence w <- w * wn per butterfly group (modem.js:26-66)
function transform(re, im, inverse) {
  const n = re.length;
  let lg = 0;
  while ((1 << lg) < n) lg++;
  for (let i = 0; i < n; i++) {
    let j = 0;
    for (let b = 0, v = i; b < lg; b++, v >>= 1) j = (j << 1) | (v & 1);
    if (j > i) {
      let t = re[i]; re[i] = re[j]; re[j] = t;
      t = im[i]; im[i] = im[j]; im[j] = t;
    }
  }
  for (let len = 2; len <= n; len <<= 1) {
    const h = len >> 1;
    const ang = (inverse ? 1 : -1) * 2 * Math.PI / len;
    const cr = Math.cos(ang), ci = Math.sin(ang);
    for (let b = 0; b < n; b += len) {
      let wr = 1, wi = 0;
      for (let k = 0; k < h; k++) {
        const p = b + k, q = p + h;
        const xr = wr * re[q] - wi * im[q];
        const xi = wr * im[q] + wi * re[q];
        re[q] = re[p] - xr; im[q] = im[p] - xi;
        re[p] += xr; im[p] += xi;
        const t = wr * cr - wi * ci;
        wi = wr * ci + wi * cr;
        wr = t;
      }
    }
  }
}

function spectrumOf(src, from) { // FFT of 512 real samples (missing / NaN samples read 0)
  const re = new Float64Array(N), im = new Float64Array(N);
  for (let i = 0; i < N; i++) re[i] = src[from + i] || 0;
  const r = Float64Array.from(re), m = Float64Array.from(im);
  transform(r, m, false);
  return [r, m];
}

// -------------------------------------------------------------- templates --
// seededRandom (modem.js:153-156): the product is a double, then ToInt32
function lcg(seed) {
  let s = seed;
  return () => { s = (s * 1103515245 + 12345) & 0x7fffffff; return s / 0x7fffffff; };
}

// a template symbol: +-1 on k = s0 .. s1 (step), Hermitian, IFFT, cyclic prefix (float32)
function templateSymbol(cfg, seed, step, known) {
  const re = new Float64Array(N), im = new Float64Array(N);
  const rnd = lcg(seed);
  for (let k = cfg.s0; k <= cfg.s1; k += step) {
    re[k] = rnd() > 0.5 ? 1 : -1;
    if (known) known[k] = re[k];
  }
  for (let k = 1; k < N / 2; k++) { re[N - k] = re[k]; im[N - k] = -im[k]; }
  re[0] = 0; re[N / 2] = 0; im[N / 2] = 0;
  const tr = Float64Array.from(re), ti = Float64Array.from(im);
  transform(tr, ti, true);
  const sc = 1 / N;
  for (let i = 0; i < N; i++) { tr[i] *= sc; ti[i] *= sc; }
  const out = new Float32Array(cfg.sym);
  for (let i = 0; i < cfg.cp; i++) out[i] = tr[N - cfg.cp + i];
  for (let i = 0; i < N; i++) out[cfg.cp + i] = tr[i];
  return out;
}

// ------------------------------------------------------------------ stages --
function normalise(x) { // preprocessSignal (modem.js:213-232)
  let mean = 0;
  for (let i = 0; i < x.length; i++) mean += x[i];
  mean /= x.length;
  const y = new Float32Array(x.length);
  let peak = 0;
  for (let i = 0; i < x.length; i++) {
    y[i] = x[i] - mean;
    peak = Math.max(peak, Math.abs(y[i]));
  }
  if (peak > 1e-6) for (let i = 0; i < y.length; i++) y[i] /= peak;
  return y;
}

function schmidlCox(y) { // detectPreamble (modem.js:286-319)
  const half = N / 2, n = y.length;
  if (n < 2 * half) return -1;
  let p = 0, ea = 0, eb = 0;
  for (let m = 0; m < half; m++) {
    const a = y[m], b = y[m + half];
    p += a * b; ea += a * a; eb += b * b;
  }
  let best = 0, at = -1;
  const last = n - 2 * half;
  for (let d = 0; d <= last; d++) {
    if (ea > 0.01 && eb > 0.01) {
      const v = (p * p) / (ea * eb);
      if (v > best) { best = v; at = d; }
    }
    if (d < last) {
      const o = y[d], mid = y[d + half], inc = y[d + 2 * half];
      p += mid * inc - o * mid;
      ea += mid * mid - o * o;
      eb += inc * inc - mid * mid;
    }
  }
  return best > 0.5 ? at : -1;
}

function fineTiming(cfg, y, coarse) { // modem.js:566-588
  const t = templateSymbol(cfg, 42, 2, null);
  let te = 0;
  for (let i = 0; i < t.length; i++) te += t[i] * t[i];
  const lo = Math.max(0, coarse - 3 * cfg.cp), hi = Math.min(y.length - t.length, coarse + 3 * cfg.cp);
  let best = -Infinity, at = coarse;
  for (let d = lo; d <= hi; d++) {
    let c = 0, e = 0;
    for (let i = 0; i < t.length; i++) {
      c += y[d + i] * t[i];
      e += y[d + i] * y[d + i];
    }
    const den = Math.sqrt(e * te);
    if (den > 0.001) {
      const v = c / den;
      if (v > best) { best = v; at = d; }
    }
  }
  return [at, best];
}

function channel(cfg, ce) { // estimateChannel with the CE symbol's known signs (modem.js:421-440)
  const known = new Float64Array(N), knownIm = new Float64Array(N);
  templateSymbol(cfg, 44, 1, known);
  const [yr, yi] = spectrumOf(ce, cfg.cp);
  const hr = new Float64Array(N), hi = new Float64Array(N);
  for (let k = cfg.s0; k <= cfg.s1; k++) {
    const xr = known[k], xi = knownIm[k];
    const d = xr * xr + xi * xi;
    if (d > 1e-10) {
      hr[k] = (yr[k] * xr + yi[k] * xi) / d;
      hi[k] = (yi[k] * xr - yr[k] * xi) / d;
    }
  }
  return [hr, hi];
}

// constellationDemap (modem.js:140-150): the first strict minimum, its bits MSB first
function nearest(pts, bps, u, v) {
  let dmin = Infinity, idx = 0;
  for (let i = 0; i < pts.length; i++) {
    const dr = u - pts[i][0], di = v - pts[i][1];
    const dd = dr * dr + di * di;
    if (dd < dmin) { dmin = dd; idx = i; }
  }
  const out = [];
  for (let b = bps - 1; b >= 0; b--) out.push((idx >> b) & 1);
  return out;
}

function demodulate(cfg, data, mod, hr, hi) { // demodulateOFDM (modem.js:365-418)
  const pts = pointsOf(mod), bps = BPS[mod];
  const nsym = Math.floor(data.length / cfg.sym);
  const bits = [];
  for (let s = 0; s < nsym; s++) {
    const [yr, yi] = spectrumOf(data, s * cfg.sym + cfg.cp);
    const er = new Float64Array(N), ei = new Float64Array(N);
    for (let k = cfg.s0; k <= cfg.s1; k++) {
      const a = hr[k], b = hi[k], g = a * a + b * b;
      if (g > 1e-10) {
        er[k] = (yr[k] * a + yi[k] * b) / g;
        ei[k] = (yi[k] * a - yr[k] * b) / g;
      } else {
        er[k] = yr[k]; ei[k] = yi[k];
      }
    }
    let acc = 0, cnt = 0;
    for (const p of cfg.pilots) {
      if (p >= cfg.s0 && p <= cfg.s1 && Math.abs(er[p]) > 1e-6) { acc += ei[p] / er[p]; cnt++; }
    }
    const ph = cnt > 0 ? acc / cnt : 0;
    for (let k = cfg.s0; k <= cfg.s1; k++) {
      if (cfg.pilots.includes(k)) continue; // OFDM.isPilot, as the reference tests it
      bits.push(...nearest(pts, bps, er[k] + ei[k] * ph, ei[k] - er[k] * ph));
    }
  }
  return bits;
}

function vote(bits, n) { // majorityVote (modem.js:487-495)
  const out = [];
  for (let i = 0; i + n - 1 < bits.length; i += n) {
    let s = 0;
    for (let j = 0; j < n; j++) s += bits[i + j];
    out.push(s >= n / 2 ? 1 : 0);
  }
  return out;
}

function pack(bits) { // bitsToBytes (modem.js:468-476)
  const out = new Uint8Array(bits.length >> 3);
  for (let i = 0, o = 0; i + 7 < bits.length; i += 8, o++) {
    let b = 0;
    for (let j = 0; j < 8; j++) b = (b << 1) | (bits[i + j] & 1);
    out[o] = b;
  }
  return out;
}

const CRC_T = new Uint32Array(256);
for (let i = 0; i < 256; i++) {
  let c = i;
  for (let j = 0; j < 8; j++) c = (c & 1) ? (0xEDB88320 ^ (c >>> 1)) : (c >>> 1);
  CRC_T[i] = c;
}
function crc32(bytes, end) { // modem.js:443-457 over bytes[0, end)
  let c = 0xFFFFFFFF;
  for (let i = 0; i < end; i++) c = CRC_T[(c ^ bytes[i]) & 0xFF] ^ (c >>> 8);
  return (c ^ 0xFFFFFFFF) >>> 0;
}

// ---------------------------------------------------------------- parsing --
const be32 = (b, o) => (b[o] << 24) | (b[o + 1] << 16) | (b[o + 2] << 8) | b[o + 3];
const TD = new util.TextDecoder();
const text = (b) => { try { return TD.decode(b); } catch (e) { return ''; } };

function withCrc(res, bytes, off) {
  res.expectedCRC = be32(bytes, off) >>> 0;
  res.actualCRC = crc32(bytes, off);
  res.crcValid = res.expectedCRC === res.actualCRC;
  return res;
}

function parseMeta(bytes) { // parseMetadataResult (modem.js:805-828)
  if (bytes.length < 16) return { error: 'Metadata frame too short', code: 8 };
  const nl = bytes[11];
  if (12 + nl + 4 > bytes.length) return { error: 'Metadata frame truncated', code: 9 };
  return withCrc({
    frameType: 0xFE, totalChunks: be32(bytes, 1), totalFileSize: be32(bytes, 5),
    chunkSize: (bytes[9] << 8) | bytes[10], fileName: text(bytes.slice(12, 12 + nl)),
  }, bytes, 12 + nl);
}

function parseChunk(bytes) { // parseDataChunkResult (modem.js:830-849)
  if (bytes.length < 11) return { error: 'Data chunk frame too short', code: 10 };
  const len = (bytes[5] << 8) | bytes[6];
  if (7 + len + 4 > bytes.length) return { error: 'Data chunk truncated', code: 11 };
  return withCrc({ frameType: 0xFF, seqNum: be32(bytes, 1), data: bytes.slice(7, 7 + len), dataLen: len },
    bytes, 7 + len);
}

function parseLegacy(bytes, at) { // modem.js:622-653
  const nl = bytes[0];
  if (1 + nl + 8 > bytes.length) return { error: 'Decoded data too short for header', code: 6 };
  const name = text(bytes.slice(1, 1 + nl));
  const len = be32(bytes, 1 + nl);
  const d0 = 5 + nl;
  if (len <= 0 || d0 + len + 4 > bytes.length) return { error: `Invalid data length: ${len}`, code: 7, aux: len };
  const r = withCrc({ data: bytes.slice(d0, d0 + len), dataLen: len, fileName: name }, bytes, d0 + len);
  r.preambleIdx = at;
  r.frameType = 'legacy';
  return r;
}

// symbols after the CE at `ce` -> payload bytes
function payloadBytes(cfg, y, ce, mod, rep) {
  const [hr, hi] = channel(cfg, y.slice(ce, ce + cfg.sym));
  let bits = demodulate(cfg, y.slice(ce + cfg.sym), mod, hr, hi);
  if (rep > 1) bits = vote(bits, rep);
  return pack(bits);
}

// decodeReceivedSignal (modem.js:557-654)
function decodeReceived(cfg, x, mod, rep) {
  rep = rep || 1;
  const y = normalise(x);
  const coarse = schmidlCox(y);
  if (coarse < 0) return { error: 'Preamble not detected', code: 1 };
  const [at, best] = fineTiming(cfg, y, coarse);
  if (best < 0.1) return { error: 'Preamble not detected (low correlation)', code: 2 };
  const ce = at + 2 * cfg.sym;
  if (ce + cfg.sym > y.length) return { error: 'Signal too short for CE', code: 3 };
  if (ce + cfg.sym >= y.length) return { error: 'No data after CE', code: 4 };
  const bytes = payloadBytes(cfg, y, ce, mod, rep);
  if (bytes.length < 10) return { error: 'Decoded data too short', code: 5 };
  if (bytes[0] === 0xFE || bytes[0] === 0xFF) {
    const r = bytes[0] === 0xFE ? parseMeta(bytes) : parseChunk(bytes);
    r.preambleIdx = at;
    return r;
  }
  return parseLegacy(bytes, at);
}

// decodeChunkFrame (modem.js:770-803): the frame starts at pre1, no preprocessing
function decodeChunk(cfg, x, mod, rep) {
  rep = rep || 1;
  const ce = 2 * cfg.sym;
  if (ce + cfg.sym > x.length) return { error: 'Frame too short for CE', code: 12 };
  if (ce + cfg.sym >= x.length) return { error: 'No data after CE', code: 4 };
  const bytes = payloadBytes(cfg, x, ce, mod, rep);
  if (bytes.length < 6) return { error: 'Decoded data too short', code: 5 };
  if (bytes[0] === 0xFE) return parseMeta(bytes);
  if (bytes[0] === 0xFF) return parseChunk(bytes);
  return { error: `Unknown frame type: 0x${bytes[0].toString(16)}`, frameType: bytes[0], code: 13 };
}

// ------------------------------------------------------------------- driver --
function loadSamples(spec) {
  const buf = fs.readFileSync(spec.samples);
  const sab = new SharedArrayBuffer(buf.length);
  new Uint8Array(sab).set(buf);
  return sab;
}

function outcome(r) { return [r.error ? r.code : 0, r.error ? 0 : r.actualCRC]; }

// decode the frames this worker owns (i = first, first + step, ...) for `seconds`
function runShare(spec, sab, first, step) {
  const x = new Float32Array(sab);
  const cfg = configFor(spec.preset);
  const dec = spec.chunk ? decodeChunk : decodeReceived;
  const own = [];
  for (let i = first; i < spec.offsets.length; i += step) own.push(i);
  const codes = [], crcs = [];
  let samples = 0, passes = 0;
  const t0 = process.hrtime.bigint();
  let el = 0;
  do {
    for (const i of own) {
      const r = dec(cfg, x.subarray(spec.offsets[i], spec.offsets[i] + spec.lengths[i]), spec.mod, spec.rep);
      if (passes === 0) { const [c, k] = outcome(r); codes.push([i, c]); crcs.push(k); }
      samples += spec.lengths[i];
    }
    passes++;
    el = Number(process.hrtime.bigint() - t0) / 1e9;
  } while (el < (spec.seconds || 0) && own.length);
  return { samples, seconds: el, passes, codes, crcs };
}

function pool(spec, sab, threads) {
  const { Worker } = require('worker_threads');
  return new Promise((resolve, reject) => {
    const out = new Array(threads);
    let left = threads;
    const t0 = process.hrtime.bigint();
    for (let w = 0; w < threads; w++) {
      const wk = new Worker(__filename, { workerData: { spec, sab, first: w, step: threads } });
      wk.on('message', (m) => {
        out[w] = m;
        if (--left === 0) resolve({ parts: out, wall: Number(process.hrtime.bigint() - t0) / 1e9 });
      });
      wk.on('error', reject);
    }
  });
}

async function bench(spec) {
  const sab = loadSamples(spec);
  const threads = Math.max(1, spec.threads || os.cpus().length);
  // one core: the first frames, for spec.single_seconds
  const one = runShare(Object.assign({}, spec, { offsets: spec.offsets.slice(0, spec.single_frames || 200),
    lengths: spec.lengths.slice(0, spec.single_frames || 200), seconds: spec.single_seconds || 1 }), sab, 0, 1);
  const all = await pool(spec, sab, threads);
  const samples = all.parts.reduce((s, p) => s + p.samples, 0);
  const status = new Array(spec.offsets.length).fill(-1), crc = new Array(spec.offsets.length).fill(0);
  for (const p of all.parts) p.codes.forEach(([i, c], j) => { status[i] = c; crc[i] = p.crcs[j]; });
  return {
    threads, cores: os.cpus().length, node: process.version,
    single_core: one.samples / one.seconds, single_core_seconds: one.seconds, single_core_frames: one.codes.length,
    all_cores: samples / all.wall, all_cores_seconds: all.wall, all_cores_samples: samples,
    passes: all.parts.map((p) => p.passes), status, crc,
  };
}

function toJson(r) { // Uint8Array fields as {hex} (the golden fixtures' shape)
  const o = {};
  for (const [k, v] of Object.entries(r)) {
    if (k === 'code' || k === 'aux') continue;
    o[k] = v instanceof Uint8Array ? { hex: Buffer.from(v).toString('hex') } : v;
  }
  return o;
}

const wt = require('worker_threads');
if (!wt.isMainThread && wt.workerData && wt.workerData.spec) {
  const { spec, sab, first, step } = wt.workerData;
  wt.parentPort.postMessage(runShare(spec, sab, first, step));
} else if (require.main === module) {
  const [cmd, file] = process.argv.slice(2);
  const spec = JSON.parse(fs.readFileSync(file, 'utf8'));
  if (cmd === 'decode') {
    const x = new Float32Array(loadSamples(spec));
    const res = spec.offsets.map((o, i) => {
      const f = x.subarray(o, o + spec.lengths[i]);
      const pick = (many, one) => (many ? many[i] : one);
      const cfg = configFor(pick(spec.presets, spec.preset));
      const dec = pick(spec.chunks, spec.chunk) ? decodeChunk : decodeReceived;
      return toJson(dec(cfg, f, pick(spec.mods, spec.mod), pick(spec.reps, spec.rep)));
    });
    process.stdout.write(JSON.stringify(res));
  } else if (cmd === 'bench') {
    bench(spec).then((r) => process.stdout.write(JSON.stringify(r)));
  } else {
    process.stderr.write('usage: rx_cpu.js decode|bench <spec.json>\n');
    process.exit(2);
  }
}

module.exports = { configFor, decodeReceived, decodeChunk, transform, crc32 };
