#!/usr/bin/env node
// Golden-vector generator (test infrastructure, runs ONLY in the build container).
//
// Loads the UNMODIFIED reference /root/reference/modem.js with vm.runInThisContext
// and records its outputs on deterministic synthetic inputs. Nothing from the
// reference source is written out: only inputs (as recipes), hashes and the
// reference's outputs.  The recipes (payload PRNG, noise, slicing) are defined
// here and restated bit-exactly by oracle/ and by the product TX so the GPU box
// (which has no reference) can rebuild every signal and check its SHA-256.
//
// Usage: node tests/golden/gen_golden.js [/root/reference/modem.js]
'use strict';
const vm = require('vm');
const fs = require('fs');
const path = require('path');
const crypto = require('crypto');

const REF = process.argv[2] || '/root/reference/modem.js';
vm.runInThisContext(fs.readFileSync(REF, 'utf8'), { filename: 'modem.js' });
const OUT = __dirname;

// ---------------------------------------------------------------- recipes --
// xorshift32 (Marsaglia 13/17/5); uint32 state, never 0.
function xs32(s) {
  s ^= s << 13; s >>>= 0;
  s ^= s >>> 17;
  s ^= s << 5; s >>>= 0;
  return s;
}
// payload bytes: state = seed; every 4 bytes advance once, emit little-endian.
function payloadBytes(seed, len) {
  const out = new Uint8Array(len);
  let s = seed >>> 0;
  for (let i = 0; i < len; i++) {
    if ((i & 3) === 0) s = xs32(s);
    out[i] = (s >>> (8 * (i & 3))) & 0xff;
  }
  return out;
}
function frameSeed(idx) { return (0x9E3779B9 ^ idx) >>> 0; }

// Noise: sigma^2 = P_active / 10^(snr/10) with snr in {10,20,30} (exact divisor);
// g = (sum of 12 uniforms u = x/2^32) - 6 ; y = fround(s + sigma*g).
// (or an explicit divisor `div`, a dyadic/small-integer value, for in-between SNRs)
function addNoise(sig, snrDb, seed, divOverride) {
  let p = 0, cnt = 0;
  for (let i = 0; i < sig.length; i++) { const v = sig[i]; if (v !== 0) { p += v * v; cnt++; } }
  p = cnt > 0 ? p / cnt : 0;
  let div = 1; for (let k = 0; k < snrDb / 10; k++) div *= 10;
  if (divOverride !== undefined) div = divOverride;
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
function addDC(sig, dc) {
  const out = new Float32Array(sig.length);
  for (let i = 0; i < sig.length; i++) out[i] = Math.fround(sig[i] + dc);
  return out;
}
// one period of a tone, stored in the recipe itself so no libm call is needed to rebuild it
function tonePeriod(period, bin, amp) {
  return Array.from({ length: period }, (_, i) => Math.fround(amp * Math.cos(2 * Math.PI * bin * i / period)));
}
function tile(n, values) {
  const out = new Float32Array(n);
  for (let i = 0; i < n; i++) out[i] = values[i % values.length];
  return out;
}

function buildTx(tx) {
  switch (tx.kind) {
    case 'legacy': {
      const data = payloadBytes(tx.seed, tx.len);
      return buildTransmitSignal(data, tx.mod, tx.name, tx.rep).signal;
    }
    case 'meta':
      return buildMetadataFrame(tx.totalChunks, tx.totalFileSize, tx.chunkSize, tx.name, tx.mod, tx.rep);
    case 'chunk':
      return buildDataChunkFrame(payloadBytes(tx.seed, tx.len), tx.seq, tx.mod, tx.rep);
    case 'test':
      return generateTestSignal(tx.mod, tx.rep).signal;
    case 'zeros':
      return new Float32Array(tx.n);
    case 'periodic':
      return tile(tx.n, tx.values);
    default: throw new Error('bad tx kind ' + tx.kind);
  }
}
function applyPost(sig, post) {
  for (const op of post || []) {
    if (op.op === 'slice') sig = sig.slice(op.start, op.end);
    else if (op.op === 'noise') sig = addNoise(sig, op.snr, op.seed, op.div);
    else if (op.op === 'dc') sig = addDC(sig, op.dc);
    else throw new Error('bad post op');
  }
  return sig;
}

// ---------------------------------------------------------------- helpers --
const hex = (u8) => Buffer.from(u8.buffer, u8.byteOffset, u8.byteLength).toString('hex');
const sha = (ta) => crypto.createHash('sha256').update(Buffer.from(ta.buffer, ta.byteOffset, ta.byteLength)).digest('hex');
const arr = (ta) => Array.from(ta);
function packBits(bits) {
  const out = new Uint8Array((bits.length + 7) >> 3);
  for (let i = 0; i < bits.length; i++) if (bits[i]) out[i >> 3] |= 0x80 >> (i & 7);
  return out;
}
function jsonResult(r) {
  const o = {};
  for (const k of Object.keys(r)) {
    const v = r[k];
    o[k] = (v instanceof Uint8Array) ? { hex: hex(v) } : v;
  }
  return o;
}

// Intermediates of the receive chain, using the reference's own functions for
// every stage that is a function; the inline fine search and the per-symbol
// equaliser are restated here only to expose their intermediate values (their
// end products are cross-checked against demodulateOFDM / decodeReceivedSignal).
function bandOf(a) { return arr(a.subarray(OFDM.SUB_START, OFDM.SUB_END + 1)); }
function symbolDetail(data, s, chRe, chIm) {
  const N = OFDM.FFT_SIZE, off = s * OFDM.SYMBOL_LEN;
  const re = new Float64Array(N), im = new Float64Array(N);
  for (let i = 0; i < N; i++) re[i] = data[off + OFDM.CP_LEN + i] || 0;
  const [Xr, Xi] = fft(re, im);
  const er = new Float64Array(N), ei = new Float64Array(N);
  for (let k = OFDM.SUB_START; k <= OFDM.SUB_END; k++) {
    const hr = chRe[k], hi = chIm[k], m = hr * hr + hi * hi;
    if (m > 1e-10) { er[k] = (Xr[k] * hr + Xi[k] * hi) / m; ei[k] = (Xi[k] * hr - Xr[k] * hi) / m; }
    else { er[k] = Xr[k]; ei[k] = Xi[k]; }
  }
  let ps = 0, pc = 0;
  for (const p of OFDM.PILOTS) if (p >= OFDM.SUB_START && p <= OFDM.SUB_END && Math.abs(er[p]) > 1e-6) { ps += ei[p] / er[p]; pc++; }
  return { Xr, Xi, er, ei, phase: pc > 0 ? ps / pc : 0 };
}
function rxDetail(data, chRe, chIm, mod, rep) {
  const nsym = Math.floor(data.length / OFDM.SYMBOL_LEN);
  const phases = [];
  const det = {};
  for (let s = 0; s < nsym; s++) {
    const d = symbolDetail(data, s, chRe, chIm);
    phases.push(d.phase);
    if (s < 2) det['sym' + s] = { fftRe: bandOf(d.Xr), fftIm: bandOf(d.Xi), eqRe: bandOf(d.er), eqIm: bandOf(d.ei) };
  }
  const bits = demodulateOFDM(data, mod, chRe, chIm);
  let vb = bits;
  if (rep > 1) vb = majorityVote(bits, rep);
  const bytes = bitsToBytes(vb);
  return {
    numSymbols: nsym, phases, ...det,
    H: { re: bandOf(chRe), im: bandOf(chIm) },
    nbits: bits.length, bitsHex: hex(packBits(bits)),
    nvoted: vb.length, bytesHex: hex(bytes),
  };
}

function legacyIntermediates(raw, mod, rep) {
  const out = {};
  let mean = 0;
  for (let i = 0; i < raw.length; i++) mean += raw[i];
  mean /= raw.length;
  const sig = preprocessSignal(raw);
  out.mean = mean;
  out.preSha = sha(sig);
  if (raw.length > 0) {
    let mx = 0;
    for (let i = 0; i < raw.length; i++) mx = Math.max(mx, Math.abs(Math.fround(raw[i] - mean)));
    out.mx = mx;
  }
  const coarse = detectPreamble(sig);
  out.coarseIdx = coarse;
  if (coarse < 0) return out;
  const pre1 = generatePreambleSymbol1();
  let tE = 0; for (let i = 0; i < pre1.length; i++) tE += pre1[i] * pre1[i];
  const R = OFDM.CP_LEN * 3;
  const fs_ = Math.max(0, coarse - R), fe = Math.min(sig.length - pre1.length, coarse + R);
  let best = -Infinity, start = coarse;
  for (let d = fs_; d <= fe; d++) {
    let c = 0, e = 0;
    for (let i = 0; i < pre1.length; i++) { c += sig[d + i] * pre1[i]; e += sig[d + i] * sig[d + i]; }
    const den = Math.sqrt(e * tE);
    if (den > 0.001) { const m = c / den; if (m > best) { best = m; start = d; } }
  }
  out.fineStart = fs_; out.fineEnd = fe;
  out.fineMetric = best === -Infinity ? null : best;
  out.startIdx = start;
  if (best < 0.1) return out;
  const ceStart = start + 2 * OFDM.SYMBOL_LEN;
  if (ceStart + OFDM.SYMBOL_LEN > sig.length) return out;
  const ce = generateChannelEstSymbol();
  const [chRe, chIm] = estimateChannel(sig.slice(ceStart, ceStart + OFDM.SYMBOL_LEN), ce.knownRe, ce.knownIm);
  const dataStart = ceStart + OFDM.SYMBOL_LEN;
  if (dataStart >= sig.length) { out.H = { re: bandOf(chRe), im: bandOf(chIm) }; return out; }
  Object.assign(out, rxDetail(sig.slice(dataStart), chRe, chIm, mod, rep));
  return out;
}
function chunkIntermediates(frame, mod, rep) {
  const ceStart = 2 * OFDM.SYMBOL_LEN;
  if (ceStart + OFDM.SYMBOL_LEN > frame.length) return {};
  const ce = generateChannelEstSymbol();
  const [chRe, chIm] = estimateChannel(frame.slice(ceStart, ceStart + OFDM.SYMBOL_LEN), ce.knownRe, ce.knownIm);
  const dataStart = ceStart + OFDM.SYMBOL_LEN;
  if (dataStart >= frame.length) return { H: { re: bandOf(chRe), im: bandOf(chIm) } };
  return rxDetail(frame.slice(dataStart), chRe, chIm, mod, rep);
}

// ------------------------------------------------------------------ cases --
const SYM = { standard: 576, acoustic: 640, narrowband: 768 };
function silencePre(cfg, first) {
  const ac = cfg !== 'standard';
  return first ? Math.round(44100 * (ac ? 0.5 : 0.3)) : Math.round(44100 * 0.05);
}
const cases = [];
function add(name, config, tx, post, rx, mod, rep, opts) {
  cases.push({ name, config, tx, post: post || [], rx, mod, rep, ...(opts || {}) });
}
// Full legacy frames (decodeReceivedSignal) — BASELINE C1/C2, C3, C5 and more.
add('std_qpsk_1k', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
add('std_qpsk_1k_f7', 'standard', { kind: 'legacy', seed: frameSeed(7), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
add('std_qam16_1k', 'standard', { kind: 'legacy', seed: frameSeed(1), len: 1024, name: 'f.bin', mod: 'QAM16', rep: 1 }, [], 'legacy', 'QAM16', 1);
add('std_bpsk_64', 'standard', { kind: 'legacy', seed: frameSeed(2), len: 64, name: 'b.dat', mod: 'BPSK', rep: 1 }, [], 'legacy', 'BPSK', 1);
add('std_qpsk_rep3_100', 'standard', { kind: 'legacy', seed: frameSeed(3), len: 100, name: 'r3', mod: 'QPSK', rep: 3 }, [], 'legacy', 'QPSK', 3);
add('ac_bpsk_64', 'acoustic', { kind: 'legacy', seed: frameSeed(4), len: 64, name: 'a.txt', mod: 'BPSK', rep: 1 }, [], 'legacy', 'BPSK', 1);
add('ac_bpsk_rep3_256', 'acoustic', { kind: 'legacy', seed: frameSeed(5), len: 256, name: 'f.bin', mod: 'BPSK', rep: 3 }, [], 'legacy', 'BPSK', 3);
add('ac_qpsk_200', 'acoustic', { kind: 'legacy', seed: frameSeed(6), len: 200, name: 'aq', mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
add('nb_bpsk_rep3_32', 'narrowband', { kind: 'legacy', seed: frameSeed(8), len: 32, name: 'n', mod: 'BPSK', rep: 3 }, [], 'legacy', 'BPSK', 3);
add('nb_bpsk_40', 'narrowband', { kind: 'legacy', seed: frameSeed(9), len: 40, name: 'nb', mod: 'BPSK', rep: 1 }, [], 'legacy', 'BPSK', 1);
add('utf8_name', 'standard', { kind: 'legacy', seed: frameSeed(10), len: 50, name: '파일-é.bin', mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
// In-app pre-test signals (generateTestSignal), incl. the narrowband rep3 reference bug.
add('test_std_qpsk', 'standard', { kind: 'test', mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
add('test_std_qam16', 'standard', { kind: 'test', mod: 'QAM16', rep: 1 }, [], 'legacy', 'QAM16', 1);
add('test_ac_bpsk', 'acoustic', { kind: 'test', mod: 'BPSK', rep: 1 }, [], 'legacy', 'BPSK', 1);
add('test_ac_bpsk_rep3', 'acoustic', { kind: 'test', mod: 'BPSK', rep: 3 }, [], 'legacy', 'BPSK', 3);
add('test_nb_bpsk_rep3', 'narrowband', { kind: 'test', mod: 'BPSK', rep: 3 }, [], 'legacy', 'BPSK', 3);
// Chunk protocol through decodeReceivedSignal (0xFE / 0xFF dispatch).
add('meta_via_legacy', 'standard', { kind: 'meta', totalChunks: 256000, totalFileSize: 524288000, chunkSize: 2048, name: 'big.bin', mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
add('chunk_via_legacy', 'standard', { kind: 'chunk', seq: 5, seed: frameSeed(11), len: 2048, mod: 'QPSK', rep: 1 }, [], 'legacy', 'QPSK', 1);
// decodeChunkFrame on windows that start at pre1 (BASELINE C4 shape).
{
  const sp = silencePre('standard', false);
  const w = 3 * 576 + Math.ceil((2048 + 11) * 8 / 410) * 576;
  add('chunk_2k_qpsk', 'standard', { kind: 'chunk', seq: 12345, seed: frameSeed(12), len: 2048, mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: sp, end: sp + w }], 'chunk', 'QPSK', 1);
  const wq = 3 * 576 + Math.ceil((4096 + 11) * 8 / 820) * 576;
  add('chunk_4k_qam16', 'standard', { kind: 'chunk', seq: 7, seed: frameSeed(13), len: 4096, mod: 'QAM16', rep: 1 }, [{ op: 'slice', start: sp, end: sp + wq }], 'chunk', 'QAM16', 1);
  add('chunk_last_short', 'standard', { kind: 'chunk', seq: 255999, seed: frameSeed(14), len: 1000, mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: sp }], 'chunk', 'QPSK', 1);
  const spm = silencePre('standard', true);
  add('meta_chunk', 'standard', { kind: 'meta', totalChunks: 3, totalFileSize: 5000, chunkSize: 2048, name: 'small.txt', mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: spm }], 'chunk', 'QPSK', 1);
  const spa = silencePre('acoustic', false);
  add('chunk_ac_bpsk_rep3', 'acoustic', { kind: 'chunk', seq: 3, seed: frameSeed(15), len: 512, mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: spa }], 'chunk', 'BPSK', 3);
  // legacy frame sliced at pre1 and fed to decodeChunkFrame -> 'Unknown frame type: 0x5'
  add('chunk_unknown_type', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: 13230 }], 'chunk', 'QPSK', 1);
  add('chunk_too_short_ce', 'standard', { kind: 'chunk', seq: 1, seed: frameSeed(16), len: 100, mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: sp, end: sp + 3 * 576 - 1 }], 'chunk', 'QPSK', 1);
  add('chunk_no_data', 'standard', { kind: 'chunk', seq: 1, seed: frameSeed(16), len: 100, mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: sp, end: sp + 3 * 576 }], 'chunk', 'QPSK', 1);
  add('chunk_trunc', 'standard', { kind: 'chunk', seq: 1, seed: frameSeed(17), len: 2048, mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: sp, end: sp + 3 * 576 + 10 * 576 }], 'chunk', 'QPSK', 1);
  add('meta_trunc', 'acoustic', { kind: 'meta', totalChunks: 9, totalFileSize: 4000, chunkSize: 512, name: 'long-file-name.bin', mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: silencePre('acoustic', true), end: silencePre('acoustic', true) + 3 * 640 + 6 * 640 }], 'chunk', 'BPSK', 3);
  add('meta_too_short', 'acoustic', { kind: 'meta', totalChunks: 9, totalFileSize: 4000, chunkSize: 512, name: 'x', mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: silencePre('acoustic', true), end: silencePre('acoustic', true) + 3 * 640 + 3 * 640 }], 'chunk', 'BPSK', 3);
  add('data_too_short', 'acoustic', { kind: 'chunk', seq: 2, seed: frameSeed(18), len: 64, mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: spa, end: spa + 3 * 640 + 3 * 640 }], 'chunk', 'BPSK', 3);
  add('chunk_decoded_too_short', 'acoustic', { kind: 'chunk', seq: 2, seed: frameSeed(18), len: 64, mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: spa, end: spa + 3 * 640 + 1 * 639 }], 'chunk', 'BPSK', 3);
}
// Error paths of decodeReceivedSignal.
add('empty', 'standard', { kind: 'zeros', n: 0 }, [], 'legacy', 'QPSK', 1);
add('short_100', 'standard', { kind: 'zeros', n: 100 }, [], 'legacy', 'QPSK', 1);
add('zeros_36k', 'standard', { kind: 'zeros', n: 35874 }, [], 'legacy', 'QPSK', 1);
add('tone_low_corr', 'standard', { kind: 'periodic', n: 20000, values: tonePeriod(256, 1, 0.5) }, [], 'legacy', 'QPSK', 1);
add('trunc_no_ce', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: 0, end: 13230 + 3 * 576 - 1 }], 'legacy', 'QPSK', 1);
add('trunc_no_data', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: 0, end: 13230 + 3 * 576 }], 'legacy', 'QPSK', 1);
add('trunc_decoded_short', 'acoustic', { kind: 'legacy', seed: frameSeed(5), len: 256, name: 'f.bin', mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: 0, end: 22050 + 4 * 640 }], 'legacy', 'BPSK', 3);
add('trunc_short_header', 'acoustic', { kind: 'legacy', seed: frameSeed(5), len: 256, name: 'f.bin', mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: 0, end: 22050 + 7 * 640 }], 'legacy', 'BPSK', 3);
add('trunc_bad_len', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [{ op: 'slice', start: 0, end: 13230 + 3 * 576 + 5 * 576 }], 'legacy', 'QPSK', 1);
add('dc_offset', 'standard', { kind: 'legacy', seed: frameSeed(19), len: 300, name: 'dc', mod: 'QPSK', rep: 1 }, [{ op: 'dc', dc: 0.0625 }], 'legacy', 'QPSK', 1);
add('meta_via_legacy_short', 'acoustic', { kind: 'meta', totalChunks: 9, totalFileSize: 4000, chunkSize: 512, name: 'x', mod: 'BPSK', rep: 3 }, [{ op: 'slice', start: 0, end: 22050 + 3 * 640 + 4 * 640 }], 'legacy', 'BPSK', 3);
// Noisy channel (BASELINE C5 and QPSK), exact reference outputs incl. bit errors.
add('ac_bpsk_rep3_256_snr20', 'acoustic', { kind: 'legacy', seed: frameSeed(5), len: 256, name: 'f.bin', mod: 'BPSK', rep: 3 }, [{ op: 'noise', snr: 20, seed: 0x1234567 }], 'legacy', 'BPSK', 3);
add('ac_bpsk_rep3_256_snr10', 'acoustic', { kind: 'legacy', seed: frameSeed(5), len: 256, name: 'f.bin', mod: 'BPSK', rep: 3 }, [{ op: 'noise', snr: 10, seed: 0x89abcde }], 'legacy', 'BPSK', 3);
add('std_qpsk_1k_snr10', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [{ op: 'noise', snr: 10, seed: 0xC0FFEE }], 'legacy', 'QPSK', 1);
add('std_qpsk_1k_snr20', 'standard', { kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }, [{ op: 'noise', snr: 20, seed: 0xBADC0DE }], 'legacy', 'QPSK', 1);
add('std_qam16_1k_snr20', 'standard', { kind: 'legacy', seed: frameSeed(1), len: 1024, name: 'f.bin', mod: 'QAM16', rep: 1 }, [{ op: 'noise', snr: 20, seed: 0x5EED }], 'legacy', 'QAM16', 1);
add('chunk_2k_qpsk_snr20', 'standard', { kind: 'chunk', seq: 42, seed: frameSeed(20), len: 2048, mod: 'QPSK', rep: 1 }, [{ op: 'noise', snr: 20, seed: 0xFACE }, { op: 'slice', start: 2205, end: 2205 + 3 * 576 + 41 * 576 }], 'chunk', 'QPSK', 1);

// ------------------------------------------------------------------- run --
function runCase(c) {
  setOFDMConfig(c.config);
  const tx = buildTx(c.tx);
  const sig = applyPost(tx, c.post);
  const rec = { ...c, n: sig.length, txLen: tx.length, txSha: sha(tx), sigSha: sha(sig) };
  const sigCopy = Float32Array.from(sig);
  if (c.rx === 'legacy') {
    rec.inter = legacyIntermediates(sig, c.mod, c.rep);
    rec.result = jsonResult(decodeReceivedSignal(sig, c.mod, c.rep));
  } else {
    rec.inter = chunkIntermediates(sig, c.mod, c.rep);
    rec.result = jsonResult(decodeChunkFrame(sig, c.mod, c.rep));
  }
  if (sha(sig) !== sha(sigCopy)) throw new Error('reference mutated its input');
  // the restated glue must agree with the reference's own entry point
  const r = rec.result, it = rec.inter;
  if (r.preambleIdx !== undefined && it.startIdx !== undefined && r.preambleIdx !== it.startIdx) throw new Error('fine mismatch ' + c.name);
  return rec;
}

const frames = cases.map(runCase);
setOFDMConfig('standard');

// ------------------------------------------------------------------- KATs --
const kat = {};
kat.crc32 = [];
for (const [label, bytes] of [['empty', new Uint8Array(0)], ['check', new TextEncoder().encode('123456789')],
  ['a', new TextEncoder().encode('a')], ['ramp256', Uint8Array.from({ length: 256 }, (_, i) => i)],
  ['xs4096', payloadBytes(frameSeed(99), 4096)], ['xs3', payloadBytes(frameSeed(98), 3)]]) {
  kat.crc32.push({ label, hex: hex(bytes), crc: crc32(bytes) });
}
kat.seededRandom = {};
for (const seed of [42, 43, 44]) { const r = seededRandom(seed); kat.seededRandom[seed] = Array.from({ length: 230 }, () => r()); }
kat.configs = {};
for (const cfg of ['standard', 'acoustic', 'narrowband']) {
  setOFDMConfig(cfg);
  const ce = generateChannelEstSymbol();
  kat.configs[cfg] = {
    FFT_SIZE: OFDM.FFT_SIZE, CP_LEN: OFDM.CP_LEN, SYMBOL_LEN: OFDM.SYMBOL_LEN, SAMPLE_RATE: OFDM.SAMPLE_RATE,
    SUB_START: OFDM.SUB_START, SUB_END: OFDM.SUB_END, PILOTS: OFDM.PILOTS.slice(), numDataSubs: OFDM.numDataSubs(),
    pre1: arr(generatePreambleSymbol1()), pre2: arr(generatePreambleSymbol2()),
    ceSamples: arr(ce.samples), knownRe: bandOf(ce.knownRe),
    estimateFrameSamples: [[16, 'QPSK', 1], [2059, 'QPSK', 1], [4107, 'QAM16', 1], [523, 'BPSK', 1], [280, 'BPSK', 3], [0, 'QPSK', 1], [1, 'QAM16', 3]]
      .map(([p, m, r]) => ({ payload: p, mod: m, rep: r, samples: estimateFrameSamples(p, m, r) })),
  };
}
setOFDMConfig('standard');
kat.twiddle = [];
for (let size = 2; size <= 4096; size <<= 1) {
  for (const inv of [false, true]) {
    const angle = (inv ? 1 : -1) * 2 * Math.PI / size;
    kat.twiddle.push({ size, inverse: inv, cos: Math.cos(angle), sin: Math.sin(angle) });
  }
}
function vec(seed, n, real) {
  let s = seed >>> 0; const re = new Float64Array(n), im = new Float64Array(n);
  for (let i = 0; i < n; i++) { s = xs32(s); re[i] = s / 4294967296 - 0.5; if (!real) { s = xs32(s); im[i] = s / 4294967296 - 0.5; } }
  return [re, im];
}
kat.fft = [];
for (const [label, n, seed, real] of [['cplx512', 512, 1, false], ['real512', 512, 2, true], ['cplx2048', 2048, 3, false], ['cplx8', 8, 4, false]]) {
  const [re, im] = vec(seed, n, real);
  const [Fr, Fi] = fft(re, im);
  const [Ir, Ii] = ifft(re, im);
  kat.fft.push({ label, n, seed, real, inRe: arr(re), inIm: arr(im), fftRe: arr(Fr), fftIm: arr(Fi), ifftRe: arr(Ir), ifftIm: arr(Ii) });
}
{ // impulse + constant
  const n = 512; const re = new Float64Array(n), im = new Float64Array(n); re[3] = 1;
  const [Fr, Fi] = fft(re, im); kat.fft.push({ label: 'impulse3', n, inRe: arr(re), inIm: arr(im), fftRe: arr(Fr), fftIm: arr(Fi) });
  const c = new Float64Array(n).fill(0.25); const [Cr, Ci] = fft(c, new Float64Array(n));
  kat.fft.push({ label: 'const', n, inRe: arr(c), inIm: arr(new Float64Array(n)), fftRe: arr(Cr), fftIm: arr(Ci) });
}
kat.constellations = {};
kat.demap = {};
for (const m of ['BPSK', 'QPSK', 'QAM16']) {
  const c = initConstellation(m);
  kat.constellations[m] = { bps: c.bps, points: c.points.map(p => p.slice()) };
  const pts = [];
  for (const p of c.points) pts.push([p[0], p[1]]);
  pts.push([0, 0], [-0, 0], [0, -0], [1e-17, -1e-17], [-1e-300, 1e-300]);
  const lv = [-3, -1, 1, 3].map(v => v / Math.sqrt(10));
  for (const a of lv) for (const b of [0, (lv[0] + lv[1]) / 2, (lv[1] + lv[2]) / 2, (lv[2] + lv[3]) / 2]) pts.push([a, b], [b, a]);
  let s = 0xABCDEF;
  for (let i = 0; i < 200; i++) { s = xs32(s); const a = (s / 4294967296 - 0.5) * 3; s = xs32(s); const b = (s / 4294967296 - 0.5) * 3; pts.push([a, b]); }
  kat.demap[m] = pts.map(([a, b]) => ({ re: a, im: b, bits: constellationDemap(c, a, b) }));
}
kat.majorityVote = [];
{
  let s = 0x777;
  for (const [len, n] of [[0, 3], [1, 3], [2, 3], [3, 3], [10, 3], [11, 2], [12, 4], [13, 5], [30, 1], [64, 3], [65, 3]]) {
    const bits = []; for (let i = 0; i < len; i++) { s = xs32(s); bits.push(s & 1); }
    kat.majorityVote.push({ bits, n, out: majorityVote(bits, n) });
  }
}
kat.bitsToBytes = [];
{
  let s = 0x999;
  for (const len of [0, 7, 8, 9, 15, 16, 410, 820]) {
    const bits = []; for (let i = 0; i < len; i++) { s = xs32(s); bits.push(s & 1); }
    kat.bitsToBytes.push({ bits, hex: hex(bitsToBytes(bits)) });
  }
}
kat.preprocess = [];
{
  for (const [label, n, seed, dc, scale] of [['rand1000', 1000, 5, 0.1, 0.7], ['rand7', 7, 6, -0.3, 2.0], ['tiny', 64, 7, 0, 1e-7]]) {
    let s = seed; const x = new Float32Array(n);
    for (let i = 0; i < n; i++) { s = xs32(s); x[i] = Math.fround((s / 4294967296 - 0.5) * scale + dc); }
    kat.preprocess.push({ label, x: arr(x), out: arr(preprocessSignal(x)) });
  }
}
kat.detectPreamble = [];
{
  setOFDMConfig('standard');
  const x = preprocessSignal(applyPost(buildTx({ kind: 'legacy', seed: frameSeed(0), len: 1024, name: 'f.bin', mod: 'QPSK', rep: 1 }), []));
  kat.detectPreamble.push({ label: 'std_qpsk_1k', config: 'standard', coarseIdx: detectPreamble(x) });
}
kat.sweepTone = [[500, 8000, 0.2, 44100], [1000, 1000, 0.05, 48000], [200, 12000, 0.5, 44100]].map(([a, b, d, sr]) => {
  const x = generateSweepTone(a, b, d, sr);
  return { args: [a, b, d, sr], n: x.length, sha: sha(x), head: arr(x.subarray(0, 64)), tail: arr(x.subarray(Math.max(0, x.length - 64))) };
});
kat.txInfo = [];
for (const [cfg, mod, rep, len, name] of [['standard', 'QPSK', 1, 1024, 'f.bin'], ['acoustic', 'BPSK', 3, 256, 'x'], ['standard', 'QAM16', 1, 100, ''], ['narrowband', 'BPSK', 1, 40, 'nb']]) {
  setOFDMConfig(cfg);
  const r = buildTransmitSignal(payloadBytes(frameSeed(7), len), mod, name, rep);
  kat.txInfo.push({ config: cfg, mod, rep, len, name, n: r.signal.length, sha: sha(r.signal), numSymbols: r.numSymbols, bitsPerSymbol: r.bitsPerSymbol, totalBits: r.totalBits, dataLen: r.dataLen });
}
setOFDMConfig('standard');
kat.payloadXs32 = { seed: frameSeed(0), hex16: hex(payloadBytes(frameSeed(0), 16)) };

// ------------------------------------------------------- analyzeLoopback --
const jsonNum = (v) => (Number.isFinite(v) ? v : String(v));
const loopback = [];
{
  const td = new Uint8Array(16);
  for (let i = 0; i < 16; i++) td[i] = i;
  const L = (name, config, tx, post, mod, rep) => {
    setOFDMConfig(config);
    const sig = applyPost(buildTx(tx), post);
    const res = analyzeLoopback(sig, mod, rep, td);
    const sc = detectPreamble(preprocessSignal(sig));
    loopback.push({
      name, config, tx, post, mod, rep, n: sig.length, sigSha: sha(sig), scCoarse: sc,
      result: { detected: res.detected, correlation: jsonNum(res.correlation), ber: res.ber,
        channelMagnitude: res.channelMagnitude.map(jsonNum), snrEstimate: jsonNum(res.snrEstimate), quality: res.quality },
    });
  };
  const T = (mod, rep) => ({ kind: 'test', mod, rep });
  L('lb_std_qpsk', 'standard', T('QPSK', 1), [], 'QPSK', 1);
  L('lb_std_qam16', 'standard', T('QAM16', 1), [], 'QAM16', 1);
  L('lb_std_bpsk_rep3', 'standard', T('BPSK', 3), [], 'BPSK', 3);
  L('lb_ac_bpsk', 'acoustic', T('BPSK', 1), [], 'BPSK', 1);
  L('lb_ac_bpsk_rep3', 'acoustic', T('BPSK', 3), [], 'BPSK', 3);
  L('lb_nb_bpsk_rep3', 'narrowband', T('BPSK', 3), [], 'BPSK', 3);
  // div = P_signal / P_noise: 100 (20 dB), 10, 4 (~6 dB), 2 (~3 dB), 1 (0 dB), 0.5 (~-3 dB)
  for (const div of [100, 10, 4, 2, 1, 0.5])
    L(`lb_std_qpsk_div${div}`, 'standard', T('QPSK', 1), [{ op: 'noise', div, seed: 0x1234 + Math.round(div * 2) }], 'QPSK', 1);
  for (const div of [4, 2, 1])
    L(`lb_ac_bpsk_rep3_div${div}`, 'acoustic', T('BPSK', 3), [{ op: 'noise', div, seed: 0x777 + div }], 'BPSK', 3);
  L('lb_zeros', 'standard', { kind: 'zeros', n: 30000 }, [], 'QPSK', 1);
  L('lb_short', 'standard', { kind: 'zeros', n: 300 }, [], 'QPSK', 1);
  L('lb_no_ce', 'standard', T('QPSK', 1), [{ op: 'slice', start: 0, end: 13230 + 2 * 576 + 300 }], 'QPSK', 1);
  L('lb_no_data', 'standard', T('QPSK', 1), [{ op: 'slice', start: 0, end: 13230 + 3 * 576 }], 'QPSK', 1);
  L('lb_one_sym', 'standard', T('QPSK', 1), [{ op: 'slice', start: 0, end: 13230 + 4 * 576 + 10 }], 'QPSK', 1);
  L('lb_dc', 'standard', T('QPSK', 1), [{ op: 'dc', dc: 0.25 }], 'QPSK', 1);
  L('lb_tone', 'standard', { kind: 'periodic', n: 20000, values: tonePeriod(64, 5, 0.5) }, [], 'QPSK', 1);
  L('lb_wrong_mod', 'standard', T('QPSK', 1), [], 'QAM16', 1);
  setOFDMConfig('standard');
}

const meta = {
  generator: 'tests/golden/gen_golden.js', node: process.version,
  reference: 'playok/audio-modem modem.js (loaded unmodified via vm.runInThisContext)',
};
fs.writeFileSync(path.join(OUT, 'kat.json'), JSON.stringify({ meta, ...kat }));
fs.writeFileSync(path.join(OUT, 'frames.json'), JSON.stringify({ meta, frames }));
fs.writeFileSync(path.join(OUT, 'loopback.json'), JSON.stringify({ meta, loopback }));
for (const c of loopback) console.log('loopback', c.name.padEnd(26), 'sc', c.scCoarse, JSON.stringify(c.result).slice(0, 90));
console.log('wrote', frames.length, 'frame cases;',
  'kat.json', fs.statSync(path.join(OUT, 'kat.json')).size, 'B; frames.json', fs.statSync(path.join(OUT, 'frames.json')).size, 'B');
for (const f of frames) {
  const r = f.result;
  console.log(f.name.padEnd(26), String(f.n).padStart(7), r.error ? 'ERR ' + r.error : `ok type=${r.frameType} crc=${r.crcValid} pre=${r.preambleIdx}`, 'coarse=' + (f.inter.coarseIdx));
}
