'use strict';
// modem.js — the playok/audio-modem `modem.js` function surface, backed by the
// MI355X engine (libamodem.so through the N-API addon amodem.node).
//
// Exports the 17 globals app.js uses (SURVEY.md §8b) with the reference's
// names, argument meaning, return shapes and error strings, as CommonJS exports
// and, when loaded in a page-like global scope, as globals:
//   fft, OFDM_CONFIGS, OFDM, setOFDMConfig, Constellations,
//   generatePreambleSymbol1, buildTransmitSignal, decodeReceivedSignal,
//   FRAME_META, FRAME_DATA, buildMetadataFrame, buildDataChunkFrame,
//   decodeChunkFrame, estimateFrameSamples, generateSweepTone,
//   generateTestSignal, analyzeLoopback
// plus the additive batch entry decodeBatch (Promise, napi_async_work).
//
// decodeReceivedSignal (modem.js:557-654) and decodeChunkFrame (modem.js:770-803)
// run on the GPU; the transmit builders run in the native host library. There is
// no JavaScript fallback: if the addon cannot load, requiring this module throws.

const path = require('path');
const util = require('util');

const native = require(process.env.AMODEM_NODE || path.join(__dirname, '..', 'lib', 'amodem.node'));

const TD = typeof TextDecoder !== 'undefined' ? TextDecoder : util.TextDecoder;
const TE = typeof TextEncoder !== 'undefined' ? TextEncoder : util.TextEncoder;

// ------------------------------------------------------------------ config --
// Presets (modem.js:69-85)
const OFDM_CONFIGS = {
  standard: {
    FFT_SIZE: 512, CP_LEN: 64, SYMBOL_LEN: 576, SAMPLE_RATE: 44100, SUB_START: 12, SUB_END: 232,
    PILOTS: [15, 29, 43, 57, 71, 85, 99, 113, 127, 141, 155, 169, 183, 197, 211, 225],
  },
  acoustic: {
    FFT_SIZE: 512, CP_LEN: 128, SYMBOL_LEN: 640, SAMPLE_RATE: 44100, SUB_START: 23, SUB_END: 93,
    PILOTS: [25, 35, 45, 55, 65, 75, 85],
  },
  narrowband: {
    FFT_SIZE: 512, CP_LEN: 256, SYMBOL_LEN: 768, SAMPLE_RATE: 44100, SUB_START: 35, SUB_END: 58,
    PILOTS: [37, 45, 53],
  },
};

// The mutable current configuration (modem.js:87-93): a copy of a preset plus helpers.
const OFDM = Object.assign({}, OFDM_CONFIGS.standard);
OFDM.isPilot = (k) => OFDM.PILOTS.includes(k);
OFDM.numDataSubs = () => {
  let n = 0;
  for (let k = OFDM.SUB_START; k <= OFDM.SUB_END; k++) if (!OFDM.isPilot(k)) n++;
  return n;
};

// setOFDMConfig: unknown names select 'standard' (modem.js:95-98)
function setOFDMConfig(name) {
  const preset = Object.prototype.hasOwnProperty.call(OFDM_CONFIGS, name) ? OFDM_CONFIGS[name] : OFDM_CONFIGS.standard;
  for (const key of Object.keys(preset)) OFDM[key] = preset[key];
}

const FRAME_META = 0xFE;
const FRAME_DATA = 0xFF;

// ----------------------------------------------------------- constellation --
// Constellations + lazily filled points (modem.js:101-131). 16-QAM: Gray per
// axis, unit average energy.
const Constellations = {
  BPSK: { bps: 1, points: null },
  QPSK: { bps: 2, points: null },
  QAM16: { bps: 4, points: null },
};
const MOD_ID = { BPSK: 0, QPSK: 1, QAM16: 2 };

function fillPoints(name) {
  const c = Constellations[name];
  if (c.points) return c;
  if (name === 'BPSK') {
    c.points = [[1, 0], [-1, 0]];
  } else if (name === 'QPSK') {
    const a = 1 / Math.SQRT2;
    c.points = [[a, a], [-a, a], [-a, -a], [a, -a]];
  } else {
    const gray = (v) => v ^ (v >> 1);
    const pts = [];
    let energy = 0;
    for (let idx = 0; idx < 16; idx++) {
      const x = 2 * gray(idx & 3) - 3, y = 2 * gray(idx >> 2) - 3;
      pts.push([x, y]);
      energy += x * x + y * y;
    }
    const scale = 1 / Math.sqrt(energy / 16);
    c.points = pts.map(([x, y]) => [x * scale, y * scale]);
  }
  return c;
}

function modulationId(modName) {
  if (!Object.prototype.hasOwnProperty.call(MOD_ID, modName)) {
    // the reference dereferences Constellations[modName].points (modem.js:108-109)
    throw new TypeError("Cannot read property 'points' of undefined");
  }
  fillPoints(modName);
  return MOD_ID[modName];
}

// amod_cfg for the native side, from the current OFDM state
function nativeCfg(modName, repetition, checkMod) {
  return {
    fft_size: OFDM.FFT_SIZE, cp_len: OFDM.CP_LEN, symbol_len: OFDM.SYMBOL_LEN, sample_rate: OFDM.SAMPLE_RATE,
    sub_start: OFDM.SUB_START, sub_end: OFDM.SUB_END, pilots: OFDM.PILOTS.slice(),
    modulation: checkMod === false ? 1 : modulationId(modName),
    repetition: Math.max(1, (repetition || 1) | 0),
  };
}

// --------------------------------------------------------------------- FFT --
// fft(re, im) -> [Float64Array re, Float64Array im] (modem.js:6-13): radix-2
// decimation in time after a bit-reversal permutation; each stage's twiddles
// come from the same complex recurrence w <- w * wn, tabulated once per size, so
// the rounding equals the reference's.
const twiddleCache = new Map();
function stageTwiddles(n) {
  let t = twiddleCache.get(n);
  if (t) return t;
  t = [];
  for (let size = 2; size <= n; size <<= 1) {
    const half = size >> 1;
    const ang = -2 * Math.PI / size;
    const cr = Math.cos(ang), ci = Math.sin(ang);
    const tr = new Float64Array(half), ti = new Float64Array(half);
    let wr = 1, wi = 0;
    for (let j = 0; j < half; j++) {
      tr[j] = wr; ti[j] = wi;
      const nr = wr * cr - wi * ci;
      wi = wr * ci + wi * cr;
      wr = nr;
    }
    t.push([tr, ti]);
  }
  twiddleCache.set(n, t);
  return t;
}

function fft(re, im) {
  const n = re.length;
  const xr = Float64Array.from(re), xi = Float64Array.from(im);
  let lg = 0;
  while ((1 << lg) < n) lg++;
  for (let i = 0; i < n; i++) {
    let r = 0;
    for (let b = 0, v = i; b < lg; b++, v >>= 1) r = (r << 1) | (v & 1);
    if (i < r) {
      let s = xr[i]; xr[i] = xr[r]; xr[r] = s;
      s = xi[i]; xi[i] = xi[r]; xi[r] = s;
    }
  }
  const tw = n > 1 ? stageTwiddles(n) : [];
  for (let st = 0, half = 1; half < n; st++, half <<= 1) {
    const [tr, ti] = tw[st];
    for (let base = 0; base < n; base += 2 * half) {
      for (let j = 0; j < half; j++) {
        const a = base + j, b = a + half;
        const pr = tr[j] * xr[b] - ti[j] * xi[b];
        const pi = tr[j] * xi[b] + ti[j] * xr[b];
        xr[b] = xr[a] - pr; xi[b] = xi[a] - pi;
        xr[a] += pr; xi[a] += pi;
      }
    }
  }
  return [xr, xi];
}

// ---------------------------------------------------------- transmit side --
function generatePreambleSymbol1() { // modem.js:158-170
  return native.preamble1(nativeCfg('QPSK', 1, false));
}

function estimateFrameSamples(payloadBytes, modName, repetition) { // modem.js:863-874
  return native.estimateFrameSamples(nativeCfg(modName, repetition), payloadBytes | 0);
}

function toBytes(x) {
  if (x instanceof Uint8Array) return x;
  if (ArrayBuffer.isView(x)) return new Uint8Array(x.buffer, x.byteOffset, x.byteLength);
  return Uint8Array.from(x || []);
}

// buildTransmitSignal(fileData, modName, fileName, repetition) (modem.js:498-555)
function buildTransmitSignal(fileData, modName, fileName, repetition) {
  const cfg = nativeCfg(modName, repetition);
  const data = toBytes(fileData);
  const name = new TE().encode(fileName || 'file');
  const signal = native.txLegacy(cfg, data, name.subarray(0, Math.min(name.length, 255)));
  const bitsPerSymbol = OFDM.numDataSubs() * Constellations[modName].bps;
  const rawBits = (1 + Math.min(name.length, 255) + 4 + data.length + 4) * 8 * cfg.repetition;
  const numSymbols = Math.ceil(rawBits / bitsPerSymbol);
  return { signal, numSymbols, bitsPerSymbol, totalBits: numSymbols * bitsPerSymbol, dataLen: data.length };
}

// buildMetadataFrame / buildDataChunkFrame (modem.js:758-766) -> Float32Array
function buildMetadataFrame(totalChunks, totalFileSize, chunkSize, fileName, modName, rep) {
  const name = new TE().encode(fileName || 'file');
  return native.txMeta(nativeCfg(modName, rep), totalChunks | 0, totalFileSize | 0, chunkSize | 0,
    name.subarray(0, Math.min(name.length, 255)));
}

function buildDataChunkFrame(chunkData, seqNum, modName, rep) {
  return native.txChunk(nativeCfg(modName, rep), toBytes(chunkData), seqNum | 0);
}

// generateTestSignal(modName, repetition) -> {signal, testData} (modem.js:914-973)
function generateTestSignal(modName, repetition) {
  const testData = new Uint8Array(16);
  for (let i = 0; i < 16; i++) testData[i] = i;
  return { signal: native.txTestSignal(nativeCfg(modName, repetition)), testData };
}

// generateSweepTone(startFreq, endFreq, duration, sampleRate) (modem.js:890-911):
// linear chirp at 0.8 peak with 50 ms linear fades at both ends.
function generateSweepTone(startFreq, endFreq, duration, sampleRate) {
  const n = Math.round(duration * sampleRate);
  const out = new Float32Array(n);
  const fade = Math.round(0.05 * sampleRate);
  const span = endFreq - startFreq, twoD = 2 * duration;
  for (let i = 0; i < n; i++) {
    const t = i / sampleRate;
    // phase = 2*pi*(f0*t + (f1-f0)*t^2/(2d)), evaluated in the reference's operation order
    let v = 0.8 * Math.sin(2 * Math.PI * (startFreq * t + span * t * t / twoD));
    if (i < fade) v *= i / fade;
    else if (i > n - fade) v *= (n - i) / fade;
    out[i] = v;
  }
  return out;
}

// ----------------------------------------------------------- receive side --
const MODE_RECEIVED = 0, MODE_CHUNK = 1;
const ERR = {
  1: 'Preamble not detected',
  2: 'Preamble not detected (low correlation)',
  3: 'Signal too short for CE',
  4: 'No data after CE',
  5: 'Decoded data too short',
  6: 'Decoded data too short for header',
  8: 'Metadata frame too short',
  9: 'Metadata frame truncated',
  10: 'Data chunk frame too short',
  11: 'Data chunk truncated',
  12: 'Frame too short for CE',
};
const PRE_DEMOD = new Set([1, 2, 3, 4, 12]); // outcomes decided before demodulateOFDM runs
const E_INVALID_LEN = 7, E_UNKNOWN_TYPE = 13, E_CAPACITY = 100;
const REC = 96; // sizeof(amod_result)

// TextDecoder().decode (the reference decodes names with a fresh TextDecoder): one
// decoder for every call, and plain ASCII (no BOM, no multi-byte sequence: the decoder's
// output is then the bytes' own code points) without it
const UTF8 = new TD();
function utf8(bytes, off, len) {
  if (off === undefined) { off = 0; len = bytes.length; }
  let s = '';
  for (let i = 0; i < len; i++) {
    const c = bytes[off + i];
    if (c > 0x7F || len > 256) return UTF8.decode(bytes.subarray(off, off + len));
    s += String.fromCharCode(c);
  }
  return s;
}

// one amod_result record (+ its payload slot) -> the reference's return object.
// share = false: `data` is a fresh Uint8Array (bytes.slice, modem.js:636,837); share =
// true (decodeBatch's opt-in shareBuffers): `data` is a view of the call's own payload
// buffer (every frame's range its own), which spares one allocation per frame
function formatResult(view, i, payload, stride, viaLegacy, share, u8) {
  const o = i * REC;
  const status = view.getInt32(o, true);
  const preambleIdx = view.getInt32(o + 4, true), frameType = view.getInt32(o + 12, true);
  if (status === E_CAPACITY) throw new Error('frame exceeds the reserved decode workspace');
  if (status === 0) {
    const base = i * stride;
    const nameOff = base + view.getInt32(o + 24, true), nameLen = view.getInt32(o + 28, true);
    const dataOff = base + view.getInt32(o + 32, true), dataLen = view.getInt32(o + 36, true);
    const crcValid = view.getInt32(o + 64, true) !== 0;
    const expectedCRC = view.getUint32(o + 56, true), actualCRC = view.getUint32(o + 60, true);
    const all = u8 || new Uint8Array(payload);
    if (frameType === FRAME_META) {
      const r = {
        frameType: FRAME_META, totalChunks: view.getInt32(o + 44, true), totalFileSize: view.getInt32(o + 48, true),
        chunkSize: view.getInt32(o + 52, true), fileName: utf8(all, nameOff, nameLen), crcValid, expectedCRC,
        actualCRC,
      };
      if (viaLegacy) r.preambleIdx = preambleIdx;
      return r;
    }
    const data = share ? all.subarray(dataOff, dataOff + dataLen) : all.slice(dataOff, dataOff + dataLen);
    if (frameType === FRAME_DATA) {
      const r = { frameType: FRAME_DATA, seqNum: view.getInt32(o + 40, true), data, dataLen, crcValid, expectedCRC,
        actualCRC };
      if (viaLegacy) r.preambleIdx = preambleIdx;
      return r;
    }
    return {
      data, dataLen, fileName: utf8(all, nameOff, nameLen), crcValid, expectedCRC, actualCRC, preambleIdx,
      frameType: 'legacy',
    };
  }
  const aux = view.getInt32(o + 16, true);
  if (status === E_INVALID_LEN) return { error: `Invalid data length: ${aux}` };
  if (status === E_UNKNOWN_TYPE) return { error: `Unknown frame type: 0x${aux.toString(16)}`, frameType: aux };
  const r = { error: ERR[status] };
  if (viaLegacy && (frameType === FRAME_META || frameType === FRAME_DATA) && status >= 8 && status <= 11) {
    r.preambleIdx = preambleIdx;
  }
  return r;
}

function asFloat32(sig) {
  return sig instanceof Float32Array ? sig : Float32Array.from(sig);
}

function decodeOne(signal, modName, repetition, mode) {
  // an unknown modulation only throws once demodulation is reached (modem.js:365-367)
  const known = Object.prototype.hasOwnProperty.call(MOD_ID, modName);
  const cfg = nativeCfg(modName, repetition, known ? undefined : false);
  const out = native.decode(asFloat32(signal), null, null, cfg, mode, 0);
  const view = new DataView(out.results);
  if (!known && !PRE_DEMOD.has(view.getInt32(0, true))) modulationId(modName);
  return formatResult(view, 0, out.payload, out.stride, mode === MODE_RECEIVED, false);
}

// decodeReceivedSignal(signal, modName, repetition) (modem.js:557-654)
function decodeReceivedSignal(signal, modName, repetition) {
  return decodeOne(signal, modName, repetition, MODE_RECEIVED);
}

// decodeChunkFrame(frameSamples, modName, repetition) (modem.js:770-803)
function decodeChunkFrame(frameSamples, modName, repetition) {
  return decodeOne(frameSamples, modName, repetition, MODE_CHUNK);
}

// decodeBatch(samples, frameOffsets, frameLens, modName, rep, {device, devices, mode,
// shareBuffers}) -> Promise<result[]>: many frames of one buffer in one GPU launch
// (additive API); devices: n > 1 splits the batch into contiguous frame ranges over GPUs
// 0 .. n-1, decoded concurrently (amod_group_decode_host), results in frame order.
// samples may also be a DeviceBatch (uploadBatch): its frames are decoded from HBM on the
// GPUs they were uploaded to (amod_resident_decode), frameOffsets / frameLens ignored.
// Every result's `data` is a fresh Uint8Array, as the reference's (bytes.slice,
// modem.js:636,837); shareBuffers: true makes them views of one payload buffer per call
// instead (no per-frame copy; `data.buffer` then holds every frame's bytes, and keeping
// one result keeps that buffer alive). onProgress(done, results): called as results[0 ..
// done) are final (host samples on one device: after each decoded 64 MB piece; otherwise
// once), before the promise resolves with the same array.
function decodeBatch(samples, frameOffsets, frameLens, modName, rep, opts) {
  const o = opts || {};
  const mode = o.mode === 'chunk' || o.mode === MODE_CHUNK ? MODE_CHUNK : MODE_RECEIVED;
  const cfg = nativeCfg(modName, rep);
  const share = o.shareBuffers === true;
  const whole = (out, n) => {
    const r = formatBatch(out.results, out.payload, out.stride, n, mode === MODE_RECEIVED, share);
    if (o.onProgress) o.onProgress(n, r);
    return r;
  };
  if (samples instanceof DeviceBatch) {
    return native.residentDecodeAsync(samples.handle, cfg, mode, o.forceExact ? 1 : 0)
      .then((out) => whole(out, samples.nframes));
  }
  const offs = frameOffsets instanceof Float64Array ? frameOffsets : Float64Array.from(frameOffsets);
  const lens = frameLens instanceof Int32Array ? frameLens : Int32Array.from(frameLens);
  const n = lens.length, viaLegacy = mode === MODE_RECEIVED;
  // one device: the frames of each decoded 64 MB piece are formatted as soon as they are
  // back (onFrames, amod_decode_host_progress), while the library uploads and decodes the
  // rest; what is left when the promise settles is formatted then. An error thrown while
  // formatting or by onProgress (which runs from the library's progress callback, where no
  // caller could catch it) is kept, and the promise rejects with it.
  const res = new Array(n);
  let done = 0, failed = null;
  const onFrames = (upto, results, payload, stride) => {
    if (failed !== null || upto <= done) return;
    try {
      formatBatch(results, payload, stride, upto, viaLegacy, share, res, done);
      done = upto;
      if (o.onProgress) o.onProgress(done, res);
    } catch (e) {
      failed = e;
    }
  };
  return native.decodeAsync(asFloat32(samples), offs, lens, cfg, mode, o.forceExact ? 1 : 0, o.device | 0,
    Math.max(1, o.devices | 0), onFrames)
    .then((out) => {
      onFrames(n, out.results, out.payload, out.stride);
      if (failed !== null) throw failed;
      return res;
    });
}

// A batch made resident on GPUs 0 .. devices-1 once (amod_group_upload: contiguous frame
// ranges of about equal sample counts), for decodeBatch to decode from HBM as often as
// needed (a Node host driving several GPUs without one upload per decode); free() when done.
class DeviceBatch {
  constructor(up, devices) {
    this.handle = up.handle;
    this.nframes = up.nframes;
    this.maxLen = up.maxLen;
    this.devices = devices;
    this.framesPerDevice = up.framesPerDevice;
  }

  // releases the batch's GPU memory (after a decode still in flight); otherwise it is
  // released when the Node environment exits, not by the garbage collector
  free() {
    native.residentFree(this.handle);
  }
}

// uploadBatch(samples, frameOffsets, frameLens, modName, rep, {devices}) -> DeviceBatch
function uploadBatch(samples, frameOffsets, frameLens, modName, rep, opts) {
  const o = opts || {};
  const devices = Math.max(1, o.devices | 0);
  const offs = frameOffsets instanceof Float64Array ? frameOffsets : Float64Array.from(frameOffsets);
  const lens = frameLens instanceof Int32Array ? frameLens : Int32Array.from(frameLens);
  return new DeviceBatch(native.residentUpload(asFloat32(samples), offs, lens, nativeCfg(modName, rep), devices),
    devices);
}

// every record of a batch -> the reference's result objects, in frame order
// the batch's result objects: successful data-chunk and legacy frames straight from an
// Int32Array over the records (the same fields, in the same key order, as formatResult,
// which takes every other outcome)
// (into `into` from frame `from` on, when given: decodeBatch formats piece by piece)
function formatBatch(results, payload, stride, n, viaLegacy, share, into, from) {
  const view = new DataView(results), u8 = new Uint8Array(payload);
  const iv = new Int32Array(results, 0, (REC >> 2) * n);
  const sh = share === true;
  const res = into || new Array(n);
  for (let i = from | 0; i < n; i++) {
    const o = (REC >> 2) * i;
    const frameType = iv[o + 3];
    if (iv[o] !== 0 || (frameType !== FRAME_DATA && frameType !== 0)) {
      res[i] = formatResult(view, i, payload, stride, viaLegacy, sh, u8);
      continue;
    }
    const base = i * stride;
    const dataOff = base + iv[o + 8], dataLen = iv[o + 9];
    const data = sh ? u8.subarray(dataOff, dataOff + dataLen) : u8.slice(dataOff, dataOff + dataLen);
    const crcValid = iv[o + 16] !== 0, expectedCRC = iv[o + 14] >>> 0, actualCRC = iv[o + 15] >>> 0;
    if (frameType === FRAME_DATA) {
      const r = { frameType: FRAME_DATA, seqNum: iv[o + 10], data, dataLen, crcValid, expectedCRC, actualCRC };
      if (viaLegacy) r.preambleIdx = iv[o + 1];
      res[i] = r;
    } else {
      res[i] = {
        data, dataLen, fileName: utf8(u8, base + iv[o + 6], iv[o + 7]), crcValid, expectedCRC, actualCRC,
        preambleIdx: iv[o + 1], frameType: 'legacy',
      };
    }
  }
  return res;
}

// analyzeLoopback(recorded, modName, repetition, testData) (modem.js:975-1082).
// The receive core runs on the GPU (exact kernel: preprocess, Schmidl-Cox with the
// cross-correlation fallback, fine timing without the 0.1 cut-off, channel estimate,
// demodulation, vote); the report below uses the reference's own arithmetic on the
// returned channel estimate and bytes.
function analyzeLoopback(recorded, modName, repetition, testData) {
  const known = Object.prototype.hasOwnProperty.call(MOD_ID, modName);
  const cfg = nativeCfg(modName, repetition, known ? undefined : false);
  const r = native.loopback(asFloat32(recorded), cfg);
  const poor = (detected, correlation) =>
    ({ detected, correlation, ber: 1, channelMagnitude: [], snrEstimate: 0, quality: 'poor' });
  if (r.status === 1) return poor(false, 0);               // not detected (modem.js:986)
  const correlation = Math.max(0, r.fineMetric);
  if (r.status === 3) return poor(true, correlation);       // no room for the CE (modem.js:1017)
  if (!known) modulationId(modName);                        // demodulateOFDM would throw here
  const channelMagnitude = [];
  for (let b = 0; b < r.hRe.length; b++) channelMagnitude.push(Math.sqrt(r.hRe[b] * r.hRe[b] + r.hIm[b] * r.hIm[b]));
  let snrSum = 0, snrCount = 0;
  for (const p of OFDM.PILOTS) {
    if (p >= OFDM.SUB_START && p <= OFDM.SUB_END) {
      const b = p - OFDM.SUB_START;
      const mag = Math.sqrt(r.hRe[b] * r.hRe[b] + r.hIm[b] * r.hIm[b]);
      if (mag > 1e-6) { snrSum += mag; snrCount++; }
    }
  }
  const avgPilotMag = snrCount > 0 ? snrSum / snrCount : 0;
  const snrEstimate = avgPilotMag > 0 ? 20 * Math.log10(avgPilotMag) : -Infinity;
  let ber = 1;
  const decoded = r.bytes;
  const start = r.preambleIdx, dataStart = start + 3 * OFDM.SYMBOL_LEN;
  if (dataStart < recorded.length && decoded.length >= 29) {
    const dataOffset = 1 + decoded[0] + 4;
    if (dataOffset + testData.length <= decoded.length) {
      let errorBits = 0;
      for (let i = 0; i < testData.length; i++) {
        const x = decoded[dataOffset + i] ^ testData[i];
        for (let b = 0; b < 8; b++) errorBits += (x >> b) & 1;
      }
      ber = errorBits / (testData.length * 8);
    }
  }
  const quality = ber === 0 && correlation > 0.8 ? 'excellent' : (ber < 0.05 ? 'good' : 'poor');
  return { detected: true, correlation, ber, channelMagnitude, snrEstimate, quality };
}


// ------------------------------------------- chunk assembly / streaming receive --
// app.js ChunkAssembler (597-704) over libamodem's host assembler (assembler.cpp): same
// methods, getters and thrown errors; chunks live in memory, or as files under
// opts.directory (the IndexedDB store's stand-in). The async methods resolve at once.
const ASM_RANGE_ERROR = -10, ASM_TYPE_ERROR = -11;
function asmThrow(st) {
  if (st === ASM_RANGE_ERROR) throw new RangeError('Invalid typed array length');
  if (st === ASM_TYPE_ERROR) throw new TypeError("Cannot read properties of null (reading 'transaction')");
  if (typeof st === 'number' && st < 0) throw new Error(`assembler error ${st}`);
  return st;
}

class ChunkAssembler {
  constructor(opts) {
    this._h = native.asmOpen((opts && opts.directory) || null);
  }
  _st() { return native.asmState(this._h); }
  get totalChunks() { return this._st().totalChunks; }
  get totalFileSize() { return this._st().totalFileSize; }
  get chunkSize() { return this._st().chunkSize; }
  get fileName() { return utf8(this._st().fileName); }
  get receivedBitmap() { return this._st().bitmap; }
  get receivedCount() { return this._st().receivedCount; }
  get crcErrors() { return this._st().crcErrors; }
  async handleMetadataFrame(meta) {
    asmThrow(native.asmMetadata(this._h, meta.totalChunks | 0, meta.totalFileSize | 0, meta.chunkSize | 0,
      new TE().encode(String(meta.fileName))));
  }
  async handleDataChunk(seqNum, data, crcValid) {
    asmThrow(native.asmChunk(this._h, seqNum | 0, toBytes(data), !!crcValid));
  }
  isReceived(seqNum) {
    const b = this._st().bitmap;
    if (!b) return false;
    return !!(b[seqNum >> 3] & (1 << (seqNum & 7)));
  }
  isComplete() { return this._st().complete; }
  getMissingChunks() { return Array.from(native.asmMissing(this._h)); }
  async assembleFile() {
    const r = native.asmFile(this._h);
    asmThrow(typeof r === 'number' ? r : 0);
    return r;
  }
  cleanup() {}
  // releases the native assembler (its chunks and maps) now, or when the last
  // StreamingReceiver on it closes; otherwise at exit (not by the garbage collector).
  // Additive: the reference's store lives as long as the page.
  close() { native.asmClose(this._h); }
}

const E_STREAM_LOST = 101;
const STREAM_REC = 24 + REC; // sizeof(amod_stream_frame)

// receiveStream(samples, modName, repetition, {assembler, device}) -> Promise<{frames,
// refineFail, framesDecoded, frameErrors, assembler}>: app.js StreamingReceiver
// (706-998) over a recorded stream fed in 4096-sample blocks (GPU pre-pass + decode,
// host state machine); every demodulated window with decodeChunkFrame's outcome
// (payload bytes go to the assembler, as _demodulateFrame does). Additive API.
// one amod_stream_frame record -> {preambleGlobalPos, expectedFrameEnd, length, result}
function streamFrame(view, b) {
  const g = (k) => view.getInt32(b + 24 + 4 * k, true);
  const status = g(0), frameType = g(3), aux = g(4);
  let result;
  if (status === 0 && frameType === FRAME_META) {
    result = { frameType, totalChunks: g(11), totalFileSize: g(12), chunkSize: g(13), crcValid: g(16) !== 0 };
  } else if (status === 0) {
    result = { frameType, seqNum: g(10), dataLen: g(9), crcValid: g(16) !== 0 };
  } else if (status === E_STREAM_LOST) {
    result = { error: 'window left the ring buffer' };
  } else if (status === E_INVALID_LEN) {
    result = { error: `Invalid data length: ${aux}` };
  } else if (status === E_UNKNOWN_TYPE) {
    result = { error: `Unknown frame type: 0x${aux.toString(16)}`, frameType: aux };
  } else {
    result = { error: ERR[status] };
  }
  return {
    preambleGlobalPos: Number(view.getBigInt64(b, true)), expectedFrameEnd: Number(view.getBigInt64(b + 8, true)),
    length: view.getInt32(b + 16, true), result,
  };
}

async function receiveStream(samples, modName, repetition, opts) {
  const o = opts || {};
  const asm = o.assembler || new ChunkAssembler();
  const r = native.receiveStream(asFloat32(samples), nativeCfg(modName, repetition), asm._h, o.device | 0);
  const view = new DataView(r.frames);
  const frames = [];
  for (let i = 0; i < r.nframes; i++) frames.push(streamFrame(view, i * STREAM_REC));
  return {
    frames, refineFail: Array.from(r.refineFail), framesDecoded: Number(r.framesDecoded),
    frameErrors: Number(r.frameErrors), assembler: asm,
  };
}

// app.js StreamingReceiver (706-998) driven live: processAudioBlock(inputSamples) once
// per audio callback (app.js:1108-1112), as startStreamingReceive does. DC removal, ring
// buffer and one state-machine step per call on the host; a completed window is decoded
// on the GPU and handed to this.assembler before the call returns. Returns the
// demodulated window ({preambleGlobalPos, expectedFrameEnd, length, result}) or null,
// and calls opts.onFrame with it. Fields mirror the reference's (state, acScanPos, ...).
const RECV_STATE = { IDLE: 0, PREAMBLE_DETECTED: 1, COLLECTING_FRAME: 2, DEMODULATING: 3 };
class StreamingReceiver {
  constructor(modName, repetition, opts) {
    const o = opts || {};
    this.modName = modName;
    this.repetition = repetition;
    this.assembler = o.assembler || new ChunkAssembler();
    this.onFrame = o.onFrame || null;
    this._h = native.liveOpen(nativeCfg(modName, repetition), this.assembler._h, o.device | 0);
    this.startTime = Date.now();
  }
  processAudioBlock(inputSamples) {
    const ab = native.liveProcess(this._h, asFloat32(inputSamples));
    if (!ab) return null;
    const frame = streamFrame(new DataView(ab), 0);
    if (this.onFrame) this.onFrame(frame);
    return frame;
  }
  _st() { return native.liveState(this._h); }
  get state() { return this._st().state; }
  get acScanPos() { return this._st().acScanPos; }
  get preambleGlobalPos() { return this._st().preambleGlobalPos; }
  get expectedFrameEnd() { return this._st().expectedFrameEnd; }
  get metaReceived() { return this._st().metaReceived !== 0; }
  get framesDecoded() { return this._st().framesDecoded; }
  get frameErrors() { return this._st().frameErrors; }
  get totalWritten() { return this._st().totalWritten; }
  cleanup() { this.assembler.cleanup(); }
  // releases the native receiver (its ring buffer and GPU workspace) now; the assembler
  // stays open for the caller (assembler.close()). Additive, like ChunkAssembler.close().
  close() { native.liveClose(this._h); }
}

const api = {
  fft, OFDM_CONFIGS, OFDM, setOFDMConfig, Constellations, generatePreambleSymbol1, buildTransmitSignal,
  decodeReceivedSignal, FRAME_META, FRAME_DATA, buildMetadataFrame, buildDataChunkFrame, decodeChunkFrame,
  estimateFrameSamples, generateSweepTone, generateTestSignal, analyzeLoopback,
  decodeBatch, uploadBatch, DeviceBatch, crc32: (data) => native.crc32(toBytes(data)), native, ChunkAssembler,
  receiveStream,
  StreamingReceiver, RECV_STATE, _formatBatch: formatBatch,
};

module.exports = api;
// browser-style globals for code written against the reference's script-tag globals
if (typeof globalThis !== 'undefined' && process.env.AMODEM_NO_GLOBALS !== '1') {
  for (const k of Object.keys(api)) if (k !== 'native' && !(k in globalThis)) globalThis[k] = api[k];
}
