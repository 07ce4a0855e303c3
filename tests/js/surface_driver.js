'use strict';
// Test driver for the JS surface (audio-modem_amd/js/modem.js). Reads a job file
// (JSON list of operations; float32 inputs as raw little-endian files) and
// prints one JSON object of results. Uint8Array values are emitted as {hex}.
const fs = require('fs');
const path = require('path');
process.env.AMODEM_NO_GLOBALS = '1';
const M = require(path.join(__dirname, '..', '..', 'audio-modem_amd', 'js', 'modem.js'));

const sha = (ta) => require('crypto').createHash('sha256').update(Buffer.from(ta.buffer, ta.byteOffset, ta.byteLength)).digest('hex');
const enc = (v) => {
  if (v instanceof Uint8Array) return { hex: Buffer.from(v.buffer, v.byteOffset, v.byteLength).toString('hex') };
  if (ArrayBuffer.isView(v)) return { sha: sha(v), n: v.length };
  if (Array.isArray(v)) return v.map(enc);
  if (v && typeof v === 'object') {
    const o = {};
    for (const k of Object.keys(v)) o[k] = enc(v[k]);
    return o;
  }
  if (typeof v === 'number' && !Number.isFinite(v)) return { num: String(v) };
  return v;
};
const f32 = (file) => {
  const b = fs.readFileSync(file);
  return new Float32Array(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength));
};

async function main() {
  const jobs = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
  const out = {};
  for (const j of jobs) {
    try {
      if (j.config) M.setOFDMConfig(j.config);
      let r;
      switch (j.op) {
        case 'exports': r = Object.keys(M).sort(); break;
        case 'fft': r = M.fft(j.re, j.im).map((a) => Array.from(a)); break;
        case 'crc32': r = M.crc32(Buffer.from(j.hex, 'hex')); break;
        case 'estimate': r = M.estimateFrameSamples(j.payload, j.mod, j.rep); break;
        case 'preamble1': r = M.generatePreambleSymbol1(); break;
        case 'sweep': r = M.generateSweepTone(...j.args); break;
        case 'tx_legacy': r = M.buildTransmitSignal(Buffer.from(j.hex, 'hex'), j.mod, j.name, j.rep); break;
        case 'tx_meta': r = M.buildMetadataFrame(j.chunks, j.size, j.chunkSize, j.name, j.mod, j.rep); break;
        case 'tx_chunk': r = M.buildDataChunkFrame(Buffer.from(j.hex, 'hex'), j.seq, j.mod, j.rep); break;
        case 'tx_test': r = M.generateTestSignal(j.mod, j.rep); break;
        case 'constellations': M.estimateFrameSamples(1, j.mod, 1); r = M.Constellations[j.mod]; break;
        case 'ofdm': r = { cfg: Object.assign({}, M.OFDM, { isPilot: undefined, numDataSubs: undefined }), nds: M.OFDM.numDataSubs() }; break;
        case 'decode': r = M.decodeReceivedSignal(f32(j.file), j.mod, j.rep); break;
        case 'decode_chunk': r = M.decodeChunkFrame(f32(j.file), j.mod, j.rep); break;
        case 'loopback': r = M.analyzeLoopback(f32(j.file), j.mod, j.rep, Uint8Array.from(j.testData)); break;
        case 'decode_batch': {
          // onProgress: every call's prefix is final (compared with the resolved results below)
          const progress = [], early = [];
          r = await M.decodeBatch(f32(j.file), j.offsets, j.lengths, j.mod, j.rep,
            { mode: j.mode, devices: j.devices, shareBuffers: j.share === true,
              onProgress: (done, res) => { progress.push(done); early.push(JSON.stringify(enc(res.slice(0, done)))); } });
          // data ownership: fresh arrays (the reference's bytes.slice) unless shareBuffers
          const own = r.every((x) => !x.data || (x.data.byteOffset === 0 && x.data.buffer.byteLength === x.data.length));
          const prefixes_final = early.every((e, k) => e === JSON.stringify(enc(r.slice(0, progress[k]))));
          r = { results: r, ownData: own, progress, prefixes_final };
          break;
        }
        case 'decode_batch_throw': {
          // onProgress throws on its first call: the promise rejects with that error (the
          // process keeps running), and the next decode on the same addon works
          let calls = 0, rejected = null;
          try {
            await M.decodeBatch(f32(j.file), j.offsets, j.lengths, j.mod, j.rep,
              { onProgress: () => { calls++; throw new Error('onProgress boom'); } });
          } catch (e) {
            rejected = String(e && e.message);
          }
          const again = await M.decodeBatch(f32(j.file), j.offsets, j.lengths, j.mod, j.rep);
          r = { rejected, calls, again: again.length };
          break;
        }
        case 'decode_resident': {
          // uploadBatch once, decodeBatch(DeviceBatch) twice: both from HBM
          const b = M.uploadBatch(f32(j.file), j.offsets, j.lengths, j.mod, j.rep, { devices: j.devices });
          const r1 = await M.decodeBatch(b, null, null, j.mod, j.rep, { mode: j.mode });
          // free() while a decode is in flight: that decode completes, later ones reject
          const p2 = M.decodeBatch(b, null, null, j.mod, j.rep, { mode: j.mode });
          b.free();
          const r2 = await p2;
          let afterFree = null;
          try { M.decodeBatch(b, null, null, j.mod, j.rep, { mode: j.mode }); } catch (e) { afterFree = String(e.message || e); }
          r = { first: r1, second: r2, framesPerDevice: b.framesPerDevice, isDeviceBatch: b instanceof M.DeviceBatch,
            afterFree };
          break;
        }
        case 'decode_resident_concurrent': {
          // two decodes of ONE DeviceBatch in flight at once, with different modulations (the
          // payload stride differs): each must equal the same decode run alone
          const b = M.uploadBatch(f32(j.file), j.offsets, j.lengths, j.mod, j.rep, { devices: j.devices });
          const alone = [];
          for (const m of j.mods) alone.push(await M.decodeBatch(b, null, null, m, j.rep, { mode: j.mode }));
          let same = true;
          for (let it = 0; it < 4; ++it) {
            const got = await Promise.all(j.mods.map((m) => M.decodeBatch(b, null, null, m, j.rep, { mode: j.mode })));
            same = same && JSON.stringify(enc(got)) === JSON.stringify(enc(alone));
          }
          b.free();
          r = { same, first: alone[0] };
          break;
        }
        case 'asm': {
          // one ChunkAssembler scenario (tests/golden/assembler.json ops); state after each op
          const a = new M.ChunkAssembler(j.directory ? { directory: j.directory } : undefined);
          r = [];
          for (const op of j.ops) {
            let error = null, file = null;
            try {
              if (op.op === 'meta') await a.handleMetadataFrame(op);
              else if (op.op === 'chunk') await a.handleDataChunk(op.seq, Buffer.from(op.hex, 'hex'), op.crc);
              else file = Buffer.from(await a.assembleFile()).toString('hex');
            } catch (e) {
              error = e.constructor.name;
            }
            const bm = a.receivedBitmap;
            r.push({
              error, file, totalChunks: a.totalChunks, totalFileSize: a.totalFileSize, chunkSize: a.chunkSize,
              fileName: a.fileName, receivedCount: a.receivedCount, crcErrors: a.crcErrors, complete: a.isComplete(),
              bitmap: bm ? Array.from(bm) : null, missing: bm ? a.getMissingChunks() : null,
              received: bm ? Array.from({ length: Math.max(0, a.totalChunks) }, (_, i) => a.isReceived(i)) : null,
            });
          }
          break;
        }
        case 'stream': {
          const s = await M.receiveStream(f32(j.file), j.mod, j.rep);
          const a = s.assembler;
          r = {
            frames: s.frames, refineFail: s.refineFail, framesDecoded: s.framesDecoded, frameErrors: s.frameErrors,
            asm: { totalChunks: a.totalChunks, totalFileSize: a.totalFileSize, chunkSize: a.chunkSize,
              fileName: a.fileName, receivedCount: a.receivedCount, crcErrors: a.crcErrors, complete: a.isComplete() },
            file: a.totalChunks > 0 ? sha(await a.assembleFile()) : null,
          };
          break;
        }
        case 'live': { // processAudioBlock per 4096-sample block, as the audio callback drives it
          const x = f32(j.file);
          const rx = new M.StreamingReceiver(j.mod, j.rep);
          const frames = [];
          for (let b = 0; b < x.length; b += 4096) {
            const f = rx.processAudioBlock(x.subarray(b, b + 4096));
            if (f) frames.push(f);
          }
          const a = rx.assembler;
          r = {
            frames, framesDecoded: rx.framesDecoded, frameErrors: rx.frameErrors, acScanPos: rx.acScanPos,
            state: rx.state, totalWritten: rx.totalWritten,
            asm: { totalChunks: a.totalChunks, totalFileSize: a.totalFileSize, chunkSize: a.chunkSize,
              fileName: a.fileName, receivedCount: a.receivedCount, crcErrors: a.crcErrors, complete: a.isComplete() },
            file: a.totalChunks > 0 ? sha(await a.assembleFile()) : null,
          };
          // close() order: the assembler first (its handle is dead at once, its native
          // object lives until the receiver on it closes), then the receiver
          a.close();
          const thrown = (f) => { try { f(); return null; } catch (e) { return e.constructor.name; } };
          r.afterAsmClose = { asm: thrown(() => a.receivedCount), rxState: rx.state,
            rxBlock: thrown(() => rx.processAudioBlock(new Float32Array(4096))) };
          rx.close();
          r.afterRxClose = { rx: thrown(() => rx.state), again: thrown(() => { rx.close(); a.close(); }) };
          break;
        }
        case 'asm_close': {
          // handles: close() frees, later use throws TypeError, a second close is a no-op;
          // open/close cycles; assemblers left open are closed at exit (clean exit code)
          const thrown = (f) => { try { f(); return null; } catch (e) { return e.constructor.name; } };
          const a = new M.ChunkAssembler();
          await a.handleMetadataFrame({ totalChunks: 2, totalFileSize: 10, chunkSize: 5, fileName: 'x' });
          const before = a.totalChunks;
          a.close();
          r = { before, after: thrown(() => a.totalChunks), chunk: thrown(() => M.native.asmChunk(a._h, 0, new Uint8Array(5), true)),
            again: thrown(() => a.close()) };
          for (let i = 0; i < j.cycles; i++) {
            const b = new M.ChunkAssembler();
            await b.handleDataChunk(0, new Uint8Array(5), true);
            b.close();
          }
          for (let i = 0; i < j.leftOpen; i++) new M.ChunkAssembler();
          r.cycles = j.cycles;
          break;
        }
        default: throw new Error('unknown op ' + j.op);
      }
      out[j.id] = { ok: enc(r) };
    } catch (e) {
      out[j.id] = { throw: e.constructor.name, message: e.message };
    }
  }
  process.stdout.write(JSON.stringify(out));
}
main().catch((e) => { console.error(e); process.exit(1); });
