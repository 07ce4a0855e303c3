#!/usr/bin/env node
// Golden-vector generator for the chunk assembler (test infrastructure, runs ONLY in
// the build container). Loads the UNMODIFIED reference modem.js and app.js with
// vm.runInThisContext (app.js behind minimal DOM / IndexedDB stand-ins that hold data
// in memory), drives the reference's own ChunkAssembler class (app.js:597-704)
// through scripted scenarios, and records its observable state after every step and
// the assembled file (or the error assembleFile raises). Only recipes and outputs are
// written (tests/golden/assembler.json); no reference source.
//
// Usage: node tests/golden/gen_assembler.js [/root/reference]
'use strict';
const vm = require('vm');
const fs = require('fs');
const path = require('path');
const util = require('util');

const REF = process.argv[2] || '/root/reference';
global.TextEncoder = util.TextEncoder;
global.TextDecoder = util.TextDecoder;
const el = () => ({ addEventListener() {}, style: {}, classList: { add() {}, remove() {}, toggle() {} },
  appendChild() {}, setAttribute() {}, getContext: () => null, textContent: '', innerHTML: '', value: '' });
global.document = { addEventListener() {}, getElementById: () => null, createElement: el,
  querySelectorAll: () => [], querySelector: () => null, body: el() };
global.window = global;

// IndexedDB stand-in: object stores as Maps, callbacks on later macrotasks like the real one
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
                get(key) {
                  const r = {};
                  later(() => { r.result = st.map.get(key); if (r.onsuccess) r.onsuccess(); });
                  return r;
                },
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
const ChunkAssemblerRef = vm.runInThisContext('ChunkAssembler');

// chunk bytes recipe (same xorshift32 payload generator as gen_golden.js)
function xs32(s) { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s; }
function payloadBytes(seed, len) {
  const out = new Uint8Array(len);
  let s = seed >>> 0;
  for (let i = 0; i < len; i++) { if ((i & 3) === 0) s = xs32(s); out[i] = (s >>> (8 * (i & 3))) & 0xff; }
  return out;
}

const M = (totalChunks, totalFileSize, chunkSize, fileName) => ({ op: 'meta', totalChunks, totalFileSize, chunkSize, fileName });
const D = (seq, seed, len, crc = true) => ({ op: 'chunk', seq, seed, len, crc });
const A = { op: 'assemble' };
const SCENARIOS = {
  inorder: [M(4, 10000, 2600, 'a.bin'), D(0, 1, 2600), D(1, 2, 2600), D(2, 3, 2600), D(3, 4, 2200), A],
  shuffled_dups_crc: [M(6, 2900, 500, 'b.dat'), D(5, 11, 400), D(1, 12, 500), D(1, 13, 500), D(3, 14, 500, false),
    D(3, 15, 500), D(0, 16, 500), D(2, 17, 500), D(4, 18, 500), D(9, 19, 10), D(6, 20, 10), D(-1, 21, 7),
    D(-9, 22, 3), A],
  overflow: [M(2, 100, 64, 'o'), D(0, 31, 64), D(1, 32, 64), A],
  short_chunks_gap: [M(3, 300, 100, 's'), D(0, 41, 10), D(2, 42, 100), A],
  before_meta: [D(0, 51, 10), A],
  negative_total: [M(-16, 100, 10, 'n'), D(0, 61, 10), D(-20, 62, 4)],
  negative_small_total: [M(-3, 50, 10, 'm'), D(-5, 71, 5), D(-5, 72, 5), D(-2, 73, 3), D(0, 74, 5), A],
  remeta: [M(2, 20, 10, 'r1'), D(0, 81, 10), M(3, 30, 10, 'r2'), D(1, 82, 10), D(2, 83, 10), D(0, 84, 10), A],
  negative_size: [M(1, -5, 10, 'z'), D(0, 91, 3), A],
  zero_chunks: [M(0, 0, 0, 'e'), D(0, 101, 4), A],
  chunksize_zero: [M(2, 10, 0, 'c'), D(0, 111, 5), D(1, 112, 3), A],
  extra_big_total: [M(20000, 65536, 4096, 'big'), D(19999, 121, 16), D(16, 122, 4096), D(19999, 123, 16), A],
};

function snapshot(a) {
  const missing = a.totalChunks > 0 && a.totalChunks <= 64 ? a.getMissingChunks() : null;
  return {
    totalChunks: a.totalChunks, totalFileSize: a.totalFileSize, chunkSize: a.chunkSize, fileName: a.fileName,
    receivedCount: a.receivedCount, crcErrors: a.crcErrors, complete: a.isComplete(),
    bitmap: a.receivedBitmap ? Array.from(a.receivedBitmap.slice(0, 64)) : null,
    bitmapLen: a.receivedBitmap ? a.receivedBitmap.length : -1, missing,
  };
}

async function run(ops) {
  const a = new ChunkAssemblerRef();
  const steps = [];
  for (const o of ops) {
    let err = null, file = null;
    try {
      if (o.op === 'meta') {
        await a.handleMetadataFrame({ totalChunks: o.totalChunks, totalFileSize: o.totalFileSize, chunkSize: o.chunkSize, fileName: o.fileName });
      } else if (o.op === 'chunk') {
        await a.handleDataChunk(o.seq, payloadBytes(o.seed, o.len), o.crc);
      } else {
        const f = await a.assembleFile();
        file = Buffer.from(f).toString('hex');
      }
    } catch (e) {
      err = e.constructor.name;
    }
    steps.push({ state: snapshot(a), error: err, file });
  }
  return steps;
}

(async () => {
  const out = { generator: 'tests/golden/gen_assembler.js', reference: 'app.js ChunkAssembler (597-704)', scenarios: {} };
  for (const [name, ops] of Object.entries(SCENARIOS)) out.scenarios[name] = { ops, steps: await run(ops) };
  fs.writeFileSync(path.join(__dirname, 'assembler.json'), JSON.stringify(out));
  console.log('wrote', Object.keys(out.scenarios).length, 'scenarios');
})();
