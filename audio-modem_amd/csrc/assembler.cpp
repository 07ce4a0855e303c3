// assembler.cpp — the chunk protocol's receive-side bookkeeping (host C++).
//
// Restates app.js ChunkAssembler (597-704) and the result dispatch of
// StreamingReceiver._demodulateFrame (926-961) over amod_result records: received
// bitmap, duplicate suppression, CRC-error count, completion test, missing list and
// assembleFile's offsets. The IndexedDB object store becomes an in-memory map, or one
// file per chunk under a directory. The reference's quirks are kept, because a
// drop-in must behave the same on the same inputs:
//   * a metadata frame with totalChunks <= -8 raises RangeError (new Uint8Array of a
//     negative length) after the header fields were assigned; the bitmap stays;
//   * a negative seqNum below totalChunks is never seen as a duplicate (typed-array
//     reads past the ends are undefined, writes are dropped), so it counts every time;
//   * assembleFile raises TypeError before any metadata (no store), RangeError for a
//     negative totalFileSize or a chunk that runs past the end of the file.
// Pinned by tests/golden/assembler.json (the reference class run under Node).
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "amodem.h"

// The file-layout store: totalChunks x chunkSize bytes, chunk seq at seq * chunkSize, mapped
// at the metadata frame (address space only: MAP_NORESERVE, huge pages where the kernel
// offers them). A helper thread pre-faults the first kPopulateMax bytes of it
// (MADV_POPULATE_WRITE, contents untouched) while the receiver is still scanning, so the
// chunk stores that follow do not pay first-touch faults one page at a time (32k 2 KB
// chunks: 65 MB); pages past that window fault in as chunks arrive, so a header that
// claims a large file commits memory only for the chunks actually received (the reference
// allocates the file only in assembleFile, app.js:668). release() stops the helper at its
// next step instead of waiting for the whole window.
// A released arena is kept for the next one (one mapping of at most kPoolMax bytes,
// process-wide): a receiver serving recording after recording reuses the pages it has
// already faulted in, and its helper thread does not hold the address-space lock (read,
// 2 MB at a time) under the next receiver's host phase, whose own mappings (thread
// stacks, vectors) queue behind it (2.4 ms of the 32k-chunk stream's sparse setup). Only
// chunks a Loc records are ever read back, so the previous file's bytes stay unseen.
struct ArenaPool {
  static constexpr size_t kPoolMax = size_t(1) << 30;
  std::mutex mu;
  uint8_t *p = nullptr;
  size_t n = 0, populated = 0;
};
static ArenaPool &arena_pool() {
  static ArenaPool pool;
  return pool;
}

struct FileArena {
  static constexpr size_t kPopulateMax = size_t(256) << 20;
  uint8_t *p = nullptr;
  size_t n = 0;                        // the mapping's length (>= the file span)
  std::atomic<size_t> populated{0};    // bytes from the start the helper has faulted in
  std::thread filler;
  std::atomic<bool> stop{false};
  // experiments (AMOD_ASM_NO_POPULATE): no background population, so the copies take the
  // first-touch faults; read once per assembler, when it is created
  const bool no_populate = getenv("AMOD_ASM_NO_POPULATE") != nullptr;
  ~FileArena() { release(); }
  void release() {
    stop.store(true, std::memory_order_relaxed);
    if (filler.joinable()) filler.join();
    stop.store(false, std::memory_order_relaxed);
    if (p) {
      ArenaPool &pool = arena_pool();
      std::lock_guard<std::mutex> lk(pool.mu);
      if (n <= ArenaPool::kPoolMax) {
        if (pool.p) munmap(pool.p, pool.n);
        pool.p = p; pool.n = n; pool.populated = populated.load(std::memory_order_relaxed);
      } else {
        munmap(p, n);
      }
    }
    p = nullptr;
    n = 0;
    populated.store(0, std::memory_order_relaxed);
  }
  bool map(size_t bytes) {
    release();
    if (!bytes) return false;
    size_t done = 0;
    {
      ArenaPool &pool = arena_pool();
      std::lock_guard<std::mutex> lk(pool.mu);
      if (pool.p && pool.n >= bytes && pool.n <= 2 * bytes + (size_t(64) << 20)) { // (not a far larger one)
        p = pool.p; n = pool.n; done = pool.populated;
        pool.p = nullptr; pool.n = pool.populated = 0;
      }
    }
    if (!p) {
      void *q = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
      if (q == MAP_FAILED) return false;
      p = (uint8_t *)q;
      n = bytes;
#ifdef MADV_HUGEPAGE
      (void)madvise(p, n, MADV_HUGEPAGE);
#endif
    }
    populated.store(done, std::memory_order_relaxed);
    const size_t len = std::min(n, kPopulateMax);
    if (no_populate || done >= len) return true;
    filler = std::thread([this, q = p, from = done, len] {
      constexpr int kPopulateWrite = 23; // MADV_POPULATE_WRITE (Linux 5.14)
      // one huge page per call: each call holds the address-space lock (read) while it
      // zeroes, and the receiver's own mappings (thread stacks, vectors) wait for it
      constexpr size_t kStep = size_t(2) << 20;
      for (size_t o = from; o < len && !stop.load(std::memory_order_relaxed); o += kStep) {
        const size_t m = std::min(kStep, len - o);
        if (madvise(q + o, m, kPopulateWrite) != 0) { // older kernels: touch every page, value kept
          for (size_t b = o; b < o + m; b += 4096) __atomic_fetch_add(q + b, (uint8_t)0, __ATOMIC_RELAXED);
        }
        populated.store(o + m, std::memory_order_relaxed);
      }
    });
    return true;
  }
};

struct amod_assembler {
  int32_t total_chunks = 0, total_size = 0, chunk_size = 0;
  std::vector<uint8_t> name;
  bool has_bitmap = false;
  std::vector<uint8_t> bitmap;
  int32_t received = 0, crc_errors = 0;
  bool has_store = false;                          // IndexedDB opened by a metadata frame
  // memory store: chunks of seq 0 <= seq < totalChunks (up to 1 M) and at most chunkSize
  // bytes in the file-layout arena; any other chunk appended to `arena`. seqNum ->
  // (offset, length, in file arena), dense for 0 <= seq < totalChunks, a map otherwise (a
  // rewrite appends a new copy)
  struct Loc { int64_t off; int32_t len; bool file; };
  FileArena farena;
  std::vector<uint8_t> arena;
  std::vector<Loc> dense;                          // offset -1: none
  std::map<int32_t, Loc> other;
  std::map<int32_t, bool> files;                   // file store: the seqNums written
  std::string dir;                                 // file store when not empty
  int32_t frames_decoded = 0, frame_errors = 0;    // StreamingReceiver counters

  std::string path(int32_t seq) const { return dir + "/chunk_" + std::to_string(seq) + ".bin"; }
  void clear_store() {
    if (!dir.empty())
      for (const auto &kv : files) remove(path(kv.first).c_str());
    files.clear();
    arena.clear();
    // (dense up to 1 M chunks; a larger claimed totalChunks keeps the map alone)
    dense.assign(total_chunks > 0 && total_chunks <= (1 << 20) ? (size_t)total_chunks : 0, Loc{-1, 0, false});
    other.clear();
    farena.release();
    // only for a consistent header (the chunks tile the file: totalChunks x chunkSize at
    // most one chunk past totalFileSize) of at most 4 GB: a claimed size is never mapped
    // and populated blindly
    const int64_t span = (int64_t)dense.size() * chunk_size;
    if (dir.empty() && !dense.empty() && chunk_size > 0 && total_size > 0 &&
        span <= (int64_t)total_size + chunk_size && span <= (int64_t(4) << 30))
      (void)farena.map((size_t)span);
  }
  bool put(int32_t seq, const uint8_t *d, int32_t n) {
    if (dir.empty()) {
      const bool in_dense = seq >= 0 && (size_t)seq < dense.size();
      if (in_dense && farena.p && n <= chunk_size) {
        const int64_t off = (int64_t)seq * chunk_size;
        memcpy(farena.p + off, d, (size_t)n);
        dense[(size_t)seq] = Loc{off, n, true};
        return true;
      }
      const Loc e{(int64_t)arena.size(), n, false};
      arena.insert(arena.end(), d, d + n);
      if (in_dense) dense[(size_t)seq] = e;
      else other[seq] = e;
      return true;
    }
    FILE *f = fopen(path(seq).c_str(), "wb");
    if (!f) return false;
    const bool ok = n == 0 || fwrite(d, 1, (size_t)n, f) == (size_t)n;
    fclose(f);
    files[seq] = true; // the bytes live in the file
    return ok;
  }
  // chunk seq's bytes in memory (memory store): pointer and length, or null
  const uint8_t *mem(int32_t seq, int32_t &len) const {
    Loc e{-1, 0, false};
    if (seq >= 0 && (size_t)seq < dense.size()) e = dense[(size_t)seq];
    else if (auto it = other.find(seq); it != other.end()) e = it->second;
    if (e.off < 0) return nullptr;
    len = e.len;
    return (e.file ? farena.p : arena.data()) + e.off;
  }
  bool get(int32_t seq, std::vector<uint8_t> &out) const {
    if (dir.empty()) {
      int32_t len = 0;
      const uint8_t *p = mem(seq, len);
      if (!p) return false;
      out.assign(p, p + len);
      return true;
    }
    if (!files.count(seq)) return false;
    {
    FILE *f = fopen(path(seq).c_str(), "rb");
    if (!f) return false;
    out.clear();
    uint8_t buf[65536];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
    fclose(f);
    return true;
    }
  }
  bool is_received(int64_t seq) const {
    if (!has_bitmap || seq < 0 || (seq >> 3) >= (int64_t)bitmap.size()) return false;
    return bitmap[seq >> 3] & (1u << (seq & 7));
  }
};

extern "C" {

int amod_asm_open(const char *dir, amod_assembler **out) {
  if (!out) return AMOD_ERR_ARG;
  auto *a = new (std::nothrow) amod_assembler();
  if (!a) return AMOD_ERR_NOMEM;
  if (dir && *dir) a->dir = dir;
  *out = a;
  return AMOD_SUCCESS;
}

int amod_asm_close(amod_assembler *a) {
  delete a;
  return AMOD_SUCCESS;
}

// handleMetadataFrame (app.js:610-626)
int amod_asm_metadata(amod_assembler *a, int32_t total_chunks, int32_t total_size, int32_t chunk_size,
                      const uint8_t *name, int32_t name_len) {
  if (!a || name_len < 0) return AMOD_ERR_ARG;
  a->total_chunks = total_chunks;
  a->total_size = total_size;
  a->chunk_size = chunk_size;
  a->name.assign(name, name + name_len);
  // new Uint8Array(Math.ceil(totalChunks / 8)): -7..-1 give -0 = length 0
  const int64_t len = total_chunks >= 0 ? ((int64_t)total_chunks + 7) / 8 : -((-(int64_t)total_chunks) / 8);
  if (len < 0) return AMOD_ASM_RANGE_ERROR;
  a->bitmap.assign((size_t)len, 0);
  a->has_bitmap = true;
  a->received = 0;
  a->crc_errors = 0;
  a->clear_store();
  a->has_store = true;
  return AMOD_SUCCESS;
}

// handleDataChunk (app.js:628-648); returns 1 if the chunk was stored, 0 if ignored
int amod_asm_chunk(amod_assembler *a, int32_t seq, const uint8_t *data, int32_t len, int32_t crc_valid) {
  if (!a || len < 0) return AMOD_ERR_ARG;
  if (!a->has_bitmap) return 0;
  if (seq >= a->total_chunks) return 0;
  if (!crc_valid) {
    ++a->crc_errors;
    return 0;
  }
  const int64_t byte = (int64_t)seq >> 3;
  const int bit = seq & 7;
  const bool inside = byte >= 0 && byte < (int64_t)a->bitmap.size();
  if (inside && (a->bitmap[byte] & (1u << bit))) return 0; // duplicate
  if (inside) a->bitmap[byte] |= (uint8_t)(1u << bit);
  ++a->received;
  if (!a->put(seq, data, len)) return AMOD_ERR_NOMEM;
  return 1;
}

// amod_asm_chunk whose bytes the caller copies: when the chunk goes to the file-layout
// arena, *dst is where its len bytes belong and nothing is copied here (the streaming
// receiver copies a batch's chunks on several threads, before any other assembler call);
// otherwise the chunk is stored as amod_asm_chunk does and *dst is null
int amod_asm_chunk_at(amod_assembler *a, int32_t seq, const uint8_t *data, int32_t len, int32_t crc_valid,
                      uint8_t **dst) {
  if (!dst) return AMOD_ERR_ARG;
  *dst = nullptr;
  if (!a || len < 0) return AMOD_ERR_ARG;
  const bool arena = a->dir.empty() && seq >= 0 && (size_t)seq < a->dense.size() && a->farena.p && len <= a->chunk_size;
  if (!arena) return amod_asm_chunk(a, seq, data, len, crc_valid);
  if (!a->has_bitmap) return 0;
  if (seq >= a->total_chunks) return 0;
  if (!crc_valid) {
    ++a->crc_errors;
    return 0;
  }
  const int64_t byte = (int64_t)seq >> 3;
  const int bit = seq & 7;
  const bool inside = byte >= 0 && byte < (int64_t)a->bitmap.size();
  if (inside && (a->bitmap[byte] & (1u << bit))) return 0; // duplicate
  if (inside) a->bitmap[byte] |= (uint8_t)(1u << bit);
  ++a->received;
  const int64_t off = (int64_t)seq * a->chunk_size;
  a->dense[(size_t)seq] = amod_assembler::Loc{off, len, true};
  *dst = a->farena.p + off;
  return 1;
}

// StreamingReceiver._demodulateFrame's dispatch (app.js:926-961) over n decode results
int amod_asm_feed(amod_assembler *a, const amod_result *res, const uint8_t *payload, int64_t stride, int32_t n) {
  if (!a || n < 0 || (n && (!res || !payload))) return AMOD_ERR_ARG;
  for (int32_t i = 0; i < n; ++i) {
    const amod_result &r = res[i];
    const uint8_t *slot = payload + (int64_t)i * stride;
    if (r.status != AMOD_OK) { ++a->frame_errors; continue; }
    ++a->frames_decoded;
    if (r.frame_type == 0xFE) {
      if (r.crc_valid) {
        if (amod_asm_metadata(a, r.total_chunks, r.total_size, r.chunk_size, slot + r.name_off, r.name_len) ==
            AMOD_ASM_RANGE_ERROR)
          ++a->frame_errors; // the thrown RangeError lands in the receiver's catch
      } else {
        ++a->frame_errors;
      }
    } else if (r.frame_type == 0xFF) {
      const int rc = amod_asm_chunk(a, r.seq_num, slot + r.data_off, r.data_len, r.crc_valid);
      if (rc < 0) return rc;
    }
  }
  return AMOD_SUCCESS;
}

int amod_asm_state(const amod_assembler *a, amod_asm_info *out) {
  if (!a || !out) return AMOD_ERR_ARG;
  out->total_chunks = a->total_chunks;
  out->total_size = a->total_size;
  out->chunk_size = a->chunk_size;
  out->received = a->received;
  out->crc_errors = a->crc_errors;
  out->complete = a->received == a->total_chunks; // isComplete (app.js:655-657)
  out->has_bitmap = a->has_bitmap;
  out->bitmap_len = a->has_bitmap ? (int64_t)a->bitmap.size() : -1;
  out->frames_decoded = a->frames_decoded;
  out->frame_errors = a->frame_errors;
  out->name_len = (int32_t)a->name.size();
  out->reserved = 0;
  return AMOD_SUCCESS;
}

int64_t amod_asm_bitmap(const amod_assembler *a, uint8_t *out, int64_t cap) {
  if (!a) return AMOD_ERR_ARG;
  const int64_t n = (int64_t)a->bitmap.size();
  if (out) std::copy(a->bitmap.begin(), a->bitmap.begin() + std::min(n, std::max<int64_t>(cap, 0)), out);
  return n;
}

int64_t amod_asm_name(const amod_assembler *a, uint8_t *out, int64_t cap) {
  if (!a) return AMOD_ERR_ARG;
  const int64_t n = (int64_t)a->name.size();
  if (out) std::copy(a->name.begin(), a->name.begin() + std::min(n, std::max<int64_t>(cap, 0)), out);
  return n;
}

// getMissingChunks (app.js:659-665): count, first min(count, cap) indices in out
int64_t amod_asm_missing(const amod_assembler *a, int32_t *out, int64_t cap) {
  if (!a) return AMOD_ERR_ARG;
  int64_t k = 0;
  for (int64_t i = 0; i < a->total_chunks; ++i)
    if (!a->is_received(i)) {
      if (out && k < cap) out[k] = (int32_t)i;
      ++k;
    }
  return k;
}

// assembleFile (app.js:667-686): the file's size (out NULL: sizing), or an error
int64_t amod_asm_file(const amod_assembler *a, uint8_t *out, int64_t cap) {
  if (!a) return AMOD_ERR_ARG;
  if (!a->has_store) return AMOD_ASM_TYPE_ERROR;
  if (a->total_size < 0) return AMOD_ASM_RANGE_ERROR;
  const int64_t size = a->total_size;
  if (!out) return size;
  if (cap < size) return AMOD_ERR_ARG;
  std::fill(out, out + size, 0);
  std::vector<uint8_t> d;
  for (int64_t i = 0; i < a->total_chunks; ++i) {
    const int64_t off = i * (int64_t)a->chunk_size;
    if (a->dir.empty()) {
      int32_t len = 0;
      const uint8_t *p = a->mem((int32_t)i, len);
      if (!p) continue;
      if (off + (int64_t)len > size) return AMOD_ASM_RANGE_ERROR; // Uint8Array.set past the end
      memcpy(out + off, p, (size_t)len);
      continue;
    }
    if (!a->get((int32_t)i, d)) continue;
    if (off + (int64_t)d.size() > size) return AMOD_ASM_RANGE_ERROR;
    std::copy(d.begin(), d.end(), out + off);
  }
  return size;
}

} // extern "C"
