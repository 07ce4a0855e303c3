// stream.cpp — app.js StreamingReceiver (706-998) over a whole recorded stream.
//
// The reference runs per 4096-sample audio block (ScriptProcessor, app.js:1103):
// EMA DC removal, ring buffer, then one step of its state machine (scan for a
// Schmidl-Cox preamble / refine by cross-correlation / collect / demodulate with
// decodeChunkFrame + ChunkAssembler dispatch). Here:
//
//   GPU   k_ema       the DC removal, bit-exact (k_stream.hip)
//         k_sc_screen hot 32-sample blocks (metric >= 0.25 at the block start)
//         k_fine      the refinement's cross-correlation sums, in the reference's
//                     order, for every position within 448 samples of a hot block
//         k_window    per-frame peak normalisation, then k_decode_fast/_exact in chunk
//                     mode over all windows of a batch
//   host  the state machine itself, replayed exactly in IEEE double: the sliding
//         Schmidl-Cox recurrence with its block-boundary behaviour (the state left at
//         scanEnd is re-read one position later, app.js:782-847), the 0.5 threshold,
//         the 0.7 x best commit and the end-of-block commit, refine windows clipped to
//         the ring buffer, frame windows from estimateFrameSamples(chunkSize + 11 | 280).
//         The fine metric comes from k_fine's exact sums (host fallback for a position
//         outside the precomputed ranges); frames are decoded in batches on the GPU,
//         and a batch is rolled back to the frame after which a metadata result
//         changed the window length (metaReceived / chunkSize, app.js:889-896).
// Decisions are the reference's own arithmetic, so outcomes match it exactly; pinned
// by tests/golden/stream.json (the reference receiver run on recipe streams).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <thread>
#include <unordered_map>
#include <vector>

#include "amodem_internal.h"

// assembler.cpp: amod_asm_chunk with the copy left to the caller (file-layout arena)
extern "C" int amod_asm_chunk_at(amod_assembler *a, int32_t seq, const uint8_t *data, int32_t len, int32_t crc_valid,
                                 uint8_t **dst);

namespace {

// A batch's chunk copies (payload row -> the assembler's file-layout arena) on a few
// persistent threads: one thread moved 32k x 2 KB at ~10 GB/s (4-5 ms of the C4-scale
// receiver's host phase). run() returns once every copy is done.
struct CopyPool {
  struct Item { uint8_t *dst; const uint8_t *src; size_t n; };
  std::vector<Item> items; // being filled (the next start() hands them to the workers)
  std::vector<Item> work;  // being copied
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable go, done;
  uint64_t gen = 0;
  int busy = 0;
  bool stop = false;
  std::atomic<size_t> next{0};
  explicit CopyPool(int n) {
    for (int i = 0; i < n; ++i) th.emplace_back([this] { worker(); });
  }
  ~CopyPool() {
    { std::lock_guard<std::mutex> lk(m); stop = true; }
    go.notify_all();
    for (auto &t : th) t.join();
  }
  void drain() {
    for (size_t i; (i = next.fetch_add(1)) < work.size();) std::memcpy(work[i].dst, work[i].src, work[i].n);
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m);
        go.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      drain();
      { std::lock_guard<std::mutex> lk(m); --busy; }
      done.notify_one();
    }
  }
  // the copies handed over by the last start() are done
  void wait() {
    std::unique_lock<std::mutex> lk(m);
    done.wait(lk, [&] { return busy == 0; });
    work.clear();
  }
  // hands `items` to the workers and returns (after the previous batch's copies are done)
  void start() {
    wait();
    if (items.empty()) return;
    if (th.empty()) {
      for (auto &it : items) std::memcpy(it.dst, it.src, it.n);
      items.clear();
      return;
    }
    work.swap(items);
    items.clear();
    next = 0;
    { std::lock_guard<std::mutex> lk(m); busy = (int)th.size(); ++gen; }
    go.notify_all();
  }
  // every copy enqueued so far done, on this thread too
  void run() {
    wait();
    for (auto &it : items) std::memcpy(it.dst, it.src, it.n);
    items.clear();
  }
};

constexpr int64_t kBlock = 4096;      // ScriptProcessor buffer (app.js:1103)
const int64_t kEmaChunk = amod_ema_chunk(); // k_ema chunk (EMA end states are reported per chunk)
constexpr int kBatch = 4096;          // frames decoded per GPU batch (after the metadata frame)
constexpr int64_t kUpPieceSamples = int64_t(16) << 20; // host streams: samples per uploaded piece (64 MB)
constexpr int kGranLog = 10, kGran = 1 << kGranLog; // sparse host copy granule (samples)
constexpr int64_t kFirstPiece = int64_t(1) << 20;   // sparse mode: the first piece copied at once
// blocks a GPU gap scan runs before it leaves the gap to the host (the kernel's time is its
// longest gap's: a stream's tail or a long silence is the host's)
constexpr int kGapBlocks = 8;
enum { IDLE = 0, DETECTED = 1, COLLECTING = 2 };

struct DBuf {
  void *p = nullptr;
  size_t cap = 0;
  ~DBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t n) { // grow-only: kept across calls (the context's stream cache)
    n = std::max<size_t>(n, 256);
    if (p && cap >= n) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
    const hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) cap = n;
    return e;
  }
  template <typename T> T *as() const { return (T *)p; }
};

#define S_TRY(expr)                                                                     \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return amod_ctx_fail(ctx, hipGetErrorString(e_), AMOD_ERR_HIP); \
  } while (0)

// receiver state that a rollback restores (everything the next block depends on)
struct RxState {
  int64_t block = 0;             // next block to process
  int state = IDLE;
  bool ac_init = false;
  int64_t ac_pos = 0;
  double ac_p = 0, ac_ra = 0, ac_rb = 0;
  int64_t pre_pos = -1, frame_end = -1;
  bool meta_received = false;
  int32_t chunk_size = 0;        // assembler.chunkSize as the window length sees it
};

struct FineTable {
  std::vector<int64_t> first, base, count;
  const double *metric = nullptr; // k_fine's metrics (pinned), NaN where the reference skips
  // or, with the metrics kept on the device (k_gap_refine reads them there), the device
  // array: a refinement the host runs itself (before the metadata frame, a stream without
  // one, a window clamped to the ring) fetches its range's metrics once, on first use,
  // instead of correlating every position on the host
  const double *dmetric = nullptr;
  hipStream_t fetch_stream = nullptr; // (non-blocking: a null-stream copy waited for queued decodes)
  double *fetch_bounce = nullptr;     // pinned, >= the longest range (device-to-pageable copies were slow)
  mutable std::mutex fmu;
  mutable std::unordered_map<size_t, std::vector<double>> fetched;
  const double *range_metrics(size_t r) const {
    if (metric) return metric + base[r];
    if (!dmetric) return nullptr;
    std::lock_guard<std::mutex> lk(fmu);
    auto it = fetched.find(r);
    if (it == fetched.end()) {
      std::vector<double> v((size_t)count[r]);
      double *const dst = fetch_bounce ? fetch_bounce : v.data();
      if (hipMemcpyAsync(dst, dmetric + base[r], sizeof(double) * v.size(), hipMemcpyDeviceToHost, fetch_stream) !=
              hipSuccess ||
          hipStreamSynchronize(fetch_stream) != hipSuccess)
        return nullptr;
      if (fetch_bounce) std::memcpy(v.data(), fetch_bounce, sizeof(double) * v.size());
      it = fetched.emplace(r, std::move(v)).first;
    }
    return it->second.data();
  }
  // refine walks consecutive positions: `last` (the caller's cursor) is tried first
  bool lookup(int64_t d, double &m, size_t &last) const {
    if (!metric && !dmetric) return false;
    size_t r = last;
    if (r >= first.size() || d < first[r] || d >= first[r] + count[r]) {
      auto it = std::upper_bound(first.begin(), first.end(), d);
      if (it == first.begin()) return false;
      r = (size_t)(it - first.begin()) - 1;
      last = r;
    }
    if (d >= first[r] + count[r]) return false;
    const double *rm = range_metrics(r);
    if (!rm) return false;
    m = rm[d - first[r]];
    return true;
  }
  // the metrics of positions [d0, d1] when one range holds them all, else nullptr
  const double *span(int64_t d0, int64_t d1, size_t &last) const {
    double m;
    if (!lookup(d0, m, last) || d1 >= first[last] + count[last]) return nullptr;
    return range_metrics(last) + (d0 - first[last]);
  }
};

// k_gap_refine's refinement of a detection at pre_pos (window pre_pos +- 3 cp)
struct GpuRefine {
  int64_t pre_pos, best_pos;
  double best;
};

struct Receiver {
  const amod_cfg *cfg;
  int64_t lo = 0, nloc = 0, cap = 0; // y[i] is stream sample lo + i, i < nloc
  const float *y = nullptr; // cleaned stream (host)
  std::vector<float> pre1;
  double pre1_energy = 0;
  const FineTable *fine = nullptr;
  const std::vector<GpuRefine> *refs = nullptr; // sorted by pre_pos
  int64_t ref_hits = 0;
  int32_t est_payload = -1, est_samples = 0; // estimateFrameSamples(max_payload), cached
  RxState st;
  std::vector<std::pair<int64_t, int64_t>> *fails = nullptr; // (block, preambleGlobalPos) of failed refinements
  int64_t fine_host = 0; // positions the host had to correlate itself
  size_t cursor = 0;     // FineTable lookup cursor
  // diagnostics (AMOD_STREAM_DIAG): scan positions stepped, time spent waiting for pieces
  int64_t scanned = 0;
  mutable double wait_ms = 0;
  double scan_ms = 0, refine_ms = 0; // (only timed with AMOD_STREAM_DIAG)
  bool timed = false;
  // speculative gap scans from the GPU (k_gap_scan), sorted by start; adopted when the
  // receiver stands exactly at a record's start and its detection falls before `stop_block`
  const std::vector<amod::GapScan> *gaps = nullptr;
  int64_t stop_block = INT64_MAX;
  int64_t gap_hits = 0;
  bool adopt_gap() {
    if (!gaps || st.ac_init || st.state != IDLE) return false;
    auto it = std::lower_bound(gaps->begin(), gaps->end(), st.ac_pos,
                               [](const amod::GapScan &g, int64_t p) { return g.s0 < p; });
    if (it == gaps->end() || it->s0 != st.ac_pos || it->b1 != st.block || it->det_block >= stop_block) return false;
    st.block = it->det_block; // (the caller steps past it)
    st.ac_pos = it->ac_pos; st.ac_p = it->p; st.ac_ra = it->ra; st.ac_rb = it->rb; st.ac_init = true;
    st.pre_pos = it->pre_pos; st.state = DETECTED;
    scanned += it->scanned;
    ++gap_hits;
    return true;
  }

  // the host copy of the cleaned stream arrives in pieces: local samples [0, avail) are
  // there; a read past it waits for the piece that holds it
  const std::function<void(int64_t)> *wait_y = nullptr;
  mutable int64_t avail = INT64_MAX;
  // live mode (amod_live): the reference's RingBuffer itself; getRange reads
  // buffer[i mod capacity] for any i at or after the oldest sample (app.js:580-589)
  const float *ring = nullptr;
  int64_t tw_live = -1; // totalWritten (live mode)
  // sparse host copy (SparseCopy below): local granule g (kGran samples) is at gptr[g], or
  // not on the host yet (null: present(g) brings it and returns its pointer)
  std::atomic<const float *> *gptr = nullptr;
  const std::function<const float *(int64_t)> *present = nullptr;
  const std::function<const float *(int64_t)> *copied = nullptr; // granule g if it is (being) copied, else null
  const float *granule(int64_t g) const {
    const float *p = gptr[g].load(std::memory_order_acquire);
    return p ? p : (*present)(g);
  }
  const float *peek(int64_t g) const { // granule g if on the host or on its way (never fetched)
    const float *p = gptr[g].load(std::memory_order_acquire);
    return p ? p : (*copied)(g);
  }
  double S(int64_t i) const {
    if (ring) { int64_t r = i % cap; if (r < 0) r += cap; return (double)ring[r]; }
    if (i < lo || i >= lo + nloc) return 0.0;
    if (gptr) return (double)granule((i - lo) >> kGranLog)[(i - lo) & (kGran - 1)];
    if (i - lo >= avail) {
      const auto t0 = std::chrono::steady_clock::now();
      (*wait_y)(i - lo + 1);
      avail = piece_end(i - lo);
      wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return (double)y[i - lo];
  }
  std::function<int64_t(int64_t)> piece_end;
  int64_t tw() const { return tw_live >= 0 ? tw_live : (st.block + 1) * kBlock; } // totalWritten after this block's write

  // _scanForPreamble (app.js:775-847)
  void scan() {
    if (adopt_gap()) return;
    const int64_t half = 256, total = tw(), oldest = total - cap;
    if (st.ac_pos < oldest + 2 * half) { st.ac_pos = std::max<int64_t>(oldest + 2 * half, 0); st.ac_init = false; }
    const int64_t scan_end = total - 2 * half;
    if (st.ac_pos > scan_end) return;
    if (!st.ac_init) {
      st.ac_p = 0; st.ac_ra = 0; st.ac_rb = 0;
      for (int64_t m = 0; m < half; ++m) {
        const double a = S(st.ac_pos + m), b = S(st.ac_pos + m + half);
        st.ac_p += a * b; st.ac_ra += a * a; st.ac_rb += b * b;
      }
      st.ac_init = true;
    }
    const double min_e = 0.001;
    double best = 0;
    int64_t best_pos = -1;
    // sparse host copy: positions whose reads lie in one contiguous run of granules on the
    // host are stepped straight from the array, the others one at a time through S()
    // (which brings their granule); only granules the scan actually reads are fetched
    if (!ring && gptr && st.ac_pos >= lo && total <= lo + nloc) {
      while (st.ac_pos <= scan_end) {
        const int64_t g0 = (st.ac_pos - lo) >> kGranLog, glim = (total - 1 - lo) >> kGranLog;
        const float *p0 = granule(g0);
        int64_t g = g0 + 1;
        while (g <= glim && peek(g) == p0 + (g - g0) * kGran) ++g;
        const int64_t lim = std::min(scan_end, lo + g * kGran - 2 * half - 1); // reads pos + 512 < run end
        const bool det = lim >= st.ac_pos ? scan_direct(p0 - (lo + g0 * kGran), lim, scan_end, min_e, best, best_pos)
                                          : scan_step(scan_end, min_e, best, best_pos);
        if (det) return;
      }
      if (best > 0.5 && best_pos >= 0) { st.pre_pos = best_pos; st.state = DETECTED; }
      return;
    }
    // the whole host copy: every sample this call can read, [ac_pos, total), is there
    if (!ring && !gptr && st.ac_pos >= lo && total <= lo + nloc && total > st.ac_pos) {
      (void)S(total - 1); // waits for the piece holding the last one
      if (total - lo <= avail) {
        if (!scan_direct(y - lo, scan_end, scan_end, min_e, best, best_pos) && best > 0.5 && best_pos >= 0) {
          st.pre_pos = best_pos;
          st.state = DETECTED;
        }
        return;
      }
    }
    // p^2 < 0.49 ra rb (rounded products, relative error ~1e-16) proves the rounded
    // quotient is below 0.5: the division is only evaluated where it can matter
    while (st.ac_pos <= scan_end) {
      if (st.ac_ra > min_e && st.ac_rb > min_e) {
        const double pp = st.ac_p * st.ac_p, rr = st.ac_ra * st.ac_rb;
        if (pp >= 0.49 * rr) {
          const double metric = pp / rr;
          if (metric > 0.5 && metric > best) { best = metric; best_pos = st.ac_pos; }
        }
      }
      if (st.ac_pos < scan_end) {
        const double a_out = S(st.ac_pos), mid = S(st.ac_pos + half), b_in = S(st.ac_pos + 2 * half);
        st.ac_p += mid * b_in - a_out * mid;
        st.ac_ra += mid * mid - a_out * a_out;
        st.ac_rb += b_in * b_in - mid * mid;
      }
      st.ac_pos++;
      ++scanned;
      if (best > 0.5 && best_pos >= 0 && st.ac_ra > min_e && st.ac_rb > min_e) {
        const double cur = (st.ac_p * st.ac_p) / (st.ac_ra * st.ac_rb);
        if (cur < best * 0.7) { st.pre_pos = best_pos; st.state = DETECTED; return; }
      }
    }
    if (best > 0.5 && best_pos >= 0) { st.pre_pos = best_pos; st.state = DETECTED; }
  }

  // the scan loop above over a plain array yy (yy[i] = stream sample i), positions up to
  // lim (<= scan_end): the same operations in the same order; true when it detected
  bool scan_direct(const float *yy, int64_t lim, int64_t scan_end, double min_e, double &best, int64_t &best_pos) {
    const int64_t half = 256;
    double p = st.ac_p, ra = st.ac_ra, rb = st.ac_rb;
    int64_t pos = st.ac_pos;
    // Quiet stretches in batches: the increments of a batch are independent of the sums
    // (one vectorisable pass, each the same rounded expression as the loop's), the three
    // sums then advance through them in order, and positions failing the metric
    // pre-check while no detection is pending change nothing else. The first batch
    // position that passes it is stepped by the position-by-position body.
    constexpr int kB = 64;
    alignas(64) double ip[kB], ia[kB], ib[kB], sp[kB], sa[kB], sb[kB];
    while (pos <= lim) {
      if (!(best > 0.5 && best_pos >= 0) && pos + kB - 1 <= std::min(lim, scan_end - 1)) {
        const float *const a0 = yy + pos, *const m0 = yy + pos + half, *const b0 = yy + pos + 2 * half;
        for (int j = 0; j < kB; ++j) {
          const double a_out = a0[j], mid = m0[j], b_in = b0[j];
          ip[j] = mid * b_in - a_out * mid;
          ia[j] = mid * mid - a_out * a_out;
          ib[j] = b_in * b_in - mid * mid;
        }
        double q = p, r = ra, t = rb;
        for (int j = 0; j < kB; ++j) { // the state at position pos + j, then its update
          sp[j] = q; sa[j] = r; sb[j] = t;
          q += ip[j]; r += ia[j]; t += ib[j];
        }
        int hit = kB;
        for (int j = 0; j < kB; ++j)
          if (sa[j] > min_e && sb[j] > min_e && sp[j] * sp[j] >= 0.49 * (sa[j] * sb[j])) { hit = j; break; }
        if (hit == kB) {
          p = q; ra = r; rb = t;
          pos += kB;
          scanned += kB;
          continue;
        }
        p = sp[hit]; ra = sa[hit]; rb = sb[hit]; // positions before it were no-ops
        pos += hit;
        scanned += hit;
      }
      if (ra > min_e && rb > min_e) {
        const double pp = p * p, rr = ra * rb;
        if (pp >= 0.49 * rr) {
          const double metric = pp / rr;
          if (metric > 0.5 && metric > best) { best = metric; best_pos = pos; }
        }
      }
      if (pos < scan_end) {
        const double a_out = yy[pos], mid = yy[pos + half], b_in = yy[pos + 2 * half];
        p += mid * b_in - a_out * mid;
        ra += mid * mid - a_out * a_out;
        rb += b_in * b_in - mid * mid;
      }
      pos++;
      ++scanned;
      if (best > 0.5 && best_pos >= 0 && ra > min_e && rb > min_e) {
        const double cur = (p * p) / (ra * rb);
        if (cur < best * 0.7) {
          st.ac_p = p; st.ac_ra = ra; st.ac_rb = rb; st.ac_pos = pos;
          st.pre_pos = best_pos; st.state = DETECTED;
          return true;
        }
      }
    }
    st.ac_p = p; st.ac_ra = ra; st.ac_rb = rb; st.ac_pos = pos;
    return false;
  }
  // one position of the scan loop through S(); true when it detected
  bool scan_step(int64_t scan_end, double min_e, double &best, int64_t &best_pos) {
    const int64_t half = 256;
    if (st.ac_ra > min_e && st.ac_rb > min_e) {
      const double pp = st.ac_p * st.ac_p, rr = st.ac_ra * st.ac_rb;
      if (pp >= 0.49 * rr) {
        const double metric = pp / rr;
        if (metric > 0.5 && metric > best) { best = metric; best_pos = st.ac_pos; }
      }
    }
    if (st.ac_pos < scan_end) {
      const double a_out = S(st.ac_pos), mid = S(st.ac_pos + half), b_in = S(st.ac_pos + 2 * half);
      st.ac_p += mid * b_in - a_out * mid;
      st.ac_ra += mid * mid - a_out * a_out;
      st.ac_rb += b_in * b_in - mid * mid;
    }
    st.ac_pos++;
    ++scanned;
    if (best > 0.5 && best_pos >= 0 && st.ac_ra > min_e && st.ac_rb > min_e) {
      const double cur = (st.ac_p * st.ac_p) / (st.ac_ra * st.ac_rb);
      if (cur < best * 0.7) { st.pre_pos = best_pos; st.state = DETECTED; return true; }
    }
    return false;
  }

  // _refineAndCollect (app.js:849-898)
  void refine() {
    const int64_t plen = cfg->symbol_len, radius = 3 * (int64_t)cfg->cp_len, total = tw();
    if (total < st.pre_pos + plen + radius) return;
    const int64_t fs = std::max(total - cap, st.pre_pos - radius), fe = std::min(total - plen, st.pre_pos + radius);
    double best = -INFINITY;
    int64_t best_pos = st.pre_pos;
    const GpuRefine *gr = nullptr;
    if (refs && fs == st.pre_pos - radius && fe == st.pre_pos + radius) {
      auto it = std::lower_bound(refs->begin(), refs->end(), st.pre_pos,
                                 [](const GpuRefine &a, int64_t p) { return a.pre_pos < p; });
      if (it != refs->end() && it->pre_pos == st.pre_pos) gr = &*it;
    }
    if (gr) {
      best = gr->best; // the same window's first maximum, from the GPU's metrics
      best_pos = gr->best_pos;
      ++ref_hits;
    } else if (const double *mv = (fine && fs <= fe) ? fine->span(fs, fe, cursor) : nullptr) {
      for (int64_t d = fs; d <= fe; ++d) // the common case: one contiguous run of k_fine metrics
        if (mv[d - fs] > best) { best = mv[d - fs]; best_pos = d; }
    } else for (int64_t d = fs; d <= fe; ++d) {
      double metric;
      if (!fine || !fine->lookup(d, metric, cursor)) {
        double corr = 0, se = 0;
        for (int64_t i = 0; i < plen; ++i) {
          const double s = S(d + i);
          corr += s * (double)pre1[i];
          se += s * s;
        }
        ++fine_host;
        const double denom = std::sqrt(se * pre1_energy);
        metric = denom > 0.001 ? corr / denom : NAN;
      }
      if (metric > best) { best = metric; best_pos = d; } // NaN: skipped (denom <= 0.001)
    }
    if (best < 0.1) {
      if (fails) fails->push_back({st.block, st.pre_pos});
      st.state = IDLE;
      st.ac_init = false;
      return;
    }
    st.pre_pos = best_pos;
    const int32_t max_payload = st.meta_received ? (st.chunk_size ? st.chunk_size : 4096) + 11 : 280;
    if (max_payload != est_payload) { est_payload = max_payload; est_samples = amod_estimate_frame_samples(cfg, max_payload); }
    st.frame_end = st.pre_pos + est_samples;
    st.state = COLLECTING;
  }

  // _resetToIdle (app.js:974-981)
  void reset() {
    st.ac_pos = st.frame_end ? st.frame_end : st.pre_pos + cfg->symbol_len;
    st.ac_init = false;
    st.pre_pos = -1;
    st.frame_end = -1;
    st.state = IDLE;
  }
};

// one demodulated window of the trajectory and the receiver state right after it
// (_resetToIdle done, positioned at the next block)
struct FrameEv {
  int64_t pos, end;
  bool lost; // getRange() returned null: counted as a frame error, nothing decoded
  RxState after;
};
struct Traj {
  std::vector<FrameEv> frames;
  std::vector<std::pair<int64_t, int64_t>> fails;
  RxState end;
};

// two runs that demodulated the same window and stand in the same post-reset state
// continue identically (the next scan re-initialises its sums)
bool same_after(const RxState &a, const RxState &b) {
  return a.block == b.block && a.state == b.state && a.ac_init == b.ac_init && a.ac_pos == b.ac_pos &&
         a.pre_pos == b.pre_pos && a.frame_end == b.frame_end && a.meta_received == b.meta_received &&
         a.chunk_size == b.chunk_size && !a.ac_init;
}

// processAudioBlock (app.js:749-773) for blocks [st.block, stop): the state step of each
// block. first_only: return after the first demodulated window. sync: return at the
// first window that `sync` also demodulated from the same state (*sync_idx = its index).
void run_blocks(Receiver &rx, const RxState &start, int64_t stop, bool first_only, const Traj *sync, Traj &out,
                int64_t *sync_idx) {
  rx.st = start;
  rx.fails = &out.fails;
  rx.stop_block = stop;
  if (sync_idx) *sync_idx = -1;
  while (rx.st.block < stop) {
    if (rx.timed && rx.st.state != COLLECTING) { // diagnostics
      const auto t0 = std::chrono::steady_clock::now();
      const bool idle = rx.st.state == IDLE;
      if (idle) rx.scan(); else rx.refine();
      (idle ? rx.scan_ms : rx.refine_ms) += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      ++rx.st.block;
      continue;
    }
    switch (rx.st.state) {
    case IDLE: rx.scan(); break;
    case DETECTED: rx.refine(); break;
    case COLLECTING:
      if (rx.tw() >= rx.st.frame_end) { // _checkFrameComplete -> _demodulateFrame (app.js:900-972)
        FrameEv ev{rx.st.pre_pos, rx.st.frame_end, rx.st.pre_pos < rx.tw() - rx.cap, RxState{}};
        rx.reset();
        ev.after = rx.st;
        ev.after.block = rx.st.block + 1;
        out.frames.push_back(ev);
        if (sync) {
          auto it = std::lower_bound(sync->frames.begin(), sync->frames.end(), ev.pos,
                                     [](const FrameEv &f, int64_t p) { return f.pos < p; });
          for (; it != sync->frames.end() && it->pos == ev.pos; ++it)
            if (it->end == ev.end && same_after(it->after, ev.after)) {
              *sync_idx = it - sync->frames.begin();
              out.end = ev.after;
              return;
            }
        }
        if (first_only) {
          out.end = ev.after;
          return;
        }
      }
      break;
    }
    ++rx.st.block;
  }
  out.end = rx.st;
}

// The receiver from `start` to the last block on up to `nthreads` host threads. Segment k
// starts speculatively (IDLE, scan resuming at its first block, the same metadata state);
// the true run is carried across each boundary until it demodulates a window that the
// speculative segment demodulated from the identical post-reset state, and adopts the
// segment's trajectory from there (or covers the whole segment itself).
Traj run_parallel(const Receiver &proto, const RxState &start, int64_t nblocks, int nthreads, int64_t &fine_host,
                  const amod::Knobs &kn) {
  const auto t_par0 = std::chrono::steady_clock::now();
  const int64_t span = nblocks - start.block;
  const int64_t minseg = kn.stream_minseg > 0 ? kn.stream_minseg : 64; // (tests force short segments)
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, span / minseg));
  std::vector<int64_t> bnd(T + 1);
  for (int k = 0; k <= T; ++k) bnd[k] = start.block + span * k / T;
  std::vector<Traj> seg(T);
  std::vector<Receiver> rxs(T, proto);
  const bool diag = kn.stream_diag;
  for (auto &r : rxs) r.timed = diag;
  std::vector<double> th_ms(T, 0.0);
  std::vector<std::thread> th;
  for (int k = 0; k < T; ++k) {
    th.emplace_back([&, k] {
      RxState st = start;
      if (k > 0) {
        st = RxState{};
        st.block = bnd[k];
        st.state = IDLE;
        st.ac_pos = bnd[k] * kBlock - 511; // where a continuous scan stands at this block
        st.meta_received = start.meta_received;
        st.chunk_size = start.chunk_size;
      }
      const auto t0 = std::chrono::steady_clock::now();
      run_blocks(rxs[k], st, bnd[k + 1], false, nullptr, seg[k], nullptr);
      th_ms[k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
  }
  for (auto &t : th) t.join();
  const auto t_threads = std::chrono::steady_clock::now();
  Traj total = std::move(seg[0]);
  Receiver rx = proto;
  for (int k = 1; k < T; ++k) {
    Traj cont;
    int64_t j = -1;
    run_blocks(rx, total.end, bnd[k + 1], false, &seg[k], cont, &j);
    total.frames.insert(total.frames.end(), cont.frames.begin(), cont.frames.end());
    total.fails.insert(total.fails.end(), cont.fails.begin(), cont.fails.end());
    if (j >= 0) {
      const int64_t after_block = seg[k].frames[j].after.block;
      total.frames.insert(total.frames.end(), seg[k].frames.begin() + j + 1, seg[k].frames.end());
      for (auto &f : seg[k].fails)
        if (f.first >= after_block) total.fails.push_back(f);
      total.end = seg[k].end;
    } else {
      total.end = cont.end;
    }
  }
  fine_host += rx.fine_host;
  for (auto &r : rxs) fine_host += r.fine_host;
  if (diag) {
    int64_t sc = rx.scanned;
    double wmax = 0;
    for (auto &r : rxs) { sc += r.scanned; wmax = std::max(wmax, r.wait_ms); }
    fprintf(stderr, "[stream] run_parallel: %d segments, threads %.3f ms (max wait %.3f ms), merge %.3f ms (wait %.3f), "
            "scanned %lld positions, frames %zu\n", T,
            std::chrono::duration<double, std::milli>(t_threads - t_par0).count(), wmax,
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_threads).count(), rx.wait_ms,
            (long long)sc, total.frames.size());
    for (int k = 0; k < T; ++k)
      fprintf(stderr, "[stream]   thread %d: %.3f ms (scan %.3f, refine %.3f), scanned %lld, frames %zu, gpu gaps %lld, "
              "gpu refinements %lld\n", k, th_ms[k], rxs[k].scan_ms, rxs[k].refine_ms, (long long)rxs[k].scanned,
              seg[k].frames.size(), (long long)rxs[k].gap_hits, (long long)rxs[k].ref_hits);
  }
  return total;
}

struct Pinned {
  float *p = nullptr; // (any element type: as<T>())
  size_t cap = 0;
  ~Pinned() { if (p) (void)hipHostFree(p); }
  void *dp = nullptr; // device view (mapped allocations)
  hipError_t alloc(size_t n, bool mapped = false) { // grow-only
    n = std::max<size_t>(n, 16);
    if (p && cap >= n) return hipSuccess;
    if (p) { (void)hipHostFree(p); p = nullptr; dp = nullptr; cap = 0; }
    hipError_t e = hipHostMalloc((void **)&p, n, mapped ? hipHostMallocMapped : hipHostMallocDefault);
    if (e == hipSuccess && mapped) e = hipHostGetDevicePointer(&dp, p, 0);
    if (e == hipSuccess) cap = n;
    return e;
  }
  template <typename T> T *as() const { return (T *)p; }
};

// Pageable host buffer (address space only until written: MAP_NORESERVE). The host copy of
// the cleaned stream is touched sparsely (its first piece, the granules the state machine
// reads); pinning all of it (hipHostMalloc of 3.6 GB for a 32k-chunk stream) cost ~150 ms
// per first call of a size, more than the whole GPU prepass.
struct PageBuf {
  float *p = nullptr;
  size_t cap = 0;
  ~PageBuf() { if (p) munmap(p, cap); }
  hipError_t alloc(size_t n) { // grow-only
    n = std::max<size_t>(n, 16);
    if (p && cap >= n) return hipSuccess;
    if (p) { munmap(p, cap); p = nullptr; cap = 0; }
    void *q = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (q == MAP_FAILED) return hipErrorOutOfMemory;
    p = (float *)q;
    cap = n;
    return hipSuccess;
  }
  template <typename T> T *as() const { return (T *)p; }
};

// device and pinned buffers of the streaming receiver, kept per context (grow-only)
struct StreamCache {
  DBuf d_x, d_y, d_warm, d_end, d_scr, d_list, d_apow, d_fixed, d_hot, d_ze;
  DBuf d_pre1, d_first, d_base, d_count, d_out, d_metric, d_rwg;
  // window decoder: three buffer sets (one batch decoding, one dispatched by the host, one
  // whose chunk bytes the copy pool is still moving into the assembler)
  static constexpr int kSets = 3;
  DBuf w_pos[kSets], w_len[kSets], w_woff[kSets], w_win[kSets], w_out[kSets]; // w_out: results, then payload rows
  hipEvent_t w_done[kSets] = {}, w_kern[kSets] = {};
  hipStream_t s3 = nullptr; // window decoder: results and payload rows to the host, beside the next batch's kernels
  DBuf d_c, d_gsrc;                         // sparse copy: packed granules, their stream granules
  DBuf d_barg, d_gaps;                      // k_fine's per-workgroup argmax, k_gap_scan's records
  Pinned gaps_h;
  PageBuf yh;
  Pinned yc, hot_h, metric_h;
  Pinned gsrc_h; // the sparse gather's granule list (pinned: its upload does not block the host)
  Pinned w_out_h[kSets];                    // window decoder: w_out's host mirror (one pinned D2H)
  // the sparse copy's per-granule tables (kept: no page faults or address-space locks per call)
  std::vector<uint8_t> sp_need;
  std::vector<std::pair<int64_t, int64_t>> sp_reg; // (kept: its pages stay faulted in across calls)
  std::vector<int32_t> sp_cidx;
  std::vector<amod::GapScan> gaps_keep; // the gap scans' records and refinements (kept: a fresh 3 MB
  std::vector<GpuRefine> refs_keep;     // vector per call spent ~1 ms in first-touch faults)
  std::unique_ptr<std::atomic<const float *>[]> sp_gptr;
  size_t sp_gcap = 0;
  bool apow_ready = false;
  hipStream_t s2 = nullptr;                 // the cleaned stream's device-to-host copy
  hipStream_t s_fetch = nullptr;            // sparse copy: granules fetched on demand
  Pinned fetch_h, mfetch_h;                 // their pinned bounce buffers (granules, a range's metrics)
  hipStream_t s_up = nullptr;               // host samples: the upload, in pieces
  std::vector<hipEvent_t> up_ev;            // one per uploaded piece (the EMA of a piece waits on it)
  static constexpr int kPieces = 16;
  hipEvent_t ema_done = nullptr, gathered = nullptr, piece[kPieces] = {}, cpiece[kPieces] = {};
  ~StreamCache() {
    if (s2) { (void)hipStreamSynchronize(s2); (void)hipStreamDestroy(s2); }
    if (s3) { (void)hipStreamSynchronize(s3); (void)hipStreamDestroy(s3); }
    if (s_fetch) { (void)hipStreamSynchronize(s_fetch); (void)hipStreamDestroy(s_fetch); }
    if (s_up) { (void)hipStreamSynchronize(s_up); (void)hipStreamDestroy(s_up); }
    for (auto e : up_ev) (void)hipEventDestroy(e);
    for (auto e : w_kern)
      if (e) (void)hipEventDestroy(e);
    if (ema_done) (void)hipEventDestroy(ema_done);
    if (gathered) (void)hipEventDestroy(gathered);
    for (auto e : piece)
      if (e) (void)hipEventDestroy(e);
    for (auto e : cpiece)
      if (e) (void)hipEventDestroy(e);
    for (auto e : w_done)
      if (e) (void)hipEventDestroy(e);
  }
};
StreamCache &stream_cache(amod_ctx *ctx) {
  void **slot = amod_ctx_ext(ctx, 0, [](void *q) { delete static_cast<StreamCache *>(q); });
  if (!*slot) *slot = new StreamCache;
  return *static_cast<StreamCache *>(*slot);
}

// The GPU part before the state machine, over stream samples [lo, lo + n) given on the
// host (n a multiple of kBlock; lo a multiple of kEmaChunk): exact DC removal (EMA
// started at lo), screening, fine sums, pinned host copy of the cleaned samples.
struct Prepass {
  StreamCache *c = nullptr;
  const float *x = nullptr; // device samples of [lo, lo + nvalid)
  FineTable ft;
  int64_t lo = 0, n = 0, fixed = 0;
  bool dev_metrics = false; // k_fine also keeps its metrics on the device (k_gap_refine reads them)
  const amod::Knobs *kn = nullptr; // the context's knobs (read at amod_open)
  int64_t nmetric = 0;
  int64_t nhot = 0;            // 32-sample blocks screened (hot flags on the device)
  // the EMA state after local chunk k (its true end state, read from the device)
  double ema_end(amod_ctx *ctx, int64_t k) const {
    double v = NAN;
    if (k >= 0 && k < (n + kEmaChunk - 1) / kEmaChunk)
      (void)hipMemcpy(&v, c->d_end.as<double>() + k, sizeof(double), hipMemcpyDeviceToHost);
    (void)ctx;
    return v;
  }
  double t_ema = 0, t_fine = 0;
  const float *y() const { return c->d_y.as<float>(); }
  std::function<void(int64_t)> wait_fn = [this](int64_t g) { wait_y(g); };
  // sparse: only the first piece of the cleaned stream is copied to the host at once (the
  // metadata phase reads the stream's start); the state machine's parallel phase then gets
  // just the granules it reads (sparse_setup), and a read past the first piece before that
  // starts the full copy
  bool sparse = false;
  mutable bool full_started = false;
  mutable std::mutex mu;
  hipStream_t s_main = nullptr;
  // piece q of the host copy is local samples [pstart(q), pstart(q + 1)); the first ends at
  // p0_end (sparse: just the metadata phase's reads, so the DMA engine is soon free again)
  int64_t p0_end = 0;
  int64_t pstart(int q) const {
    return q == 0 ? 0 : q == 1 ? p0_end : q >= StreamCache::kPieces ? n : n * q / StreamCache::kPieces;
  }
  // the host copy of the cleaned stream holds local samples [0, g)
  void wait_y(int64_t g) const {
    if (g > p0_end) start_full();
    for (int q = 0; q < StreamCache::kPieces; ++q) {
      const int64_t a = pstart(q);
      if (a >= g) break;
      (void)hipEventSynchronize(c->piece[q]);
    }
  }
  // pieces [q0, kPieces) of the full copy (q0 = 1: the rest after the first)
  hipError_t enqueue_pieces(int q0) const {
    for (int q = q0; q < StreamCache::kPieces; ++q) {
      const int64_t a = pstart(q), b = pstart(q + 1);
      if (b > a) {
        const hipError_t e = hipMemcpyAsync(c->yh.p + a, c->d_y.as<float>() + a, sizeof(float) * (size_t)(b - a),
                                            hipMemcpyDeviceToHost, c->s2);
        if (e != hipSuccess) return e;
      }
      const hipError_t e = hipEventRecord(c->piece[q], c->s2);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  void start_full() const {
    std::lock_guard<std::mutex> lk(mu);
    if (full_started) return;
    (void)enqueue_pieces(1);
    full_started = true;
  }

  // ---- sparse copy of the cleaned stream (the parallel phase's reads)
  int64_t ng = 0, first_g = 0; // granules; those inside the first piece
  int32_t *cidx = nullptr;     // granule -> packed index (-1: not packed)
  std::atomic<const float *> *gptr = nullptr; // granule -> host pointer once there
  std::unique_ptr<std::atomic<bool>[]> cready; // packed piece q has landed
  std::atomic<bool> first_ready{false};
  mutable std::atomic<int64_t> fallbacks{0};
  std::atomic<int64_t> wait_us{0}, fetch_us{0}; // diagnostics: piece waits, on-demand fetches
  int64_t npacked = 0;
  std::function<const float *(int64_t)> present_fn = [this](int64_t g) { return present(g); };
  std::function<const float *(int64_t)> copied_fn = [this](int64_t g) -> const float * {
    return g < first_g || cidx[g] >= 0 ? present(g) : nullptr;
  };
  // granule g on the host: the first piece, the packed copy, or fetched now (16 granules)
  const float *present(int64_t g) {
    const float *p;
    if (g < first_g) {
      if (!first_ready.load(std::memory_order_acquire)) {
        (void)hipEventSynchronize(c->piece[0]);
        first_ready.store(true, std::memory_order_release);
      }
      p = c->yh.as<float>() + g * kGran;
    } else if (cidx[g] >= 0) {
      const int q = (int)(cidx[g] * (int64_t)StreamCache::kPieces / std::max<int64_t>(npacked, 1));
      if (!cready[q].load(std::memory_order_acquire)) {
        const auto t0 = std::chrono::steady_clock::now();
        (void)hipEventSynchronize(c->cpiece[q]);
        cready[q].store(true, std::memory_order_release);
        wait_us += std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
      }
      p = c->yc.as<float>() + (int64_t)cidx[g] * kGran;
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      std::lock_guard<std::mutex> lk(mu);
      if ((p = gptr[g].load(std::memory_order_acquire))) return p;
      const int64_t g1 = std::min(ng, g + 16);
      // on a non-blocking stream of its own, after the EMA: a plain hipMemcpy went on the
      // null stream and waited for every decode batch queued on the context's stream
      // (281 granules fetched this way took 7-9 ms of the host phase, AMOD_STREAM_DIAG)
      // (and into pinned memory: a device-to-pageable copy went through HIP's staging path
      // and still took ≈ 0.5 ms per 64 KB under the running decode)
      if (!c->s_fetch) (void)hipStreamCreateWithFlags(&c->s_fetch, hipStreamNonBlocking);
      const size_t nb = sizeof(float) * (size_t)((g1 - g) * kGran);
      if (c->fetch_h.alloc(sizeof(float) * 16 * kGran) == hipSuccess) {
        (void)hipStreamWaitEvent(c->s_fetch, c->ema_done, 0);
        (void)hipMemcpyAsync(c->fetch_h.p, c->d_y.as<float>() + g * kGran, nb, hipMemcpyDeviceToHost, c->s_fetch);
        (void)hipStreamSynchronize(c->s_fetch);
        std::memcpy(c->yh.as<float>() + g * kGran, c->fetch_h.p, nb);
      } else {
        (void)hipMemcpy(c->yh.as<float>() + g * kGran, c->d_y.as<float>() + g * kGran, nb, hipMemcpyDeviceToHost);
      }
      fetch_us += std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
      if (kn->stream_diag && fallbacks.load() < 400) fprintf(stderr, "[stream] fetch granule %lld\n", (long long)g);
      fallbacks += g1 - g;
      for (int64_t k = g + 1; k < g1; ++k)
        if (!gptr[k].load(std::memory_order_acquire) && cidx[k] < 0)
          gptr[k].store(c->yh.as<float>() + k * kGran, std::memory_order_release);
      p = c->yh.as<float>() + g * kGran;
    }
    gptr[g].store(p, std::memory_order_release);
    return p;
  }
  // Marks the granules the state machine reads from `start` on (the scan from each frame's
  // end through the next hot region and its block, the refine windows, the start of every
  // speculative segment), packs them on the GPU and copies them to the host in pieces.
  // Reads outside them still work (present() fetches). Returns false when the full copy
  // is (or was) used instead.
  // ---- speculative gap scans on the GPU (k_gap_scan): one per fine range, from where the
  // receiver would stand after the frame detected there (window length F)
  int nbx = 0, nfr = 0;
  std::vector<amod::GapScan> gaps;
  std::vector<GpuRefine> refs; // k_gap_refine's refinements, by pre_pos
  bool gap_launched = false;
  int gap_scan_launch(const amod_cfg *cfg, const RxState &start, int64_t nblocks, int64_t cap) {
    gaps.clear();
    gap_launched = false;
    if (nfr <= 0 || kn->no_gap_scan) return AMOD_SUCCESS;
    const int32_t maxp = start.meta_received ? (start.chunk_size ? start.chunk_size : 4096) + 11 : 280;
    const int64_t F = amod_estimate_frame_samples(cfg, maxp);
    if (c->d_gaps.alloc(sizeof(amod::GapScan) * (size_t)nfr) != hipSuccess ||
        c->gaps_h.alloc(sizeof(amod::GapScan) * (size_t)nfr) != hipSuccess ||
        amod_launch_gap_scan(c->d_y.as<float>(), n, lo, c->d_first.as<int64_t>(), c->d_barg.as<double2>(), nbx, nfr,
                             F, cap, nblocks, kGapBlocks, c->d_gaps.as<amod::GapScan>(), s_main) != hipSuccess ||
        (dev_metrics && nmetric > 0 &&
         amod_launch_gap_refine(c->d_gaps.as<amod::GapScan>(), nfr, lo, c->d_first.as<int64_t>(), c->d_base.as<int64_t>(),
                                c->d_count.as<int64_t>(), nfr, c->d_metric.as<double>(), 3 * (int64_t)cfg->cp_len,
                                s_main) != hipSuccess) ||
        hipMemcpyAsync(c->gaps_h.p, c->d_gaps.p, sizeof(amod::GapScan) * (size_t)nfr, hipMemcpyDeviceToHost,
                       s_main) != hipSuccess)
      return AMOD_ERR_HIP;
    gap_launched = true;
    return AMOD_SUCCESS;
  }
  int gap_scan_finish() {
    if (!gap_launched) return AMOD_SUCCESS;
    if (gaps.capacity() < c->gaps_keep.capacity()) { gaps.swap(c->gaps_keep); gaps.clear(); }
    if (refs.capacity() < c->refs_keep.capacity()) { refs.swap(c->refs_keep); refs.clear(); }
    gaps.reserve((size_t)nfr);
    refs.reserve((size_t)nfr);
    if (hipStreamSynchronize(s_main) != hipSuccess) return AMOD_ERR_HIP;
    const amod::GapScan *g = c->gaps_h.as<amod::GapScan>();
    refs.clear();
    for (int r = 0; r < nfr; ++r) {
      if (g[r].status != 1) continue;
      gaps.push_back(g[r]);
      if (dev_metrics && g[r].ref_ok) refs.push_back({g[r].pre_pos, g[r].ref_pos, g[r].ref_best});
    }
    // (records come in fine-range order, which is stream order: usually sorted already)
    auto by_s0 = [](const amod::GapScan &a, const amod::GapScan &b) { return a.s0 < b.s0; };
    auto by_pre = [](const GpuRefine &a, const GpuRefine &b) { return a.pre_pos < b.pre_pos; };
    if (!std::is_sorted(gaps.begin(), gaps.end(), by_s0)) std::sort(gaps.begin(), gaps.end(), by_s0);
    if (!std::is_sorted(refs.begin(), refs.end(), by_pre)) std::sort(refs.begin(), refs.end(), by_pre);
    return AMOD_SUCCESS;
  }
  ~Prepass() { // the record vectors' pages go back to the context's cache
    if (c && gaps.capacity() > c->gaps_keep.capacity()) c->gaps_keep.swap(gaps);
    if (c && refs.capacity() > c->refs_keep.capacity()) c->refs_keep.swap(refs);
  }

  double setup_ms[4] = {}; // diagnostics: marks, index, pointer table, gather + copies
  bool sparse_setup(const amod_cfg *cfg, const RxState &start, int64_t nblocks, int nthreads) {
    if (!sparse || full_started) return false;
    auto tick = [t = std::chrono::steady_clock::now()](double &acc) mutable {
      const auto now = std::chrono::steady_clock::now();
      acc = std::chrono::duration<double, std::milli>(now - t).count();
      t = now;
    };
    ng = n >> kGranLog;
    first_g = p0_end >> kGranLog;
    std::vector<uint8_t> &need = c->sp_need;
    need.assign((size_t)ng, 0);
    double tm_assign = 0, tm_reg = 0;
    tick(tm_assign);
    // need[g]: 1 = read by the state machine, 2 = read first (a speculative segment's or the
    // true run's first scan: packed at the front, so each thread waits for one piece only)
    uint8_t mark_val = 1;
    auto mark = [&](int64_t a, int64_t b) { // local samples [a, b)
      a = std::max<int64_t>(a, first_g * kGran);
      b = std::min<int64_t>(b, n);
      for (int64_t g = a >> kGranLog; a < b && g <= (b - 1) >> kGranLog; ++g)
        need[(size_t)g] = std::max(need[(size_t)g], mark_val);
    };
    // hot regions (local), blocks less than 2 K samples apart merged
    // (a fresh 512 KB vector here took 2.4 ms of first-touch faults on the 32k-chunk stream
    // while the runtime's copy threads fault in the host mirror)
    std::vector<std::pair<int64_t, int64_t>> &reg = c->sp_reg;
    reg.clear();
    reg.reserve(ft.first.size());
    if (gap_launched) { // (the fine ranges: hot blocks +- 448 samples, merged)
      for (size_t r = 0; r < ft.first.size(); ++r) reg.push_back({ft.first[r] - lo + 448, ft.first[r] - lo + ft.count[r] - 448});
    } else {
      if (c->hot_h.alloc((size_t)std::max<int64_t>(nhot, 1)) != hipSuccess ||
          (nhot && hipMemcpy(c->hot_h.p, c->d_hot.p, (size_t)nhot, hipMemcpyDeviceToHost) != hipSuccess)) {
        start_full();
        return false;
      }
      const uint8_t *hot = c->hot_h.as<uint8_t>();
      for (int64_t b = 0; b < n / 32; ++b) {
        if (!hot[b]) continue;
        if (!reg.empty() && 32 * b <= reg.back().second + 2048) reg.back().second = 32 * b + 32;
        else reg.push_back({32 * b, 32 * b + 32});
      }
    }
    tick(tm_reg);
    const int32_t maxp = start.meta_received ? (start.chunk_size ? start.chunk_size : 4096) + 11 : 280;
    const int64_t F = amod_estimate_frame_samples(cfg, maxp);
    const int64_t R = 3 * (int64_t)cfg->cp_len + cfg->symbol_len + 64; // refine radius + correlation
    const int64_t W = 2048;                                             // the metric's drop after the plateau
    // the scan from local position p to the detection in the first hot region after it,
    // and through that region (the detection, its 0.7 drop and refinement read there: with
    // the GPU gap scans nothing else marks it, and every speculative segment's first scan
    // fetched its region on demand, AMOD_STREAM_DIAG)
    auto scan_from = [&](int64_t p) {
      auto it = std::lower_bound(reg.begin(), reg.end(), std::make_pair(p, (int64_t)0));
      mark(p - 1024, it == reg.end() ? p + F + W : it->second + R + W);
    };
    for (size_t k = 0; k < reg.size(); ++k) {
      if (gap_launched) { // the scans come from the GPU: the refinement window only (and with
        if (!dev_metrics) mark(reg[k].first - R, reg[k].second + R); // k_gap_refine, not even that)
        continue;
      }
      mark(reg[k].first - R - 1024, reg[k].second + R + W);
      scan_from(reg[k].first - R + F); // the scan after the frame detected in region k
    }
    mark_val = 2;
    scan_from(start.ac_pos - lo);
    const int64_t span = nblocks - start.block; // run_parallel's speculative segments
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, span / 64));
    for (int k = 1; k < T; ++k) scan_from((start.block + span * k / T) * kBlock - 511 - lo - 1024);
    tick(setup_ms[0]);
    if (kn->stream_diag)
      fprintf(stderr, "[stream] marks: assign %.3f ms, regions %.3f ms (%zu), marks %.3f ms\n", tm_assign, tm_reg,
              reg.size(), setup_ms[0]);
    setup_ms[0] += tm_assign + tm_reg;
    std::vector<int32_t> src;
    c->sp_cidx.assign((size_t)ng, -1);
    cidx = c->sp_cidx.data();
    for (const uint8_t pass : {uint8_t(2), uint8_t(1)}) // the first scans' granules first
      for (int64_t g = first_g; g < ng; ++g)
        if (need[(size_t)g] == pass) { cidx[(size_t)g] = (int32_t)src.size(); src.push_back((int32_t)g); }
    if (2 * (int64_t)src.size() > ng - first_g) { start_full(); return false; } // not worth it
    npacked = (int64_t)src.size();
    tick(setup_ms[1]);
    if (c->sp_gcap < (size_t)ng) { c->sp_gptr.reset(new std::atomic<const float *>[(size_t)ng]); c->sp_gcap = (size_t)ng; }
    gptr = c->sp_gptr.get();
    for (int64_t g = 0; g < ng; ++g) gptr[g].store(nullptr, std::memory_order_relaxed);
    tick(setup_ms[2]);
    cready.reset(new std::atomic<bool>[StreamCache::kPieces]);
    for (int q = 0; q < StreamCache::kPieces; ++q) cready[q].store(npacked == 0, std::memory_order_relaxed);
    if (npacked) {
      if (c->d_c.alloc(sizeof(float) * (size_t)npacked * kGran) || c->d_gsrc.alloc(sizeof(int32_t) * src.size()) ||
          c->yc.alloc(sizeof(float) * (size_t)npacked * kGran)) { start_full(); return false; }
      if (!c->gathered) (void)hipEventCreateWithFlags(&c->gathered, hipEventDisableTiming);
      for (auto &e : c->cpiece)
        if (!e) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
      // the granule list goes up from pinned memory and the gather runs on s2 (which waited
      // for the EMA): a pageable copy on the launch stream held the host until the gap scans
      // queued there had run, and the gap scans' wait then also waited for the gather
      bool ok = c->gsrc_h.alloc(sizeof(int32_t) * src.size()) == hipSuccess;
      if (ok) std::memcpy(c->gsrc_h.p, src.data(), sizeof(int32_t) * src.size());
      ok = ok && hipMemcpyAsync(c->d_gsrc.p, c->gsrc_h.p, sizeof(int32_t) * src.size(), hipMemcpyHostToDevice, c->s2) == hipSuccess &&
           amod_launch_gather(c->d_y.as<float>(), c->d_gsrc.as<int32_t>(), (int)npacked, c->d_c.as<float>(), c->s2) == hipSuccess &&
           hipEventRecord(c->gathered, c->s2) == hipSuccess;
      for (int q = 0; ok && q < StreamCache::kPieces; ++q) {
        const int64_t a = npacked * q / StreamCache::kPieces, b = npacked * (q + 1) / StreamCache::kPieces;
        if (b > a)
          ok = hipMemcpyAsync(c->yc.as<float>() + a * kGran, c->d_c.as<float>() + a * kGran,
                              sizeof(float) * (size_t)((b - a) * kGran), hipMemcpyDeviceToHost, c->s2) == hipSuccess;
        ok = ok && hipEventRecord(c->cpiece[q], c->s2) == hipSuccess;
      }
      if (!ok) { (void)hipStreamSynchronize(c->s2); start_full(); return false; }
    }
    tick(setup_ms[3]);
    return true;
  }

  // samples: host memory, or device memory when `device` (read for [0, nvalid); the
  // padding up to n is zeros, as the reference's last block)
  int run(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t nvalid, int64_t lo_, int64_t n_,
          hipStream_t s, bool device = false) {
    c = &stream_cache(ctx);
    lo = lo_; n = n_;
    const int64_t nchunks = std::max<int64_t>(1, (n + kEmaChunk - 1) / kEmaChunk);
    if (!device) S_TRY(c->d_x.alloc(sizeof(float) * (size_t)n + 64));
    S_TRY(c->d_y.alloc(sizeof(float) * (size_t)n + 64));
    S_TRY(c->d_warm.alloc(sizeof(double) * nchunks));
    S_TRY(c->d_end.alloc(sizeof(double) * nchunks));
    S_TRY(c->d_scr.alloc(sizeof(double) * nchunks));
    S_TRY(c->d_list.alloc((sizeof(int64_t) + 1) * nchunks + 64)); // list, then one flag byte per chunk
    S_TRY(c->d_apow.alloc(sizeof(double) * kEmaChunk));
    S_TRY(c->d_fixed.alloc(16));
    if (!c->apow_ready) {
      std::vector<double> ap((size_t)kEmaChunk);
      double a = 1.0;
      for (auto &v : ap) { v = a; a *= 0.999; }
      S_TRY(hipMemcpy(c->d_apow.p, ap.data(), sizeof(double) * ap.size(), hipMemcpyHostToDevice));
      c->apow_ready = true;
    }
    S_TRY(c->d_hot.alloc((size_t)(n / 32 + 1)));
    S_TRY(c->d_ze.alloc(sizeof(double2) * (size_t)(n / 32 + 1)));
    hipEvent_t ev[3];
    for (auto &e : ev) S_TRY(hipEventCreate(&e));
    S_TRY(hipEventRecord(ev[0], s));
    float *const yd = c->d_y.as<float>();
    double *const wd_ = c->d_warm.as<double>(), *const ed = c->d_end.as<double>(), *const sd = c->d_scr.as<double>();
    if (device) {
      x = samples;
      S_TRY(amod_launch_ema_part(x, nvalid, n, yd, wd_, ed, sd, c->d_apow.as<double>(), 0, n, s, kn));
    } else {
      // the host samples go up in pieces on the upload stream (HIP's pageable copy runs at
      // ~51 GB/s in 64 MB pieces, ~14 GB/s as one multi-GB copy), and each piece's EMA
      // waves run on s as soon as it has landed (they read only it and the pieces before)
      x = c->d_x.as<float>();
      const int64_t wsz = amod_ema_wave_samples(kn);
      const int64_t P = std::max<int64_t>(1, kUpPieceSamples / wsz) * wsz;
      const int64_t npc = (n + P - 1) / P;
      if (!c->s_up) S_TRY(hipStreamCreateWithFlags(&c->s_up, hipStreamNonBlocking));
      while ((int64_t)c->up_ev.size() < npc + 1) {
        hipEvent_t e;
        S_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->up_ev.push_back(e);
      }
      S_TRY(hipEventRecord(c->up_ev[npc], s)); // (the previous call's reads of d_x are done)
      S_TRY(hipStreamWaitEvent(c->s_up, c->up_ev[npc], 0));
      for (int64_t q = 0; q < npc; ++q) {
        const int64_t a = q * P, b = std::min(n, a + P);
        const int64_t va = std::min(a, nvalid), vb = std::min(b, nvalid);
        if (vb > va)
          S_TRY(hipMemcpyAsync(c->d_x.as<float>() + va, samples + va, sizeof(float) * (size_t)(vb - va),
                               hipMemcpyHostToDevice, c->s_up));
        S_TRY(hipEventRecord(c->up_ev[q], c->s_up));
        S_TRY(hipStreamWaitEvent(s, c->up_ev[q], 0));
        S_TRY(amod_launch_ema_part(x, nvalid, n, yd, wd_, ed, sd, c->d_apow.as<double>(), a, b, s, kn));
      }
    }
    S_TRY(amod_launch_ema_fix(x, nvalid, n, yd, wd_, ed, c->d_list.as<int64_t>(), c->d_fixed.as<unsigned long long>(), s, kn));
    S_TRY(hipEventRecord(ev[1], s));
    S_TRY(amod_launch_sc_screen(c->d_y.as<float>(), n, 0.25f, c->d_ze.as<double2>(), c->d_hot.as<uint8_t>(), s));
    // the fine ranges (every position within 448 samples of a hot block), built on the GPU
    nhot = n / 32;
    const int64_t max_ranges = nhot / (1 + 29) + 2; // starts are more than 29 blocks apart
    S_TRY(c->d_rwg.alloc(sizeof(int32_t) * (size_t)(nhot / 256 + 4)));
    S_TRY(c->d_first.alloc(sizeof(int64_t) * (size_t)max_ranges));
    S_TRY(c->d_count.alloc(sizeof(int64_t) * (size_t)max_ranges));
    S_TRY(amod_launch_ranges(c->d_hot.as<uint8_t>(), nhot, c->d_rwg.as<int32_t>(), c->d_first.as<int64_t>(),
                             c->d_count.as<int64_t>(), s));
    int32_t nr_dev = 0;
    S_TRY(hipMemcpyAsync(&nr_dev, c->d_rwg.as<int32_t>() + (nhot > 0 ? (nhot + 255) / 256 : 0), sizeof(int32_t),
                         hipMemcpyDeviceToHost, s));
    unsigned long long fx = 0;
    S_TRY(hipMemcpyAsync(&fx, c->d_fixed.p, 8, hipMemcpyDeviceToHost, s));
    // the cleaned stream to the host (pinned) on a second stream, in pieces, under the
    // screening / fine-sum work and the receiver's first segments
    S_TRY(c->yh.alloc(sizeof(float) * (size_t)std::max<int64_t>(n, 1)));
    if (!c->s2) {
      S_TRY(hipStreamCreateWithFlags(&c->s2, hipStreamNonBlocking));
      S_TRY(hipEventCreateWithFlags(&c->ema_done, hipEventDisableTiming));
      for (auto &e : c->piece) S_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    S_TRY(hipEventRecord(c->ema_done, s));
    S_TRY(hipStreamWaitEvent(c->s2, c->ema_done, 0));
    s_main = s;
    full_started = false;
    p0_end = sparse ? std::min<int64_t>(n / StreamCache::kPieces, kFirstPiece) : n / StreamCache::kPieces;
    if (sparse) { // the first piece now, the rest on demand (sparse_setup / start_full)
      const int64_t b = p0_end;
      if (b > 0)
        S_TRY(hipMemcpyAsync(c->yh.p, c->d_y.as<float>(), sizeof(float) * (size_t)b, hipMemcpyDeviceToHost, c->s2));
      S_TRY(hipEventRecord(c->piece[0], c->s2));
    } else {
      S_TRY(enqueue_pieces(0));
      full_started = true;
    }
    const auto tq0 = std::chrono::steady_clock::now();
    S_TRY(hipStreamSynchronize(s));
    const auto tq1 = std::chrono::steady_clock::now();
    fixed = (int64_t)fx;
    const int nr = nr_dev;
    std::vector<int64_t> first_loc((size_t)nr);
    ft.first.resize((size_t)nr); ft.count.resize((size_t)nr); ft.base.resize((size_t)nr);
    if (nr) {
      S_TRY(hipMemcpyAsync(first_loc.data(), c->d_first.p, sizeof(int64_t) * nr, hipMemcpyDeviceToHost, s));
      S_TRY(hipMemcpyAsync(ft.count.data(), c->d_count.p, sizeof(int64_t) * nr, hipMemcpyDeviceToHost, s));
      S_TRY(hipStreamSynchronize(s));
    }
    int64_t total = 0;
    for (int r = 0; r < nr; ++r) { ft.first[(size_t)r] = lo + first_loc[(size_t)r]; ft.base[(size_t)r] = total; total += ft.count[(size_t)r]; }
    // without the GPU refinements k_fine writes its metrics straight into mapped host memory
    // for the host's lookups (no copy queued behind the cleaned stream's transfer); with them
    // they stay on the device, and the few refinements left to the host correlate there
    ft.metric = nullptr;
    ft.dmetric = nullptr;
    ft.fetched.clear();
    if (!dev_metrics) {
      S_TRY(c->metric_h.alloc(sizeof(double) * (size_t)std::max<int64_t>(total, 1), true));
      ft.metric = c->metric_h.as<double>();
    }
    if (total) {
      std::vector<float> p1(cfg->symbol_len);
      if (amod_preamble1(cfg, p1.data()) != AMOD_SUCCESS) return amod_ctx_fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
      double p1e = 0.0; // this.pre1Energy (app.js:744-745)
      for (float v : p1) p1e += (double)v * (double)v;
      nmetric = total;
      if (dev_metrics) {
        S_TRY(c->d_metric.alloc(sizeof(double) * (size_t)total));
        ft.dmetric = c->d_metric.as<double>();
        if (!c->s_fetch) S_TRY(hipStreamCreateWithFlags(&c->s_fetch, hipStreamNonBlocking));
        ft.fetch_stream = c->s_fetch; // (the metrics are read after this prepass's final sync)
      }
      std::vector<double> p1d(p1.begin(), p1.end()); // (exact: k_fine's fma operand)
      S_TRY(c->d_pre1.alloc(sizeof(double) * p1.size()));
      S_TRY(c->d_base.alloc(sizeof(int64_t) * nr));
      S_TRY(hipMemcpyAsync(c->d_pre1.p, p1d.data(), sizeof(double) * p1d.size(), hipMemcpyHostToDevice, s));
      S_TRY(hipMemcpyAsync(c->d_base.p, ft.base.data(), sizeof(int64_t) * nr, hipMemcpyHostToDevice, s));
      const int64_t maxc = *std::max_element(ft.count.begin(), ft.count.end());
      ft.fetch_bounce = nullptr;
      if (dev_metrics && c->mfetch_h.alloc(sizeof(double) * (size_t)maxc) == hipSuccess)
        ft.fetch_bounce = c->mfetch_h.as<double>(); // (fetches hold FineTable's lock: one at a time)
      nbx = (int)((maxc + amod::kFinePositions - 1) / amod::kFinePositions);
      nfr = nr;
      S_TRY(c->d_barg.alloc(sizeof(double2) * (size_t)nr * nbx));
      for (int r0 = 0; r0 < nr; r0 += 65535) {
        const int k = std::min(65535, nr - r0);
        S_TRY(amod_launch_fine(c->d_y.as<float>(), n, c->d_pre1.as<double>(), cfg->symbol_len, p1e,
                               c->d_first.as<int64_t>() + r0, c->d_base.as<int64_t>() + r0,
                               c->d_count.as<int64_t>() + r0, k, maxc, dev_metrics ? nullptr : (double *)c->metric_h.dp,
                               dev_metrics ? c->d_metric.as<double>() : nullptr,
                               c->d_barg.as<double2>() + (int64_t)r0 * nbx, s));
      }
    }
    const auto tq2 = std::chrono::steady_clock::now();
    S_TRY(hipEventRecord(ev[2], s));
    S_TRY(hipStreamSynchronize(s));
    if (kn->stream_diag)
      fprintf(stderr, "[stream] prepass: wait for EMA+screen %.3f ms, fine ranges + launch %.3f ms (%zu ranges, %lld "
              "positions, longest %lld), k_fine wait %.3f ms\n",
              std::chrono::duration<double, std::milli>(tq1 - tq0).count(),
              std::chrono::duration<double, std::milli>(tq2 - tq1).count(), ft.first.size(), (long long)total,
              (long long)(ft.count.empty() ? 0 : *std::max_element(ft.count.begin(), ft.count.end())),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq2).count());
    float ta = 0, tb = 0;
    S_TRY(hipEventElapsedTime(&ta, ev[0], ev[1]));
    S_TRY(hipEventElapsedTime(&tb, ev[1], ev[2]));
    t_ema = ta; t_fine = tb;
    for (auto &e : ev) (void)hipEventDestroy(e);
    return AMOD_SUCCESS;
  }

  Receiver receiver(const amod_cfg *cfg) const {
    Receiver rx;
    rx.cfg = cfg;
    rx.lo = lo; rx.nloc = n; rx.y = c->yh.p; rx.fine = &ft;
    rx.wait_y = &wait_fn;
    rx.avail = 0;
    rx.piece_end = [this](int64_t g) { // end of the piece holding local sample g
      for (int q = 0; q < StreamCache::kPieces; ++q)
        if (g < pstart(q + 1)) return pstart(q + 1);
      return n;
    };
    rx.cap = (int64_t)amod_estimate_frame_samples(cfg, 4096 + 16) * 3 + 8192; // RingBuffer capacity (app.js:711-714)
    rx.pre1.resize(cfg->symbol_len);
    amod_preamble1(cfg, rx.pre1.data());
    for (float v : rx.pre1) rx.pre1_energy += (double)v * (double)v;
    return rx;
  }
};

// Decodes frames' windows on the GPU (k_window peak normalisation + chunk-mode decode);
// res[i] / payload row i for frame i (lost frames get AMOD_E_STREAM_LOST).
struct WindowDecoder {
  std::vector<amod_result> res; // frame i - a of the last collected batch
  std::vector<int> slot;         // its row in the pinned payload (-1: lost)
  const uint8_t *ph = nullptr;   // pinned payload rows
  std::vector<uint8_t> zero_row;
  int64_t stride = 16;
  double t_ms = 0, t_launch = 0; // host time in launch + collect (t_launch: launch alone)
  bool diag = false;      // (AMOD_STREAM_DIAG: slow launch steps reported as they happen)
  int d2h_mode = 1;       // (AMOD_STREAM_D2H)
  double t_sub[8] = {}; // (diagnostics) launch: host prep, device buffers + input copies, memset, k_window, reserve, decode, event + wait, D2H enqueue
  // a batch in flight in buffer set k
  struct Flight {
    std::vector<int64_t> pos, woff; // (host arrays kept until the batch is collected)
    std::vector<int32_t> len;
    std::vector<int> slot;
    int64_t stride = 16;
    size_t rb = 0; // the results' bytes ahead of the rows in w_out
    int nw = 0;
    size_t a = 0, b = 0;
    bool live = false;
  } fl[StreamCache::kSets];
  // payload row of frame i - a of the last collected batch (zeros for a lost window)
  const uint8_t *row(size_t k) const { return slot[k] < 0 ? zero_row.data() : ph + (size_t)stride * slot[k]; }

  // enqueues frames [a, b)'s windows (k_window peak normalisation) and their decode on s
  int launch(amod_ctx *ctx, const amod_cfg *cfg, const Prepass &pp, const std::vector<FrameEv> &fr, size_t a,
             size_t b, hipStream_t s, int k) {
    const auto t0 = std::chrono::steady_clock::now();
    Flight &f = fl[k];
    f.pos.clear(); f.woff.clear(); f.len.clear();
    f.slot.assign(b - a, -1);
    f.a = a; f.b = b;
    int64_t tot = 0, maxlen = 0;
    for (size_t i = a; i < b; ++i) {
      if (fr[i].lost) continue;
      f.slot[i - a] = (int)f.pos.size();
      const int64_t L = fr[i].end - fr[i].pos;
      f.pos.push_back(fr[i].pos - pp.lo); f.len.push_back((int32_t)L); f.woff.push_back(tot);
      tot += (L + 3) & ~int64_t(3);
      maxlen = std::max(maxlen, L);
    }
    const int nw = f.nw = (int)f.pos.size();
    f.stride = amod_payload_stride(cfg, std::max<int64_t>(maxlen, 1));
    StreamCache &c = *pp.c;
    DBuf &d_pos = c.w_pos[k], &d_len = c.w_len[k], &d_woff = c.w_woff[k], &d_win = c.w_win[k], &d_out = c.w_out[k];
    // results and rows in one buffer, so they come back in one copy (a separate 400 KB
    // results copy held the host ~7 ms on the host-sample path: HIP ran it as a blocking copy)
    const size_t rb = f.rb = (sizeof(amod_result) * (size_t)std::max(nw, 1) + 255) & ~size_t(255);
    const size_t ob = rb + (size_t)f.stride * std::max(nw, 1);
    S_TRY(c.w_out_h[k].alloc(ob, d2h_mode == 2));
    if (!c.w_done[k]) S_TRY(hipEventCreateWithFlags(&c.w_done[k], hipEventDisableTiming));
    if (!c.w_kern[k]) S_TRY(hipEventCreateWithFlags(&c.w_kern[k], hipEventDisableTiming));
    if (!c.s3) S_TRY(hipStreamCreateWithFlags(&c.s3, hipStreamNonBlocking));
    auto lap = [t = t0](double &acc) mutable {
      const auto now = std::chrono::steady_clock::now();
      acc += std::chrono::duration<double, std::milli>(now - t).count();
      t = now;
    };
    lap(t_sub[0]);
    if (nw) {
      S_TRY(d_pos.alloc(sizeof(int64_t) * nw));
      S_TRY(d_len.alloc(sizeof(int32_t) * nw));
      S_TRY(d_woff.alloc(sizeof(int64_t) * nw));
      S_TRY(d_win.alloc(sizeof(float) * (size_t)tot + 64));
      S_TRY(d_out.alloc(ob));
      amod_result *const d_res = reinterpret_cast<amod_result *>(d_out.p);
      uint8_t *const d_pay = reinterpret_cast<uint8_t *>(d_out.p) + rb;
      S_TRY(hipMemcpyAsync(d_pos.p, f.pos.data(), sizeof(int64_t) * nw, hipMemcpyHostToDevice, s));
      S_TRY(hipMemcpyAsync(d_len.p, f.len.data(), sizeof(int32_t) * nw, hipMemcpyHostToDevice, s));
      S_TRY(hipMemcpyAsync(d_woff.p, f.woff.data(), sizeof(int64_t) * nw, hipMemcpyHostToDevice, s));
      lap(t_sub[1]);
      S_TRY(hipMemsetAsync(d_pay, 0, (size_t)f.stride * nw, s));
      lap(t_sub[2]);
      S_TRY(amod_launch_window(pp.y(), pp.n, d_pos.as<int64_t>(), d_len.as<int32_t>(),
                               d_woff.as<int64_t>(), nw, d_win.as<float>(), s));
      lap(t_sub[3]);
      int rc = amod_reserve(ctx, cfg, nw, maxlen);
      if (rc) return rc;
      lap(t_sub[4]);
      rc = amod_decode_device(ctx, cfg, AMOD_MODE_CHUNK, d_win.as<float>(), d_woff.as<int64_t>(), d_len.as<int32_t>(),
                              nw, d_res, d_pay, f.stride, 0, s);
      if (rc) return rc;
      lap(t_sub[5]);
      // the rows go to the host on the launch stream, behind the batch's kernels (round 5,
      // interleaved on one box: host samples 1.01 -> 1.07e10, device-resident 4.54 -> 4.8e10
      // samples/s against the copy stream s3, which an earlier layout needed so the next
      // batch's kernels did not queue behind 9 MB of rows; AMOD_STREAM_D2H=0 keeps that)
      hipStream_t s_out = d2h_mode == 1 ? s : c.s3;
      if (s_out != s) {
        S_TRY(hipEventRecord(c.w_kern[k], s));
        S_TRY(hipStreamWaitEvent(c.s3, c.w_kern[k], 0));
      }
      lap(t_sub[6]);
      const double d7 = t_sub[7];
      int busy = 0; // (diagnostics: which streams still have work queued as the copies go in)
      if (diag) {
        const hipStream_t qs[5] = {s, c.s2, c.s3, c.s_up, amod_ctx_stream(ctx)};
        for (int i = 0; i < 5; ++i) busy |= (qs[i] && hipStreamQuery(qs[i]) == hipErrorNotReady) << i;
      }
      const auto tq0 = std::chrono::steady_clock::now();
      if (d2h_mode == 2 && c.w_out_h[k].dp)
        S_TRY(hipMemcpyAsync(c.w_out_h[k].dp, d_out.p, rb + (size_t)f.stride * nw, hipMemcpyDeviceToDevice, s_out));
      else
        S_TRY(hipMemcpyAsync(c.w_out_h[k].p, d_out.p, rb + (size_t)f.stride * nw, hipMemcpyDeviceToHost, s_out));
      const auto tq1 = std::chrono::steady_clock::now();
      S_TRY(hipEventRecord(c.w_done[k], s_out));
      lap(t_sub[7]);
      if (diag && t_sub[7] - d7 > 0.5)
        fprintf(stderr, "[stream]   slow D2H enqueue: set %d, %d windows, busy streams 0x%x (s, s2, s3, s_up, ctx), rows %zu B: copy %.3f ms, event %.3f ms\n", k, nw, busy,
                (size_t)f.stride * nw, std::chrono::duration<double, std::milli>(tq1 - tq0).count(),
                t_sub[7] - d7 - std::chrono::duration<double, std::milli>(tq1 - tq0).count());
    } else {
      S_TRY(hipEventRecord(c.w_done[k], s));
    }
    f.live = true;
    const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    t_ms += dt;
    t_launch += dt;
    return AMOD_SUCCESS;
  }
  // waits for batch k; res / row() then describe it
  int collect(amod_ctx *ctx, const Prepass &pp, int k) {
    const auto t0 = std::chrono::steady_clock::now();
    Flight &f = fl[k];
    StreamCache &c = *pp.c;
    S_TRY(hipEventSynchronize(c.w_done[k]));
    f.live = false;
    const amod_result *rh = c.w_out_h[k].as<amod_result>();
    ph = reinterpret_cast<const uint8_t *>(c.w_out_h[k].p) + f.rb;
    stride = f.stride;
    if (zero_row.size() != (size_t)stride) zero_row.assign((size_t)stride, 0);
    slot = f.slot;
    res.resize(f.b - f.a);
    for (size_t i = 0; i < res.size(); ++i) {
      amod_result &o = res[i];
      if (slot[i] < 0) {
        o = amod_result{};
        o.status = AMOD_E_STREAM_LOST; o.preamble_idx = -1; o.coarse_idx = -1; o.frame_type = -1;
      } else {
        o = rh[slot[i]];
      }
    }
    t_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return AMOD_SUCCESS;
  }
  // a batch launched but not collected (dropped: a metadata frame changed what follows) is
  // waited for, so its buffers can be reused
  int drain(amod_ctx *ctx, const Prepass &pp) {
    for (int k = 0; k < StreamCache::kSets; ++k)
      if (fl[k].live) { S_TRY(hipEventSynchronize(pp.c->w_done[k])); fl[k].live = false; }
    return AMOD_SUCCESS;
  }
  int run(amod_ctx *ctx, const amod_cfg *cfg, const Prepass &pp, const std::vector<FrameEv> &fr, size_t a, size_t b,
          hipStream_t s) {
    const int rc = launch(ctx, cfg, pp, fr, a, b, s, 0);
    return rc ? rc : collect(ctx, pp, 0);
  }
};

// What a decoded metadata result does to the receiver's window length
// (_demodulateFrame -> handleMetadataFrame, app.js:926-940): chunkSize is assigned even
// when the bitmap allocation throws (totalChunks <= -8), metaReceived only without it.
void apply_meta(const amod_result &r, RxState &after) {
  if (r.status != AMOD_OK || r.frame_type != 0xFE || !r.crc_valid) return;
  after.chunk_size = r.chunk_size;
  if (r.total_chunks > -8) after.meta_received = true;
}

int receiver_threads(const amod::Knobs &kn) { // (AMOD_STREAM_THREADS=1 in tests: the plain sequential receiver)
  return kn.stream_threads > 0 ? kn.stream_threads
                               : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

void to_state(const RxState &a, amod_stream_state &o) {
  o.block = a.block; o.ac_pos = a.ac_pos; o.pre_pos = a.pre_pos; o.frame_end = a.frame_end;
  o.ac_p = a.ac_p; o.ac_ra = a.ac_ra; o.ac_rb = a.ac_rb;
  o.state = a.state; o.ac_init = a.ac_init; o.meta_received = a.meta_received; o.chunk_size = a.chunk_size;
}
RxState from_state(const amod_stream_state &o) {
  RxState a;
  a.block = o.block; a.ac_pos = o.ac_pos; a.pre_pos = o.pre_pos; a.frame_end = o.frame_end;
  a.ac_p = o.ac_p; a.ac_ra = o.ac_ra; a.ac_rb = o.ac_rb;
  a.state = o.state; a.ac_init = o.ac_init != 0; a.meta_received = o.meta_received != 0; a.chunk_size = o.chunk_size;
  return a;
}

} // namespace

// processAudioBlock's DC removal (app.js:751-755) over a device buffer, from a zero EMA
// state at x[0]: y = cleaned samples (device), *end_state = the state after x[n - 1]
extern "C" int amod_dc_remove_device(amod_ctx *ctx, const float *x, int64_t n, float *y, double *end_state,
                                     int64_t *chunks_fixed, void *stream) {
  if (!ctx || n < 0 || (n && (!x || !y))) return amod_ctx_fail(ctx, "invalid argument", AMOD_ERR_ARG);
  if (n == 0) { if (end_state) *end_state = 0.0; if (chunks_fixed) *chunks_fixed = 0; return AMOD_SUCCESS; }
  S_TRY(hipSetDevice(amod_ctx_device(ctx)));
  hipStream_t s = stream ? (hipStream_t)stream : amod_ctx_stream(ctx);
  const int64_t nch = (n + kEmaChunk - 1) / kEmaChunk;
  DBuf warm, end, scr, list, apow, fixed;
  S_TRY(warm.alloc(sizeof(double) * nch));
  S_TRY(end.alloc(sizeof(double) * nch));
  S_TRY(scr.alloc(sizeof(double) * nch));
  S_TRY(list.alloc((sizeof(int64_t) + 1) * nch + 64)); // list, then one flag byte per chunk
  S_TRY(apow.alloc(sizeof(double) * kEmaChunk));
  S_TRY(fixed.alloc(16));
  std::vector<double> ap((size_t)kEmaChunk);
  double a = 1.0;
  for (auto &v : ap) { v = a; a *= 0.999; }
  S_TRY(hipMemcpyAsync(apow.p, ap.data(), sizeof(double) * ap.size(), hipMemcpyHostToDevice, s));
  S_TRY(amod_launch_ema(x, n, n, y, warm.as<double>(), end.as<double>(), scr.as<double>(), list.as<int64_t>(),
                        apow.as<double>(), fixed.as<unsigned long long>(), s, amod_ctx_knobs(ctx)));
  double e = 0.0;
  unsigned long long fx = 0;
  S_TRY(hipMemcpyAsync(&e, end.as<double>() + nch - 1, sizeof(double), hipMemcpyDeviceToHost, s));
  S_TRY(hipMemcpyAsync(&fx, fixed.p, sizeof fx, hipMemcpyDeviceToHost, s));
  S_TRY(hipStreamSynchronize(s));
  if (end_state) *end_state = e;
  if (chunks_fixed) *chunks_fixed = (int64_t)fx;
  return AMOD_SUCCESS;
}

static int stream_receive(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t n, bool device,
                          amod_assembler *assembler, amod_stream_frame *frames, int64_t max_frames,
                          int64_t *nframes_out, int64_t *refine_fail, int64_t max_refine_fail,
                          amod_stream_stats *stats) {
  using clk = std::chrono::steady_clock;
  const auto t_start = clk::now();
  if (!ctx || !cfg || n < 0 || (n && !samples) || (max_frames > 0 && !frames) || !nframes_out)
    return amod_ctx_fail(ctx, "invalid argument", AMOD_ERR_ARG);
  if (!amod_cfg_valid(cfg)) return amod_ctx_fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  S_TRY(hipSetDevice(amod_ctx_device(ctx)));
  hipStream_t s = amod_ctx_stream(ctx);
  const int64_t nblocks = (n + kBlock - 1) / kBlock, npad = nblocks * kBlock;
  amod_stream_stats stt{};
  Prepass pp;
  const amod::Knobs &kn = *amod_ctx_knobs(ctx);
  pp.kn = &kn;
  pp.sparse = !kn.stream_fullcopy; // (diagnostics: the whole cleaned stream to the host)
  pp.dev_metrics = !kn.no_gap_scan; // refinements of the gap scans' detections on the GPU
  {
    const int rc = pp.run(ctx, cfg, samples, n, 0, npad, s, device);
    if (rc) return rc;
  }
  stt.ema_chunks_fixed = pp.fixed;
  stt.t_ema_ms = pp.t_ema;
  stt.t_fine_ms = pp.t_fine;
  const auto t_gpu_pre = clk::now();

  // ---- host: the receiver
  amod_assembler *own = nullptr;
  if (!assembler) {
    if (amod_asm_open(nullptr, &own) != AMOD_SUCCESS) return amod_ctx_fail(ctx, "assembler", AMOD_ERR_NOMEM);
    assembler = own;
  }
  struct Guard { amod_assembler *a; ~Guard() { if (a) amod_asm_close(a); } } guard{own};
  Receiver proto = pp.receiver(cfg);
  const int nthreads = receiver_threads(kn);
  bool sparse_done = false;
  int64_t nfr = 0, frames_decoded = 0, frame_errors = 0, fine_host = 0;
  std::vector<int64_t> fails_out;
  WindowDecoder wd;
  wd.diag = kn.stream_diag;
  wd.d2h_mode = kn.stream_d2h;
  CopyPool copies(std::max(0, std::min(8, nthreads) - 1));
  double t_loop = 0, t_copy = 0; // (diagnostics: the dispatch's per-frame loop and its copies)

  // decode frames[a, b) and dispatch them in order (_demodulateFrame, app.js:907-972);
  // `changed`: the first frame whose metadata result changed the window length of what
  // follows (its `after` updated), or -1
  auto dispatch_body = [&](std::vector<FrameEv> &fr, size_t a, size_t b, int64_t &changed) -> int {
    changed = -1;
    // batch j + 1 decodes (buffer set (j + 1) % 3) while the host dispatches batch j and the
    // copy pool moves batch j - 1's chunks
    if (a < b) {
      const int rc = wd.launch(ctx, cfg, pp, fr, a, std::min(b, a + (size_t)kBatch), s, 0);
      if (rc) return rc;
    }
    for (size_t c0 = a, j = 0; c0 < b; c0 += kBatch, ++j) {
      const size_t c1 = std::min(b, c0 + (size_t)kBatch);
      if (c1 < b) {
        const int rc = wd.launch(ctx, cfg, pp, fr, c1, std::min(b, c1 + (size_t)kBatch), s, (int)((j + 1) % 3));
        if (rc) return rc;
      }
      const int rc = wd.collect(ctx, pp, (int)(j % 3));
      if (rc) return rc;
      const auto tl0 = clk::now();
      for (size_t i = c0; i < c1; ++i) {
        FrameEv &ev = fr[i];
        const amod_result &r = wd.res[i - c0];
        if (nfr < max_frames) {
          amod_stream_frame &f = frames[nfr];
          f.pos = ev.pos; f.end = ev.end; f.window_len = ev.lost ? 0 : (int32_t)(ev.end - ev.pos); f.reserved = 0;
          f.result = r;
        }
        ++nfr;
        if (r.status != AMOD_OK) { ++frame_errors; continue; }
        ++frames_decoded;
        const uint8_t *sl = wd.row(i - c0);
        if (r.frame_type == 0xFE) {
          if (!r.crc_valid) { ++frame_errors; continue; }
          copies.run(); // (the chunks before it land before the store is reset)
          const int m = amod_asm_metadata(assembler, r.total_chunks, r.total_size, r.chunk_size, sl + r.name_off,
                                          r.name_len);
          if (m == AMOD_ASM_RANGE_ERROR) ++frame_errors; // caught by the receiver; metaReceived unchanged
          RxState upd = ev.after;
          apply_meta(r, upd);
          const bool chg = upd.meta_received != ev.after.meta_received ||
                           (upd.meta_received && upd.chunk_size != ev.after.chunk_size);
          ev.after = upd;
          if (chg) { changed = (int64_t)i; copies.wait(); return wd.drain(ctx, pp); }
        } else if (r.frame_type == 0xFF) {
          uint8_t *dst = nullptr;
          const int c = amod_asm_chunk_at(assembler, r.seq_num, sl + r.data_off, r.data_len, r.crc_valid, &dst);
          if (c < 0) return amod_ctx_fail(ctx, "assembler store", c);
          if (dst && r.data_len > 0) copies.items.push_back({dst, sl + r.data_off, (size_t)r.data_len});
        }
      }
      const auto tl1 = clk::now();
      copies.start(); // (batch j - 1's copies done first: its buffer set is the next launch's)
      const auto tl2 = clk::now();
      t_loop += std::chrono::duration<double, std::milli>(tl1 - tl0).count();
      t_copy += std::chrono::duration<double, std::milli>(tl2 - tl1).count();
    }
    copies.run();
    return AMOD_SUCCESS;
  };
  // every exit of a failed dispatch first lands the queued chunk copies (their bitmap bits
  // are set) and drains the batches in flight (their D2H copies write the pinned rows the
  // next call may reallocate)
  auto decode_dispatch = [&](std::vector<FrameEv> &fr, size_t a, size_t b, int64_t &changed) -> int {
    const int rc = dispatch_body(fr, a, b, changed);
    if (rc != AMOD_SUCCESS) {
      copies.run();
      (void)wd.drain(ctx, pp);
    }
    return rc;
  };

  RxState st{};
  {
    amod_asm_info inf;
    amod_asm_state(assembler, &inf);
    st.chunk_size = inf.chunk_size; // this.assembler.chunkSize as the receiver starts
  }
  RxState final_state = st;
  for (;;) {
    Traj tr;
    if (!st.meta_received) {
      // before the metadata frame each window decides the next one's length: one at a time
      Receiver rx = proto;
      run_blocks(rx, st, nblocks, true, nullptr, tr, nullptr);
      fine_host += rx.fine_host;
    } else {
      if (!sparse_done) { // from here on the state machine reads only where frames start
        sparse_done = true;
        // the GPU's gap scans run while the host sets up the sparse copy
        const auto tg0 = clk::now();
        int grc = pp.gap_scan_launch(cfg, st, nblocks, proto.cap);
        if (grc) return amod_ctx_fail(ctx, "gap scan", grc);
        const bool sp_ok = pp.sparse_setup(cfg, st, nblocks, nthreads);
        const auto tg1 = clk::now();
        grc = pp.gap_scan_finish();
        if (grc) return amod_ctx_fail(ctx, "gap scan", grc);
        if (!pp.gaps.empty()) proto.gaps = &pp.gaps;
        if (!pp.refs.empty()) proto.refs = &pp.refs;
        if (kn.stream_diag) {
          int64_t smax = 0, ssum = 0;
          for (auto &g : pp.gaps) { smax = std::max(smax, g.scanned); ssum += g.scanned; }
          fprintf(stderr, "[stream] sparse setup %.3f ms (marks %.3f, index %.3f, pointers %.3f, copies %.3f), then gap scan: "
                  "%zu records (%lld positions, longest %lld), +%.3f ms\n",
                  std::chrono::duration<double, std::milli>(tg1 - tg0).count(), pp.setup_ms[0], pp.setup_ms[1],
                  pp.setup_ms[2], pp.setup_ms[3], pp.gaps.size(), (long long)ssum,
                  (long long)smax, std::chrono::duration<double, std::milli>(clk::now() - tg1).count());
        }
        if (sp_ok) {
          proto.gptr = pp.gptr; proto.present = &pp.present_fn; proto.copied = &pp.copied_fn;
        }
      }
      tr = run_parallel(proto, st, nblocks, nthreads, fine_host, kn);
    }
    int64_t chg = -1;
    const auto t_dd = clk::now();
    const int rc = decode_dispatch(tr.frames, 0, tr.frames.size(), chg);
    if (rc) return rc;
    if (kn.stream_diag)
      fprintf(stderr, "[stream] decode_dispatch of %zu frames: %.3f ms (since prepass %.3f ms; window decoder %.3f ms (launches %.3f), "
              "per-frame loop %.3f ms, chunk copies %.3f ms so far)\n", tr.frames.size(),
              std::chrono::duration<double, std::milli>(clk::now() - t_dd).count(),
              std::chrono::duration<double, std::milli>(t_dd - t_gpu_pre).count(), wd.t_ms, wd.t_launch, t_loop, t_copy);
    if (kn.stream_diag)
      fprintf(stderr, "[stream]   launches: host prep %.3f ms, buffers + input copies %.3f, memset %.3f, k_window %.3f, "
              "reserve %.3f, decode %.3f, event %.3f, D2H enqueue %.3f\n", wd.t_sub[0], wd.t_sub[1], wd.t_sub[2], wd.t_sub[3],
              wd.t_sub[4], wd.t_sub[5], wd.t_sub[6], wd.t_sub[7]);
    if (chg >= 0) {
      // keep what happened up to that frame; re-run the rest with the new window length
      const RxState after = tr.frames[chg].after;
      for (auto &f : tr.fails)
        if (f.first < after.block) fails_out.push_back(f.second);
      st = after;
      continue;
    }
    for (auto &f : tr.fails) fails_out.push_back(f.second);
    if (!tr.frames.empty() && tr.end.block < nblocks) { // first_only stop: continue from there
      st = tr.end;
      continue;
    }
    final_state = tr.end;
    break;
  }
  for (size_t i = 0; i < fails_out.size() && (int64_t)i < max_refine_fail; ++i) refine_fail[i] = fails_out[i];
  *nframes_out = nfr;
  if (stats) {
    stt.nframes = nfr;
    stt.nrefine_fail = (int64_t)fails_out.size();
    stt.frames_decoded = frames_decoded;
    stt.frame_errors = frame_errors;
    stt.final_state = final_state.state;
    stt.final_scan_pos = final_state.ac_pos;
    stt.fine_host_positions = fine_host;
    if (kn.stream_diag)
      fprintf(stderr, "[stream] sparse copy: %lld of %lld granules packed, %lld fetched on demand (%.3f ms), piece waits "
              "%.3f ms, full copy %d; fine positions on the host %lld\n",
              (long long)pp.npacked, (long long)pp.ng, (long long)pp.fallbacks.load(), pp.fetch_us.load() * 1e-3,
              pp.wait_us.load() * 1e-3, (int)pp.full_started, (long long)fine_host);
    stt.t_decode_ms = wd.t_ms;
    stt.t_total_ms = std::chrono::duration<double, std::milli>(clk::now() - t_start).count();
    stt.t_host_ms = std::chrono::duration<double, std::milli>(clk::now() - t_gpu_pre).count() - wd.t_ms;
    *stats = stt;
  }
  return AMOD_SUCCESS;
}

extern "C" int amod_stream_receive(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t n,
                                   amod_assembler *assembler, amod_stream_frame *frames, int64_t max_frames,
                                   int64_t *nframes_out, int64_t *refine_fail, int64_t max_refine_fail,
                                   amod_stream_stats *stats) {
  return stream_receive(ctx, cfg, samples, n, false, assembler, frames, max_frames, nframes_out, refine_fail,
                        max_refine_fail, stats);
}
extern "C" int amod_stream_receive_device(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t n,
                                          amod_assembler *assembler, amod_stream_frame *frames, int64_t max_frames,
                                          int64_t *nframes_out, int64_t *refine_fail, int64_t max_refine_fail,
                                          amod_stream_stats *stats) {
  return stream_receive(ctx, cfg, samples, n, true, assembler, frames, max_frames, nframes_out, refine_fail,
                        max_refine_fail, stats);
}

extern "C" int amod_stream_shard(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t lo, int64_t hi,
                                 int64_t own_lo, int64_t own_hi, const amod_stream_state *start, int32_t meta_received,
                                 int32_t chunk_size, int32_t until_meta, amod_stream_event *events,
                                 int64_t max_events, int64_t *nevents, uint8_t *payload, int64_t stride, int64_t *fails,
                                 int64_t max_fails, int64_t *nfails, double *ema, amod_stream_state *end) {
  if (!ctx || !cfg || lo < 0 || hi < lo || own_lo < lo || own_lo > hi || lo % kEmaChunk || hi % kBlock ||
      own_lo % kBlock || (hi > lo && !samples) || !nevents || !nfails || (max_events > 0 && !events) ||
      (max_events > 0 && payload && stride <= 0))
    return amod_ctx_fail(ctx, "invalid shard arguments", AMOD_ERR_ARG);
  if (!amod_cfg_valid(cfg)) return amod_ctx_fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  S_TRY(hipSetDevice(amod_ctx_device(ctx)));
  hipStream_t s = amod_ctx_stream(ctx);
  Prepass pp;
  const amod::Knobs &kn = *amod_ctx_knobs(ctx);
  pp.kn = &kn;
  {
    const int rc = pp.run(ctx, cfg, samples, hi - lo, lo, hi - lo, s);
    if (rc) return rc;
  }
  if (ema) {
    auto state_after = [&](int64_t g) -> double { // EMA state after stream sample g (a chunk end)
      const int64_t k = (g + 1 - lo) / kEmaChunk - 1;
      return (g + 1 - lo) % kEmaChunk == 0 ? pp.ema_end(ctx, k) : NAN;
    };
    ema[0] = own_lo > lo ? state_after(own_lo - 1) : NAN;
    ema[1] = own_hi > lo ? state_after(own_hi - 1) : NAN;
  }
  RxState st;
  if (start) {
    st = from_state(*start);
  } else {
    st.block = own_lo / kBlock;
    st.state = IDLE;
    st.ac_pos = std::max<int64_t>(0, own_lo - 511); // where a continuous scan stands at this block
  }
  if (!start) { st.meta_received = meta_received != 0; st.chunk_size = chunk_size; }
  const int64_t stop = hi / kBlock;
  // a window whose decoded bytes do not fit the caller's rows is an error, never a cut row
  auto row_too_narrow = [&] {
    return amod_ctx_fail(ctx, "payload stride too small for a decoded window (pass the chunk size)", AMOD_ERR_ARG);
  };
  Traj tr;
  int64_t fine_host = 0;
  WindowDecoder wd;
  std::vector<amod_result> res;
  std::vector<uint8_t> pay;
  if (until_meta) {
    // one window at a time until a result makes the metadata state known
    for (;;) {
      Traj t1;
      Receiver rx = pp.receiver(cfg);
      run_blocks(rx, st, stop, true, nullptr, t1, nullptr);
      tr.fails.insert(tr.fails.end(), t1.fails.begin(), t1.fails.end());
      if (t1.frames.empty()) { tr.end = t1.end; break; }
      const int rc = wd.run(ctx, cfg, pp, t1.frames, 0, 1, s);
      if (rc) return rc;
      apply_meta(wd.res[0], t1.frames[0].after);
      tr.frames.push_back(t1.frames[0]);
      res.push_back(wd.res[0]);
      if (wd.res[0].payload_valid > stride) return row_too_narrow();
      pay.insert(pay.end(), wd.row(0), wd.row(0) + std::min<int64_t>(wd.stride, stride));
      if (wd.stride < stride) pay.insert(pay.end(), (size_t)(stride - wd.stride), 0);
      st = t1.frames[0].after;
      tr.end = st;
      if (st.meta_received || st.block >= stop) break;
    }
  } else {
    tr = run_parallel(pp.receiver(cfg), st, stop, receiver_threads(kn), fine_host, kn);
  }
  *nevents = 0;
  size_t first = 0;
  while (first < tr.frames.size() && tr.frames[first].pos < own_lo) ++first; // owned by the previous shard
  std::vector<FrameEv> fr(tr.frames.begin() + first, tr.frames.end());
  if (until_meta) {
    res.erase(res.begin(), res.begin() + first);
    pay.erase(pay.begin(), pay.begin() + (size_t)stride * first);
  } else {
    for (size_t c0 = 0; c0 < fr.size(); c0 += kBatch) {
      const size_t c1 = std::min(fr.size(), c0 + (size_t)kBatch);
      const int rc = wd.run(ctx, cfg, pp, fr, c0, c1, s);
      if (rc) return rc;
      res.insert(res.end(), wd.res.begin(), wd.res.end());
      for (size_t i = c0; i < c1; ++i) { // rows at the caller's stride
        const uint8_t *row = wd.row(i - c0);
        if (wd.res[i - c0].payload_valid > stride) return row_too_narrow();
        pay.insert(pay.end(), row, row + std::min<int64_t>(wd.stride, stride));
        if (wd.stride < stride) pay.insert(pay.end(), (size_t)(stride - wd.stride), 0);
      }
    }
  }
  for (size_t i = 0; i < fr.size(); ++i) {
    if ((int64_t)i >= max_events) break;
    amod_stream_event &e = events[i];
    std::memset(&e, 0, sizeof e);
    e.frame.pos = fr[i].pos; e.frame.end = fr[i].end;
    e.frame.window_len = fr[i].lost ? 0 : (int32_t)(fr[i].end - fr[i].pos);
    e.frame.result = res[i];
    to_state(fr[i].after, e.after);
    if (payload) std::memcpy(payload + (size_t)stride * i, pay.data() + (size_t)stride * i, (size_t)stride);
  }
  *nevents = (int64_t)fr.size();
  *nfails = (int64_t)tr.fails.size();
  for (size_t i = 0; i < tr.fails.size() && (int64_t)i < max_fails; ++i) {
    fails[2 * i] = tr.fails[i].first;
    fails[2 * i + 1] = tr.fails[i].second;
  }
  if (end) to_state(tr.end, *end);
  return AMOD_SUCCESS;
}

// ---------------------------------------------------------------- live receiver
// StreamingReceiver.processAudioBlock (app.js:749-773) one block at a time, as an
// AudioWorklet / ScriptProcessor callback drives it: EMA DC removal on the host (a
// block is a few thousand samples), the reference's RingBuffer, one state-machine
// step per call (the same Receiver code as the recorded-stream path), and a window
// that completes is peak-normalised and decoded on the GPU (decodeChunkFrame), then
// handed to the ChunkAssembler exactly as _demodulateFrame does (app.js:907-972).
struct amod_live {
  amod_ctx *ctx = nullptr;
  amod_cfg cfg{};
  amod_assembler *assembler = nullptr;
  bool own_assembler = false;
  std::vector<float> ring;
  int64_t tw = 0, block = 0;
  double dc_mean = 0.0;
  Receiver rx;
  std::vector<std::pair<int64_t, int64_t>> fails;
  std::vector<float> win;
  std::vector<uint8_t> pay;
  int64_t frames_decoded = 0, frame_errors = 0;
};

extern "C" int amod_live_open(amod_ctx *ctx, const amod_cfg *cfg, amod_assembler *assembler, amod_live **out) {
  if (!ctx || !cfg || !out) return amod_ctx_fail(ctx, "invalid argument", AMOD_ERR_ARG);
  if (!amod_cfg_valid(cfg)) return amod_ctx_fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  auto *lv = new amod_live;
  lv->ctx = ctx;
  lv->cfg = *cfg;
  if (!assembler) {
    if (amod_asm_open(nullptr, &lv->assembler) != AMOD_SUCCESS) { delete lv; return amod_ctx_fail(ctx, "assembler", AMOD_ERR_NOMEM); }
    lv->own_assembler = true;
  } else {
    lv->assembler = assembler;
  }
  Receiver &rx = lv->rx;
  rx.cfg = &lv->cfg;
  rx.cap = (int64_t)amod_estimate_frame_samples(cfg, 4096 + 16) * 3 + 8192; // RingBuffer (app.js:711-715)
  lv->ring.assign((size_t)rx.cap, 0.f);
  rx.ring = lv->ring.data();
  rx.tw_live = 0;
  rx.pre1.resize(cfg->symbol_len);
  if (amod_preamble1(cfg, rx.pre1.data()) != AMOD_SUCCESS) {
    if (lv->own_assembler) amod_asm_close(lv->assembler);
    delete lv;
    return amod_ctx_fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  }
  for (float v : rx.pre1) rx.pre1_energy += (double)v * (double)v;
  rx.fails = &lv->fails;
  amod_asm_info inf;
  amod_asm_state(lv->assembler, &inf);
  rx.st.chunk_size = inf.chunk_size;
  *out = lv;
  return AMOD_SUCCESS;
}

extern "C" int amod_live_process_block(amod_live *lv, const float *samples, int64_t n, amod_stream_frame *frame,
                                       int32_t *has_frame) {
  if (!lv || n < 0 || (n && !samples) || !frame || !has_frame) return amod_ctx_fail(lv ? lv->ctx : nullptr, "invalid argument", AMOD_ERR_ARG);
  *has_frame = 0;
  Receiver &rx = lv->rx;
  const int64_t cap = rx.cap;
  // DC removal (app.js:751-755) and ringBuffer.write (571-577)
  double m = lv->dc_mean;
  for (int64_t i = 0; i < n; ++i) {
    m = 0.999 * m + (1 - 0.999) * (double)samples[i];
    lv->ring[(size_t)(lv->tw % cap)] = (float)((double)samples[i] - m);
    ++lv->tw;
  }
  lv->dc_mean = m;
  rx.tw_live = lv->tw;
  rx.st.block = lv->block++;
  switch (rx.st.state) {
  case IDLE: rx.scan(); break;
  case DETECTED: rx.refine(); break;
  case COLLECTING:
    if (lv->tw >= rx.st.frame_end) { // _checkFrameComplete -> _demodulateFrame
      amod_stream_frame &f = *frame;
      std::memset(&f, 0, sizeof f);
      f.pos = rx.st.pre_pos;
      f.end = rx.st.frame_end;
      const int64_t len = rx.st.frame_end - rx.st.pre_pos;
      amod_result &r = f.result;
      if (rx.st.pre_pos < lv->tw - cap) { // getRange -> null: a frame error, nothing decoded
        r.status = AMOD_E_STREAM_LOST; r.preamble_idx = -1; r.coarse_idx = -1; r.frame_type = -1;
        f.window_len = 0;
        ++lv->frame_errors;
        rx.reset();
      } else {
        f.window_len = (int32_t)len;
        lv->win.resize((size_t)len);
        float mx = 0.f;
        for (int64_t i = 0; i < len; ++i) {
          const float v = (float)rx.S(rx.st.pre_pos + i);
          lv->win[(size_t)i] = v;
          mx = std::max(mx, std::fabs(v));
        }
        if ((double)mx > 1e-6) // per-window peak normalisation (app.js:918-925)
          for (auto &v : lv->win) v = (float)((double)v / (double)mx);
        const int64_t stride = amod_payload_stride(&lv->cfg, std::max<int64_t>(len, 1));
        lv->pay.assign((size_t)stride, 0);
        const int64_t off0 = 0;
        const int32_t len32 = (int32_t)len;
        const int rc = amod_decode_host(lv->ctx, &lv->cfg, AMOD_MODE_CHUNK, lv->win.data(), len, &off0, &len32, 1, &r,
                                        lv->pay.data(), stride, 0);
        if (rc) return rc;
        rx.reset();
        if (r.status != AMOD_OK) {
          ++lv->frame_errors;
        } else {
          ++lv->frames_decoded;
          const uint8_t *sl = lv->pay.data();
          if (r.frame_type == 0xFE) {
            if (!r.crc_valid) {
              ++lv->frame_errors;
            } else {
              const int mr = amod_asm_metadata(lv->assembler, r.total_chunks, r.total_size, r.chunk_size, sl + r.name_off,
                                               r.name_len);
              if (mr == AMOD_ASM_RANGE_ERROR) ++lv->frame_errors;
              apply_meta(r, rx.st);
            }
          } else if (r.frame_type == 0xFF) {
            const int c = amod_asm_chunk(lv->assembler, r.seq_num, sl + r.data_off, r.data_len, r.crc_valid);
            if (c < 0) return amod_ctx_fail(lv->ctx, "assembler store", c);
          }
        }
      }
      *has_frame = 1;
    }
    break;
  }
  return AMOD_SUCCESS;
}

extern "C" int amod_live_state(const amod_live *lv, amod_stream_state *state, amod_live_stats *stats) {
  if (!lv) return amod_ctx_fail(nullptr, "invalid argument", AMOD_ERR_ARG);
  if (state) { to_state(lv->rx.st, *state); state->block = lv->block; }
  if (stats) {
    stats->total_written = lv->tw;
    stats->frames_decoded = lv->frames_decoded;
    stats->frame_errors = lv->frame_errors;
    stats->refine_fails = (int64_t)lv->fails.size();
    stats->last_refine_fail = lv->fails.empty() ? -1 : lv->fails.back().second;
    stats->fine_host_positions = lv->rx.fine_host;
  }
  return AMOD_SUCCESS;
}

extern "C" int64_t amod_live_refine_fails(const amod_live *lv, int64_t *pos, int64_t max) {
  if (!lv) return -1;
  for (size_t i = 0; i < lv->fails.size() && (int64_t)i < max; ++i) pos[i] = lv->fails[i].second;
  return (int64_t)lv->fails.size();
}

extern "C" void amod_live_close(amod_live *lv) {
  if (!lv) return;
  if (lv->own_assembler) amod_asm_close(lv->assembler);
  delete lv;
}
