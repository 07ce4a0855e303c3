// amodem_internal.h — shared host/device definitions of the MI355X demodulator.
//
// Frame pipeline (per frame, mirrors modem.js decodeReceivedSignal 557-654 and
// decodeChunkFrame 770-803):
//   fast path      (k_decode_fast.hip) k_detect (one workgroup per frame, the frame
//                   streamed once from HBM) -> k_demod (persistent waves, one frame
//                   at a time per wave); fp32 arithmetic with guard bands on every
//                   discrete decision; a frame whose decision falls inside a guard band
//                   (or that exceeds the launch's capacities) is appended to the exact
//                   list.
//   k_decode_exact (k_decode_exact.hip) replays the reference arithmetic in IEEE
//                   double, operation for operation, for the listed frames.
// Both end in finish_frame() below: majority vote, MSB-first byte packing, frame
// parsing and CRC-32 — integer work, bit-exact by construction.
//   k_tx           (k_tx.hip) the transmitter (modulateOFDM + frame builders) in
//                   IEEE double, bit-exact, for synthetic input at HBM rate.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "amodem.h"

namespace amod {

constexpr int kFft = 512;
constexpr int kMaxBand = 256;  // sub_end < fft/2
constexpr int kCrcLanes = 256; // CRC chunks per frame pass (16 bytes each)
constexpr int kCrcChunk = 16;
constexpr int kCrcBlock = kCrcLanes * kCrcChunk; // 4096 bytes per pass
constexpr int kCrcMats = 512; // GF(2) shift matrices: up to 512 16-byte chunks (8 KB) in one wave pass
constexpr int kFinePositions = 512; // k_fine: fine-sum positions per workgroup (per k_gap_scan argmax record)
constexpr int kTlHead = 4;    // DevWork::tl: marks before the per-wave k_demod end stamps

// Device-resident tables, built once per configuration by the runtime.
struct DevTables {
  const float *pre1;       // [symbol_len] preamble 1 (f32, generatePreambleSymbol1)
  const float2 *tw1;       // [8][64] e^{-2πi l q/512}, pass-1 twiddles (row 0 unused)
  const float2 *tw2;       // [8][8]  e^{-2πi 8 l1 p1/512}, pass-2 twiddles
  const double2 *tw_exact; // [511] per-stage recurrence twiddles (fftIterative 34-44)
  const float *known;      // [nband] CE symbol values ±1 (generateChannelEstSymbol)
  const int16_t *band_di;  // [nband] data-subcarrier index, -1 for pilots
  const uint32_t *crc_s4;  // [4][256] slice-by-4 CRC tables
  const uint32_t *crc_m1;  // [32][4][256] shift-by-(16*q) zero-byte operators, q<32
  const uint32_t *crc_m2;  // [32][4][256] shift-by-(512*q) operators, q<32
  const uint32_t *crc_mb;  // [4][256] shift-by-4096 operator (pass to pass)
  const uint32_t *crc_mat; // [kCrcMats][32] shift-by-(16*q) zero-byte operators as GF(2) matrices (column i = image of bit i)
  const uint32_t *crc_pre; // [16] register k zero bytes before the message start that becomes ~0 there
                           // (the inverse k-byte shift of ~0): chunk 0 left-padded to 16 bytes
  const uint32_t *crc_unpad; // [16][32] inverse k-zero-byte operators (same layout as crc_mat)
  const double2 *points;   // [16] constellation points of cfg.mod (initConstellation)
  const double2 *tw_inv;   // [511] inverse-transform recurrence twiddles (fftIterative, ifft)
  const float *tmpl;       // [3][symbol_len] pre1, pre2, CE symbols (f32, before normalisation)
};

struct DevCfg {
  int32_t cp, sym, sub_start, sub_end, nband, npilots, ndata, bps, mod, rep;
  int32_t origin_idx;  // constellationDemap(0,0): decision for an all-zero spectrum
  int32_t mode;        // AMOD_MODE_*
  int32_t pilots[AMOD_MAX_PILOTS];
  double te;           // sum pre1^2 in reference order (f64)
  float te_f;
  int32_t fold;        // +-1: pre1[i + 256] = fold * pre1[i] (fast fine stage folds on it), 0: no fold
  float guard;         // fast-path guard scale (1 = default)
  int32_t stop_after;  // diagnostics only (AMOD_STOP_AFTER): fast kernel returns after this stage
  float tx_tmax;       // max |tmpl| (k_tx normalisation)
  DevTables t;
};

// k_tx: one frame per workgroup; every pointer device memory
struct DevTxWork {
  const uint8_t *pkt;     // packet bytes (legacy packet / metadata / data-chunk payload)
  const int64_t *pkt_off; // [nframes] byte offset of frame f's packet
  const int32_t *pkt_len; // [nframes]
  const int32_t *pre;     // [nframes] leading silence samples
  const int32_t *post;    // [nframes] trailing silence samples
  float *out;             // output samples
  const int64_t *out_off; // [nframes] first output sample of frame f
  int32_t nframes;
};

// k_detect / k_chunk_prep -> k_demod: one record per frame
enum { ROUTE_DEMOD = 0, ROUTE_DONE = 1, ROUTE_EXACT = 2, ROUTE_REPLAY = 3 };
struct DetRec {
  int32_t route;   // ROUTE_DEMOD: demodulate; ROUTE_DONE: result written; ROUTE_EXACT: listed;
                   // ROUTE_REPLAY: detection replayed by the exact kernel, for k_demod's list launch
  int32_t flags;   // 0; a replayed detection: AMOD_FLAG_REPLAY | the flags that listed it
  int32_t start;   // preambleIdx (fine timing); 0 in chunk mode
  int32_t M, T;    // whole data symbols (demodulateOFDM numSym); symbols demodulated (prefix)
  int32_t coarse;  // Schmidl-Cox index (in the plateau)
  float A, B;      // normalisation y = A x + B (preprocessSignal)
  float fbest;     // best fine metric
  int32_t sc_lo, sc_hi; // listed frames: positions that can hold detectPreamble's argmax
                        // (every other position's metric is proven lower), or -1
  float pad;
};
static_assert(sizeof(DetRec) == 48, "DetRec layout");

struct DevWork {
  const float *samples;
  const int64_t *off;
  const int32_t *len;
  int32_t nframes;
  int32_t f0, f1;     // k_detect / k_chunk_prep / k_demod: the launch's frames [f0, f1)
  amod_result *res;
  uint8_t *payload;
  int64_t stride;
  amod_debug *dbg;
  int32_t *fb_count; // exact-kernel work list
  int32_t *fb_list;
  int32_t *fb_flags;
  float *xs;          // exact kernel: per-slot normalised samples
  uint32_t *bits;     // exact kernel: per-slot bit arrays
  int64_t xs_stride;  // floats per slot
  int64_t bits_stride;// words per slot
  uint32_t options;
  unsigned long long *stamps; // diagnostics (AMOD_STAMPS=1): per-frame s_memtime marks, 32 per frame
  int32_t nb_cap;     // k_detect: Schmidl-Cox moment blocks per frame (dynamic LDS)
  int32_t fine_cap;   // k_detect: fine-search positions (dynamic LDS), >= 12 CP + 1
  int32_t mcap;       // data symbols a frame of fast_len samples can hold (k_demod stream LDS)
  int32_t stream_words; // k_demod: LDS words per wave (bit stream, then the voted stream)
  int32_t vote_off;   // k_demod: word offset of the voted stream
  int64_t fast_len;   // frames longer than this go to the exact kernel (AMOD_FLAG_BIG)
  DetRec *det;        // [nframes] detection records
  float *soft;        // exact kernel, AMOD_OPT_SOFT_COMBINE: per-slot soft bit values
  int64_t soft_stride;// floats per slot
  // detection replay: the exact kernel appends frames listed only for detection-stage
  // guards (COARSE / FINE / THRESH) to this list once its fp64 detection is done, with
  // their detection record, and leaves the demodulation to a k_demod launch over the list
  int32_t *rp_count;  // exact kernel: the list it fills (null: demodulate every frame itself)
  int32_t *rp_list;
  const int32_t *dm_count; // k_demod: frames dm_list[0 .. *dm_count) instead of [f0, f1)
  const int32_t *dm_list;
  // k_demod beside a running exact kernel: when *yield_count > 0 (detection listed
  // frames) only the first yield_blocks workgroups run, so every CU keeps room for the
  // exact kernel's waves (0: the whole grid)
  const int32_t *yield_count;
  int32_t yield_blocks;
  // The decode's counters are zeroed by its own launches, so neither the next decode nor
  // a graph replay needs a memset: list B's exact launch (the last) zeroes *fb_reset,
  // list A's count, and k_detect / k_chunk_prep (the first) zero fb_zero[0 .. 2], the
  // counts of list B and of the replay list and k_demod's claim counter, which only later
  // launches use (null: not this launch)
  int32_t *fb_reset;
  int32_t *fb_zero;
  // k_demod (main launch): with at least claim_min frames per wave, the frames past all but
  // the last claim_rounds static rounds are claimed one at a time from this counter (null:
  // every frame static)
  int32_t *claim;
  int32_t claim_rounds, claim_min;
  // profiled decodes only (amod_aux_overlap): device real-time marks, [0] the first listed
  // frame list A's replica took (atomic min over the few workgroups that take one; k_detect
  // / k_chunk_prep's workgroup 0 initialises it), [kTlHead + i] the end of k_demod's wave i
  // (a plain store per wave, 0 for a wave that took no frame: no contended atomics in the
  // timed launch); the host reduces them when it collects the stage times
  unsigned long long *tl;
};

// Diagnostic / experiment knobs, read from the environment once when a context opens
// (never per decode): a context's routing and grid shapes stay fixed for its lifetime.
struct Knobs {
  float guard_scale = 1.f;  // AMOD_GUARD_SCALE: fast-path guard bands (tests)
  int stop_after = 99;      // AMOD_STOP_AFTER: fast kernel stops after this stage (k_corr_scan)
  int demod_mcap = 0;       // AMOD_DEMOD_MCAP: cap k_demod's symbol capacity (0: none)
  bool stamps = false;      // AMOD_STAMPS: per-frame s_memtime marks
  int demod_bpc = 0;        // AMOD_DEMOD_BPC: k_demod workgroups per CU (0: occupancy)
  int chunks = 0;           // AMOD_CHUNKS: detect/demod chunks over two streams (0: 1)
  int xslots = 0;           // AMOD_XSLOTS: cap the exact grid (0: none)
  bool no_replay = false;   // AMOD_NO_REPLAY: listed frames demodulate in the replica too
  bool exact_serial = false;// AMOD_EXACT_SERIAL: list A after k_demod on the launch stream
  int64_t up_piece = 0;     // AMOD_UP_PIECE: amod_decode_host upload piece (samples; 0: 64 MB)
  int pipe_stagger = 0;     // AMOD_PIPE_STAGGER: a pipe decode starts once the other slot's
                            // k_detect is done (detections back to back, k_demod beside)
  int64_t mall_flush_mb = 0; // AMOD_MALL_FLUSH_MB: stream this many MB of a scratch buffer
                            // between k_detect and k_demod (experiments: Infinity Cache probe)
  bool demod_static = false;// AMOD_DEMOD_STATIC: k_demod takes every frame by the static stride
  int claim_rounds = 2;     // AMOD_CLAIM_ROUNDS: k_demod's claimed tail, in rounds of frames
  int claim_min = 4;        // AMOD_CLAIM_MIN: frames per wave below which k_demod stays static
  int aux_priority = 1;     // AMOD_AUX_PRIORITY: the second stream at the device's highest (1) or
                            // default (0) priority (experiments)
  // streaming receiver (stream.cpp)
  int stream_minseg = 0;    // AMOD_STREAM_MINSEG
  bool stream_diag = false; // AMOD_STREAM_DIAG
  int stream_d2h = 1;       // AMOD_STREAM_D2H: window rows back by 1 a D2H copy on the launch stream
                            // (default), 0 one on the copy stream s3, 2 a device copy into mapped pinned memory
  bool no_gap_scan = false; // AMOD_NO_GAP_SCAN
  int stream_threads = -1;  // AMOD_STREAM_THREADS (-1: unset)
  bool stream_fullcopy = false; // AMOD_STREAM_FULLCOPY
  // the EMA kernels' experiment shapes (k_stream.hip; < 0: the kernel defaults)
  int ema_per = -1;         // AMOD_EMA_PER: output chunks per k_ema_out lane
  int ema_warm = -1;        // AMOD_EMA_WARM: warm-up chunks per output chunk
  int ema_rounds = -1;      // AMOD_EMA_ROUNDS: parallel fix rounds before the serial safety net
};

// k_gap_scan -> streaming receiver: the scan that follows the frame of fine range r, run
// from its speculated start (s0, block b1) to its detection (status 1)
struct GapScan {
  int64_t s0, b1;              // start: ac_pos = s0 (sums not initialised), IDLE in block b1
  int64_t det_block, pre_pos;  // the block whose scan call detected, the coarse position
  int64_t ac_pos, scanned;     // the scan position after it; positions stepped
  double p, ra, rb;            // the running sums after it
  int32_t status, ref_ok;      // ref_ok: the refinement of pre_pos below is valid (k_gap_refine)
  double ref_best;             // _refineAndCollect over [pre_pos - 3 cp, pre_pos + 3 cp]: the first
  int64_t ref_pos;             // maximum (NaN skipped; -inf and pre_pos when none)
};

// AMOD_OPT_SOFT_COMBINE applies to repeated BPSK / QPSK frames
__host__ __device__ inline bool soft_combine_applies(uint32_t options, int rep, int mod) {
  return (options & AMOD_OPT_SOFT_COMBINE) && rep > 1 && (mod == AMOD_BPSK || mod == AMOD_QPSK);
}
// ... and k_demod's soft instance decides it (not a parity-debug launch; a repeat group
// spans at most two symbols; a symbol's (value, bound) pairs and the junk slots of 64
// lanes fit the wave's 1152-float exchange buffer)
__host__ __device__ inline bool soft_fast(uint32_t options, const DevCfg &cfg, bool dbg = false) {
  return soft_combine_applies(options, cfg.rep, cfg.mod) && !dbg && cfg.rep <= cfg.ndata * cfg.bps &&
         2 * (cfg.bps * cfg.ndata + 8 + 64 * cfg.bps) <= 1152;
}



// ---------------------------------------------------------------- helpers --
// Lane id through an opaque copy: inside persistent frame loops this keeps the
// compiler from hoisting lane-derived addresses out of the loop (they would stay
// live across every stage and exhaust the register file).
__device__ __forceinline__ int ltid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ int wave_lane() { return ltid() & 63; }

template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T> __device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o, 64); v = w > v ? w : v; }
  return v;
}
template <typename T> __device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o, 64); v = w < v ? w : v; }
  return v;
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}

// byte i of an MSB-first packed bit stream (word w holds bytes 4w..4w+3, big-endian)
__device__ __forceinline__ uint32_t stream_byte(const uint32_t *w, int i) {
  return (w[i >> 2] >> (24 - 8 * (i & 3))) & 0xFFu;
}
__device__ __forceinline__ int32_t be32_at(const uint32_t *w, int i) {
  return (int32_t)((stream_byte(w, i) << 24) | (stream_byte(w, i + 1) << 16) |
                   (stream_byte(w, i + 2) << 8) | stream_byte(w, i + 3));
}

// apply a zero-byte shift operator stored as 4 byte tables
__device__ __forceinline__ uint32_t crc_apply(const uint32_t *op, uint32_t r) {
  return op[r & 0xFF] ^ op[256 + ((r >> 8) & 0xFF)] ^ op[512 + ((r >> 16) & 0xFF)] ^ op[768 + (r >> 24)];
}

// Per-frame parse, modem.js:607-653 (legacy), 805-849 (meta/data), 793-802 (chunk).
// Fills r (status, offsets, header fields); returns the CRC range length or -1.
__device__ inline int parse_stream(const uint32_t *v, int nbytes, int mode, amod_result &r) {
  r.nbytes = nbytes;
  const int min_bytes = mode == AMOD_MODE_CHUNK ? 6 : 10;
  if (nbytes < min_bytes) { r.status = AMOD_E_DECODED_SHORT; r.frame_type = -1; return -1; }
  const int t = (int)stream_byte(v, 0);
  if (t == 0xFE) {
    r.frame_type = 0xFE;
    if (nbytes < 16) { r.status = AMOD_E_META_SHORT; return -1; }
    r.total_chunks = be32_at(v, 1);
    r.total_size = be32_at(v, 5);
    r.chunk_size = (int32_t)((stream_byte(v, 9) << 8) | stream_byte(v, 10));
    const int nl = (int)stream_byte(v, 11);
    int off = 12;
    if (off + nl + 4 > nbytes) { r.status = AMOD_E_META_TRUNC; return -1; }
    r.name_off = off; r.name_len = nl;
    off += nl;
    r.expected_crc = (uint32_t)be32_at(v, off);
    r.status = AMOD_OK;
    return off;
  }
  if (t == 0xFF) {
    r.frame_type = 0xFF;
    if (nbytes < 11) { r.status = AMOD_E_CHUNK_SHORT; return -1; }
    r.seq_num = be32_at(v, 1);
    const int dl = (int)((stream_byte(v, 5) << 8) | stream_byte(v, 6));
    int off = 7;
    if (off + dl + 4 > nbytes) { r.status = AMOD_E_CHUNK_TRUNC; return -1; }
    r.data_off = off; r.data_len = dl;
    off += dl;
    r.expected_crc = (uint32_t)be32_at(v, off);
    r.status = AMOD_OK;
    return off;
  }
  if (mode == AMOD_MODE_CHUNK) { r.frame_type = t; r.aux = t; r.status = AMOD_E_UNKNOWN_TYPE; return -1; }
  r.frame_type = 0;
  const int nl = t;
  int off = 1;
  if (off + nl + 4 + 4 > nbytes) { r.status = AMOD_E_SHORT_HEADER; return -1; }
  r.name_off = off; r.name_len = nl;
  off += nl;
  const int32_t dl = be32_at(v, off);
  off += 4;
  if (dl <= 0 || (int64_t)off + dl + 4 > nbytes) { r.status = AMOD_E_INVALID_LEN; r.aux = dl; return -1; }
  r.data_off = off; r.data_len = dl;
  off += dl;
  r.expected_crc = (uint32_t)be32_at(v, off);
  r.status = AMOD_OK;
  return off;
}

// Byte i of the majority-voted stream (modem.js:487-495 then 468-476), read from
// the raw MSB-first bit array; rep == 1 reads the raw stream directly.
__device__ inline uint32_t voted_byte(const uint32_t *raw, int i, int rep) {
  if (rep == 1) return stream_byte(raw, i);
  const int thr = (rep + 1) >> 1;
  uint32_t out = 0;
  for (int b = 0; b < 8; ++b) {
    const int j = 8 * i + b;
    int sum = 0;
    for (int u = 0; u < rep; ++u) {
      const int pos = j * rep + u;
      sum += (raw[pos >> 5] >> (31 - (pos & 31))) & 1;
    }
    out = (out << 1) | (uint32_t)(sum >= thr);
  }
  return out;
}

// How many leading bytes of the voted stream parse_stream() reads for a stream of
// nbytes bytes, given that the first `avail` are known. The answer only ever
// grows as more bytes become known; the parse is final once it is <= avail.
// Reads exactly the bytes parse_stream branches on (modem.js:607-640, 793-849).
// *final: the value no longer depends on bytes past `avail` (the header is decoded)
__device__ inline int parse_need(const uint32_t *raw, int rep, int avail, int nbytes, int mode, bool *final = nullptr) {
  bool fin = true;
  int r;
  const int min_bytes = mode == AMOD_MODE_CHUNK ? 6 : 10;
  if (nbytes < min_bytes) r = 0;
  else if (avail < 1) { r = 1; fin = false; }
  else {
    const int t = (int)voted_byte(raw, 0, rep);
    if (t == 0xFE) {
      if (nbytes < 16) r = 1;
      else if (avail < 12) { r = 12; fin = false; }
      else {
        const int nl = (int)voted_byte(raw, 11, rep);
        r = 12 + nl + 4 > nbytes ? 12 : 12 + nl + 4;
      }
    } else if (t == 0xFF) {
      if (nbytes < 11) r = 1;
      else if (avail < 7) { r = 7; fin = false; }
      else {
        const int dl = (int)((voted_byte(raw, 5, rep) << 8) | voted_byte(raw, 6, rep));
        r = 7 + dl + 4 > nbytes ? 7 : 7 + dl + 4;
      }
    } else if (mode == AMOD_MODE_CHUNK) {
      r = 1;
    } else {
      const int nl = t;
      if (1 + nl + 8 > nbytes) r = 1;
      else if (avail < 1 + nl + 4) { r = 1 + nl + 4; fin = false; }
      else {
        int32_t dl = 0;
        for (int q = 0; q < 4; ++q) dl = (int32_t)(((uint32_t)dl << 8) | voted_byte(raw, 1 + nl + q, rep));
        r = (dl <= 0 || (int64_t)1 + nl + 4 + dl + 4 > nbytes) ? 1 + nl + 4 : 1 + nl + 4 + dl + 4;
      }
    }
  }
  if (final) *final = fin;
  return r;
}

// Workgroup CRC-32 (modem.js:443-457) of bytes [0, L) of stream v.
// 256 threads each hash one 16-byte chunk with slice-by-4 tables; the chunk
// registers are moved to the end of the message with precomputed zero-byte
// shift operators and XOR-combined (CRC linearity). `red` is >= 8 words of LDS.
__device__ inline uint32_t block_crc32(const uint32_t *v, int L, const DevTables &t, uint32_t *red) {
  const int tid = ltid();
  uint32_t reg = 0xFFFFFFFFu; // register carried between 4096-byte passes (uniform)
  const int npass = (L + kCrcBlock - 1) / kCrcBlock;
  for (int pass = 0; pass < npass; ++pass) {
    const int p0 = pass * kCrcBlock;
    const int plen = min(kCrcBlock, L - p0);
    const int nch = (plen + kCrcChunk - 1) / kCrcChunk; // chunks, right-aligned
    uint32_t contrib = 0;
    if (tid < kCrcLanes) {
      const int j = tid - (kCrcLanes - nch); // chunk index from the left, may be negative
      if (j >= 0) {
        const int end = plen - (nch - 1 - j) * kCrcChunk; // exclusive, relative to p0
        const int beg = max(0, end - kCrcChunk);
        uint32_t c = (j == 0) ? reg : 0u;
        int i = beg;
        for (; i + 4 <= end; i += 4) {
          c ^= (stream_byte(v, p0 + i) | (stream_byte(v, p0 + i + 1) << 8) |
                (stream_byte(v, p0 + i + 2) << 16) | (stream_byte(v, p0 + i + 3) << 24));
          c = t.crc_s4[768 + (c & 0xFF)] ^ t.crc_s4[512 + ((c >> 8) & 0xFF)] ^
              t.crc_s4[256 + ((c >> 16) & 0xFF)] ^ t.crc_s4[c >> 24];
        }
        for (; i < end; ++i) c = t.crc_s4[(c ^ stream_byte(v, p0 + i)) & 0xFF] ^ (c >> 8);
        const int q = nch - 1 - j; // chunks to its right -> shift by 16q bytes
        if (q & 31) c = crc_apply(t.crc_m1 + (q & 31) * 1024, c);
        if (q >> 5) c = crc_apply(t.crc_m2 + (q >> 5) * 1024, c);
        contrib = c;
      }
    }
    contrib = wave_xor(contrib);
    __syncthreads();
    if ((tid & 63) == 0 && tid < kCrcLanes) red[tid >> 6] = contrib;
    __syncthreads();
    reg = red[0] ^ red[1] ^ red[2] ^ red[3];
    __syncthreads();
  }
  return reg ^ 0xFFFFFFFFu;
}

// Majority vote (modem.js:487-495) of the bit stream `bits` (nbits) into `voted`
// (words), returns the voted bit count. rep == 1 is a pass-through handled by
// the caller. Whole workgroup.
// soft vote: bit j = sign of the sum (in order, double) of its group's soft values
// (a value < 0 stands for bit 1)
__device__ inline int soft_vote(const float *sv, int nbits, int rep, uint32_t *voted) {
  const int nv = nbits / rep;
  const int nw = (nv + 31) >> 5;
  for (int w = ltid(); w < nw; w += blockDim.x) {
    uint32_t word = 0;
    for (int b = 0; b < 32; ++b) {
      const int j = w * 32 + b;
      if (j >= nv) break;
      double sum = 0.0;
      for (int u = 0; u < rep; ++u) sum += (double)sv[j * rep + u];
      word |= (uint32_t)(sum < 0.0) << (31 - b);
    }
    voted[w] = word;
  }
  return nv;
}

__device__ inline int block_vote(const uint32_t *bits, int nbits, int rep, uint32_t *voted) {
  const int nv = nbits / rep;
  const int nw = (nv + 31) >> 5;
  if (rep == 3) {
    // voted word w is raw bits [96 w, 96 w + 96) = raw words 3w .. 3w + 2 (MSB-first): the
    // majority of bits k, k + 1, k + 2 lands at bit k of maj(p, p << 1, p << 2) (shifts
    // across the three words), and bits k = 0, 3, ..., 93 are gathered into the word.
    // (The raw words read past nbits are zero: the callers clear nwords + 8.)
    for (int w = ltid(); w < nw; w += blockDim.x) {
      const uint32_t p0 = bits[3 * w], p1 = bits[3 * w + 1], p2 = bits[3 * w + 2];
      const uint32_t q0 = (p0 << 1) | (p1 >> 31), q1 = (p1 << 1) | (p2 >> 31), q2 = p2 << 1;
      const uint32_t r0 = (p0 << 2) | (p1 >> 30), r1 = (p1 << 2) | (p2 >> 30), r2 = p2 << 2;
      const uint32_t m[3] = {(p0 & q0) | (p0 & r0) | (q0 & r0), (p1 & q1) | (p1 & r1) | (q1 & r1),
                             (p2 & q2) | (p2 & r2) | (q2 & r2)};
      uint32_t word = 0;
#pragma unroll
      for (int o = 0; o < 32; ++o) word |= ((m[(3 * o) >> 5] >> (31 - ((3 * o) & 31))) & 1u) << (31 - o);
      const int left = nv - 32 * w; // voted bits in this word (the rest stay 0)
      if (left < 32) word &= ~(0xFFFFFFFFu >> left);
      voted[w] = word;
    }
    return nv;
  }
  const int thr = (rep + 1) >> 1; // sum >= rep/2  <=>  sum >= ceil(rep/2)
  for (int w = ltid(); w < nw; w += blockDim.x) {
    uint32_t word = 0;
    for (int b = 0; b < 32; ++b) {
      const int j = w * 32 + b;
      if (j >= nv) break;
      int sum = 0;
      for (int u = 0; u < rep; ++u) {
        const int pos = j * rep + u;
        sum += (bits[pos >> 5] >> (31 - (pos & 31))) & 1;
      }
      word |= (uint32_t)(sum >= thr) << (31 - b);
    }
    voted[w] = word;
  }
  return nv;
}

// Parse + CRC + store of one frame whose (voted) bit stream is in `v`.
// r must already hold status = AMOD_OK and the detection fields. Whole workgroup.
// store_bytes: how many leading payload bytes are decoded and stored (the fast
// kernel demodulates only the symbols holding header, data and CRC bytes).
__device__ inline void finish_frame(const uint32_t *v, int nvoted, const DevCfg &cfg, amod_result &r_in,
                                    amod_result *out, uint8_t *slot, int64_t stride, uint32_t *red,
                                    int *shared_status, int store_bytes) {
  const int nbytes = nvoted >> 3;
  store_bytes = min(store_bytes, nbytes);
  __shared__ amod_result r_sh;
  __shared__ int crc_len;
  if (threadIdx.x == 0) {
    r_sh = r_in;
    crc_len = parse_stream(v, nbytes, cfg.mode, r_sh);
    if (cfg.mode == AMOD_MODE_RECEIVED) {
      // preambleIdx is reported on legacy success and on every 0xFE/0xFF result (609-620)
      const bool keep = (r_sh.frame_type == 0xFE || r_sh.frame_type == 0xFF) ||
                        (r_sh.frame_type == 0 && r_sh.status == AMOD_OK);
      if (!keep) r_sh.preamble_idx = -1;
    } else {
      r_sh.preamble_idx = -1;
    }
  }
  __syncthreads();
  const int L = crc_len;
  if (L >= 0) {
    const uint32_t crc = block_crc32(v, L, cfg.t, red);
    if (threadIdx.x == 0) {
      r_sh.actual_crc = crc;
      r_sh.crc_valid = r_sh.expected_crc == crc;
    }
  }
  // payload bytes, big-endian words -> memory order
  const int nw = (store_bytes + 3) >> 2;
  uint32_t *dst = reinterpret_cast<uint32_t *>(slot);
  const int cap_w = (int)(stride >> 2);
  for (int w = ltid(); w < nw && w < cap_w; w += blockDim.x) {
    uint32_t word = v[w];
    const int keep = store_bytes - 4 * w; // bytes of this word that were decoded
    if (keep < 4) word &= ~(0xFFFFFFFFu >> (8 * keep));
    dst[w] = __builtin_bswap32(word);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    r_sh.payload_valid = store_bytes;
    *out = r_sh;
    if (shared_status) *shared_status = r_sh.status;
  }
}

// the first launch of a decode: the counters later launches append to (DevWork::fb_zero),
// and a profiled decode's timeline slot (DevWork::tl)
__device__ inline void tl_init(const DevWork &w) {
  if (w.fb_zero && blockIdx.x == 0 && threadIdx.x == 0) { w.fb_zero[0] = 0; w.fb_zero[1] = 0; w.fb_zero[2] = 0; }
  if (w.tl && blockIdx.x == 0 && threadIdx.x == 0) {
    w.tl[0] = ~0ull; w.tl[1] = 0ull; w.tl[2] = 0ull; w.tl[3] = 0ull;
  }
}

__device__ inline void init_result(amod_result &r) {
  r.status = AMOD_OK; r.preamble_idx = -1; r.coarse_idx = -1; r.frame_type = -1; r.aux = 0;
  r.nbytes = 0; r.name_off = 0; r.name_len = 0; r.data_off = 0; r.data_len = 0;
  r.seq_num = 0; r.total_chunks = 0; r.total_size = 0; r.chunk_size = 0;
  r.expected_crc = 0; r.actual_crc = 0; r.crc_valid = 0; r.nbits = 0; r.flags = 0;
  r.fine_metric = 0.f; r.payload_valid = 0; r.reserved[0] = r.reserved[1] = r.reserved[2] = 0;
}

} // namespace amod

// kernels (defined in k_decode_fast.hip / k_decode_exact.hip)
extern "C" {
hipError_t amod_launch_detect(const amod::DevCfg &cfg, const amod::DevWork &w, hipStream_t s); // k_detect / k_chunk_prep
hipError_t amod_launch_demod(const amod::DevCfg &cfg, const amod::DevWork &w, int nblocks, hipStream_t s);
int amod_demod_blocks_per_cu(const amod::DevCfg &cfg, int lds, bool soft);
void amod_demod_stream_words(const amod::DevCfg &cfg, int mcap, int *stream_words, int *vote_off);
hipError_t amod_launch_exact(const amod::DevCfg &cfg, const amod::DevWork &w, int nslots, hipStream_t s,
                             bool beside_demod = false); // list A runs beside k_demod
hipError_t amod_launch_tx(const amod::DevCfg &cfg, const amod::DevTxWork &w, hipStream_t s);
hipError_t amod_launch_flush(const void *buf, size_t bytes, float *sink, hipStream_t s); // experiments
int amod_fast_lds_bytes(int nb_cap, int fine_cap, int sym); // dynamic LDS of one k_detect workgroup
// streaming receiver pieces (k_stream.hip)
// (kn: the calling context's knobs, for the EMA's experiment shapes; null: the defaults)
int64_t amod_ema_chunk();
hipError_t amod_launch_ema(const float *x, int64_t nx, int64_t n, float *y, double *warm, double *end, double *scr,
                           int64_t *list, const double *apow, unsigned long long *fixed, hipStream_t s,
                           const amod::Knobs *kn);
int64_t amod_ema_wave_samples(const amod::Knobs *kn); // the stream piece granule of amod_launch_ema_part
hipError_t amod_launch_ema_part(const float *x, int64_t nx, int64_t n, float *y, double *warm, double *end, double *scr,
                                const double *apow, int64_t s0, int64_t s1, hipStream_t s, const amod::Knobs *kn);
hipError_t amod_launch_ema_fix(const float *x, int64_t nx, int64_t n, float *y, double *warm, double *end,
                               int64_t *list, unsigned long long *fixed, hipStream_t s, const amod::Knobs *kn);
hipError_t amod_launch_sc_screen(const float *y, int64_t n, float thresh, double2 *ze, uint8_t *hot, hipStream_t s);
hipError_t amod_launch_fine(const float *y, int64_t n, const double *pre1, int sym, double pre1_energy,
                            const int64_t *first, const int64_t *base, const int64_t *count, int nranges,
                            int64_t maxcount, double *out, double *out_dev, double2 *barg, hipStream_t s);
hipError_t amod_launch_gap_scan(const float *y, int64_t n, int64_t lo, const int64_t *first, const double2 *barg,
                                int nbx, int nranges, int64_t F, int64_t cap, int64_t nblocks, int max_blocks,
                                amod::GapScan *out, hipStream_t s);
hipError_t amod_launch_ranges(const uint8_t *hot, int64_t nhot, int32_t *wg, int64_t *first, int64_t *count,
                              hipStream_t s);
hipError_t amod_launch_gap_refine(amod::GapScan *g, int nrec, int64_t lo, const int64_t *first, const int64_t *base,
                                  const int64_t *count, int nranges, const double *metric, int64_t radius, hipStream_t s);
hipError_t amod_launch_window(const float *y, int64_t n, const int64_t *pos, const int32_t *len, const int64_t *woff,
                              int nwin, float *out, hipStream_t s);
hipError_t amod_launch_gather(const float *y, const int32_t *src, int ng, float *out, hipStream_t s);
// runtime.cpp: a context's device and stream for the host-side orchestrators
int amod_ctx_device(const amod_ctx *ctx);
hipStream_t amod_ctx_stream(const amod_ctx *ctx);
const amod::Knobs *amod_ctx_knobs(const amod_ctx *ctx); // read once at amod_open
// the event recorded on the launch stream right after the latest decode's k_detect (null if
// that decode had none: chunk mode, chunked or serial diagnostics, a captured decode)
hipEvent_t amod_ctx_detect_event(const amod_ctx *ctx);
int amod_ctx_fail(amod_ctx *ctx, const char *msg, int code);
// per-context state owned by another module (slot: 0 = streaming receiver): *amod_ctx_ext
// holds it; free_fn runs at amod_close, after the context's streams are drained
void **amod_ctx_ext(amod_ctx *ctx, int slot, void (*free_fn)(void *));
int amod_cfg_valid(const amod_cfg *cfg); // the decode entry points' configuration check
}
