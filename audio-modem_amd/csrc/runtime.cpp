// runtime.cpp — host side of libamodem.so: the C ABI declared in include/amodem.h.
//
// Owns one HIP stream and a grow-only device workspace per context, builds the
// per-configuration device tables (preamble template, CE signs, FFT twiddles,
// CRC operators, constellation), and enqueues k_decode_fast followed by
// k_decode_exact. Also carries the reference-equivalent transmit builders used
// to synthesise benchmark input (modem.js buildTransmitSignal & co.).
// Built with -ffp-contract=off: the template/twiddle arithmetic must round
// exactly like modem.js.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "amodem.h"
#include "amodem_internal.h"

namespace {

thread_local std::string g_last_error;

// ------------------------------------------------------------ reference math
// seededRandom (modem.js:153-156): product and sum in double, ToInt32, & 0x7fffffff
struct SeededRandom {
  double s;
  explicit SeededRandom(double seed) : s(seed) {}
  double next() {
    const double prod = s * 1103515245.0;
    const double sum = prod + 12345.0;
    const uint64_t as_u = (uint64_t)std::fmod(sum, 18446744073709551616.0);
    const uint32_t v = (uint32_t)as_u & 0x7fffffffu;
    s = (double)v;
    return (double)v / 2147483647.0;
  }
};

// per-stage twiddle recurrence of fftIterative (modem.js:28-44), 511 entries:
// stage with half-size h uses entries [h-1, 2h-1)
std::vector<double> stage_twiddles(bool inverse) {
  std::vector<double> t(2 * 511);
  for (int size = 2; size <= amod::kFft; size <<= 1) {
    const int half = size >> 1;
    const double sign = inverse ? 1.0 : -1.0;
    const double angle = sign * 2.0 * M_PI / (double)size;
    const double wn_re = std::cos(angle), wn_im = std::sin(angle);
    double w_re = 1.0, w_im = 0.0;
    for (int j = 0; j < half; ++j) {
      t[2 * (half - 1 + j)] = w_re;
      t[2 * (half - 1 + j) + 1] = w_im;
      const double nw = w_re * wn_re - w_im * wn_im;
      w_im = w_re * wn_im + w_im * wn_re;
      w_re = nw;
    }
  }
  return t;
}

// 512-point transform with the reference's exact rounding (bitReverse + stages)
void ref_fft512(double *re, double *im, bool inverse) {
  static const std::vector<double> fw = stage_twiddles(false), bw = stage_twiddles(true);
  const std::vector<double> &tw = inverse ? bw : fw;
  const int n = amod::kFft;
  for (int i = 0; i < n; ++i) {
    int j = 0;
    for (int b = 0, x = i; b < 9; ++b, x >>= 1) j = (j << 1) | (x & 1);
    if (i < j) { std::swap(re[i], re[j]); std::swap(im[i], im[j]); }
  }
  for (int half = 1; half < n; half <<= 1) {
    for (int start = 0; start < n; start += 2 * half) {
      for (int j = 0; j < half; ++j) {
        const double wr = tw[2 * (half - 1 + j)], wi = tw[2 * (half - 1 + j) + 1];
        const int a = start + j, b = a + half;
        const double tr = wr * re[b] - wi * im[b];
        const double ti = wr * im[b] + wi * re[b];
        re[b] = re[a] - tr; im[b] = im[a] - ti;
        re[a] += tr; im[a] += ti;
      }
    }
  }
  if (inverse) {
    const double scale = 1.0 / (double)n;
    for (int i = 0; i < n; ++i) { re[i] *= scale; im[i] *= scale; }
  }
}

void constellation(int mod, int idx, double &re, double &im) { // initConstellation 107-131
  if (mod == AMOD_BPSK) { re = idx == 0 ? 1.0 : -1.0; im = 0.0; return; }
  if (mod == AMOD_QPSK) {
    const double s = 1.0 / M_SQRT2;
    re = (idx == 0 || idx == 3) ? s : -s;
    im = (idx <= 1) ? s : -s;
    return;
  }
  const int row = idx >> 2, col = idx & 3;
  const int gr = row ^ (row >> 1), gc = col ^ (col >> 1);
  const double s = 1.0 / std::sqrt(10.0);
  re = (double)(2 * gc - 3) * s;
  im = (double)(2 * gr - 3) * s;
}
int npoints(int mod) { return mod == AMOD_BPSK ? 2 : mod == AMOD_QPSK ? 4 : 16; }
int bps_of(int mod) { return mod == AMOD_BPSK ? 1 : mod == AMOD_QPSK ? 2 : 4; }

int demap_exact(int mod, double re, double im) { // constellationDemap 140-150
  double best = INFINITY;
  int bi = 0;
  for (int i = 0; i < npoints(mod); ++i) {
    double pr, pi;
    constellation(mod, i, pr, pi);
    const double dr = re - pr, di = im - pi, d = dr * dr + di * di;
    if (d < best) { best = d; bi = i; }
  }
  return bi;
}

bool is_pilot(const amod_cfg &c, int k) {
  for (int i = 0; i < c.npilots; ++i)
    if (c.pilots[i] == k) return true;
  return false;
}

// Hermitian-complete a half spectrum, IFFT, prepend the cyclic prefix (modem.js:166-169, 202-208)
void symbol_from_spectrum(const amod_cfg &c, double *re, double *im, bool zero_dc_im, float *out) {
  const int n = amod::kFft;
  for (int k = 1; k < n / 2; ++k) { re[n - k] = re[k]; im[n - k] = -im[k]; }
  re[0] = 0;
  if (zero_dc_im) im[0] = 0;
  else re[n / 2] = 0;
  im[n / 2] = 0;
  ref_fft512(re, im, true);
  for (int i = 0; i < c.cp_len; ++i) out[i] = (float)re[n - c.cp_len + i];
  for (int i = 0; i < n; ++i) out[c.cp_len + i] = (float)re[i];
}

// generatePreambleSymbol1/2 and generateChannelEstSymbol (modem.js:158-200)
void template_symbol(const amod_cfg &c, double seed, int step, float *out, double *known) {
  double re[amod::kFft] = {0}, im[amod::kFft] = {0};
  SeededRandom rng(seed);
  for (int k = c.sub_start; k <= c.sub_end; k += step) {
    re[k] = rng.next() > 0.5 ? 1.0 : -1.0;
    if (known) known[k] = re[k];
  }
  symbol_from_spectrum(c, re, im, false, out);
}

// ------------------------------------------------------------------- CRC ---
uint32_t crc_step_zero(uint32_t r) { // feed one zero byte (reflected 0xEDB88320)
  for (int j = 0; j < 8; ++j) r = (r & 1) ? (0xEDB88320u ^ (r >> 1)) : (r >> 1);
  return r;
}
const uint32_t *crc_table() {
  static uint32_t t[256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; ++i) t[i] = crc_step_zero(i);
  });
  return t;
}
// operator tables for "advance the register over n zero bytes"
void shift_operator(int64_t nbytes, uint32_t *op /*4*256*/) {
  // basis images of the 32 single-bit registers, then byte tables
  uint32_t basis[32];
  for (int b = 0; b < 32; ++b) {
    uint32_t r = 1u << b;
    for (int64_t i = 0; i < nbytes; ++i) r = crc_table()[r & 0xFF] ^ (r >> 8);
    basis[b] = r;
  }
  for (int byte = 0; byte < 4; ++byte)
    for (int v = 0; v < 256; ++v) {
      uint32_t acc = 0;
      for (int bit = 0; bit < 8; ++bit)
        if (v & (1 << bit)) acc ^= basis[8 * byte + bit];
      op[byte * 256 + v] = acc;
    }
}

// ---------------------------------------------------------------- device ---
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      g_last_error = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
      return AMOD_ERR_HIP;                                                              \
    }                                                                                   \
  } while (0)

// Grow-only device buffer. A buffer a captured hipGraph may still reference (`keep`
// set once a decode was captured) is never freed when it grows: the old allocation moves
// to `retired` and lives until the context closes, so replays keep valid memory.
struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  const bool *keep = nullptr;
  std::vector<void *> *retired = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) {
      if (keep && *keep && retired) retired->push_back(p);
      else (void)hipFree(p);
      p = nullptr; n = 0;
    }
    hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 256));
    if (e == hipSuccess) n = std::max<size_t>(bytes, 256);
    return e;
  }
};

// Grow-only pinned host buffer (amod_decode_host's per-piece copies of the outputs)
struct HostBuf {
  void *p = nullptr;
  size_t n = 0;
  ~HostBuf() { if (p) (void)hipHostFree(p); }
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) { (void)hipHostFree(p); p = nullptr; n = 0; }
    hipError_t e = hipHostMalloc(&p, std::max<size_t>(bytes, 256), hipHostMallocDefault);
    if (e == hipSuccess) n = std::max<size_t>(bytes, 256);
    return e;
  }
};

struct TableSet {
  DevBuf buf;
  amod::DevCfg cfg{};
};

using CfgKey = std::tuple<std::vector<int32_t>>;

std::vector<int32_t> cfg_key(const amod_cfg &c) {
  std::vector<int32_t> k = {c.fft_size, c.cp_len, c.symbol_len, c.sub_start, c.sub_end, c.npilots,
                            c.modulation, c.repetition};
  for (int i = 0; i < c.npilots; ++i) k.push_back(c.pilots[i]);
  return k;
}

} // namespace

constexpr int kTlSlots = 64;     // profiled decodes whose timeline marks are kept between harvests
constexpr int kMaxChunks = 16;   // frame chunks of one decode (two-stream overlap)
constexpr int kOverlapChunks = 1; // default chunk count (measured: overlap slows both launches)

struct amod_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::map<std::vector<int32_t>, std::unique_ptr<TableSet>> tables; // per cfg x mode-independent
  DevBuf crc;          // shared CRC tables
  DevBuf fb;           // fb_count + list + flags
  DevBuf xs, bits;     // exact-kernel scratch
  DevBuf soft;         // exact-kernel soft bit values (AMOD_OPT_SOFT_COMBINE only)
  DevBuf det;          // fast path: per-frame detection records (k_detect -> k_demod)
  hipStream_t aux = nullptr;  // k_demod of chunk c beside k_detect of chunk c + 1
  std::array<hipEvent_t, kMaxChunks + 1> chunk_ev{};
  int cu_count = 0, demod_lds = -1, demod_mod = -1, demod_nband = -1, demod_bpc = 0, demod_soft = -1;
  // fb[0 .. 2] are the decode's counts (lists from fb + 64), zeroed by the decode's own first
  // and last launches (DevWork::fb_zero, fb_reset). fb_zeroed: they are zero when this decode's
  // launches run; a reallocation or an aborted launch sequence clears it (memset)
  bool fb_zeroed = false;
  bool detect_ev = false; // chunk_ev[0] marks the end of the latest decode's k_detect (pipes)
  bool fb_captured = false; // a decode was captured into a hipGraph: a buffer that grows is
                            // kept (not freed) until amod_close, for the graph's replays
  void *ext[4] = {nullptr, nullptr, nullptr, nullptr}; // other modules' per-context state
  void (*ext_free[4])(void *) = {nullptr, nullptr, nullptr, nullptr};
  int64_t soft_stride = 0;
  int soft_slots = 0;
  int64_t xs_stride = 0, bits_stride = 0;
  int nslots = 0;
  int64_t max_len = 0; // longest frame any reservation was sized for (exact-kernel workspace)
  // device path (amod_decode_device): the fast-path capacity, in samples, of the latest
  // amod_reserve (default 65536 before any). A frame's route depends on the frame, the
  // options and this capacity only, never on other calls' shapes (host paths size it from
  // the launch's own longest frame)
  int64_t dev_cap = 65536;
  std::vector<void *> retired; // buffers a captured graph may reference (freed at close)
  // host-path staging
  DevBuf h_samples, h_off, h_len, h_res, h_payload, h_dbg;
  // amod_decode_host's pipeline: the upload stream and one event per uploaded piece
  hipStream_t up = nullptr;
  std::vector<hipEvent_t> up_ev;
  // ... and its outputs: each piece's records and payload slots come back (DMA into pinned
  // mirrors, one event per piece) while later pieces upload, then go to the caller's buffers
  HostBuf pin_res, pin_payload;
  std::vector<hipEvent_t> dn_ev;
  std::mutex mu;
  DevBuf stamps;
  DevBuf flush; // AMOD_MALL_FLUSH_MB scratch (experiments)
  DevBuf tx_pkt, tx_meta, tx_out; // amod_tx_host staging
  int64_t nstamps = 0;
  // kernel timing (amod_set_profiling)
  bool profiling = false;
  // per decode: before k_detect, after k_detect, after k_demod (on the launch stream),
  // the end of the second stream's chain (list A's exact kernel + replay k_demod), after
  // the launch stream has joined it, after list B's exact kernel
  std::vector<std::array<hipEvent_t, 6>> ev_used, ev_free;
  // the device timeline marks of profiled decodes (amod_aux_overlap): kTlSlots slots of
  // tl_words each (amod::kTlHead + one per k_demod wave), one per decode in ring order;
  // tl_of[i] is ev_used[i]'s (slot, k_demod waves)
  DevBuf tl;
  int64_t tl_next = 0, tl_words = 0;
  std::vector<std::pair<int64_t, int64_t>> tl_of;
  int64_t ov_listed = 0, ov_beside = 0;
  double ov_lead_us = 0.0;
  amod::Knobs knobs; // read once at amod_open
};

namespace {

int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}
// the diagnostic / experiment knobs (amod::Knobs), read once per context at amod_open
void read_knobs(amod::Knobs &k) {
  if (const char *g = getenv("AMOD_GUARD_SCALE")) k.guard_scale = (float)atof(g);
  k.stop_after = env_int("AMOD_STOP_AFTER", 99);
  k.demod_mcap = std::max(0, env_int("AMOD_DEMOD_MCAP", 0));
  k.stamps = getenv("AMOD_STAMPS") != nullptr;
  k.demod_bpc = std::max(0, env_int("AMOD_DEMOD_BPC", 0));
  k.chunks = std::max(0, env_int("AMOD_CHUNKS", 0));
  k.xslots = std::max(0, env_int("AMOD_XSLOTS", 0));
  k.no_replay = getenv("AMOD_NO_REPLAY") != nullptr;
  k.exact_serial = getenv("AMOD_EXACT_SERIAL") != nullptr;
  if (const char *e = getenv("AMOD_UP_PIECE")) k.up_piece = std::max<int64_t>(0, atoll(e));
  k.aux_priority = env_int("AMOD_AUX_PRIORITY", 1);
  k.pipe_stagger = env_int("AMOD_PIPE_STAGGER", 0);
  k.demod_static = getenv("AMOD_DEMOD_STATIC") != nullptr;
  k.claim_rounds = std::max(1, env_int("AMOD_CLAIM_ROUNDS", 2));
  k.claim_min = std::max(2, env_int("AMOD_CLAIM_MIN", 4));
  k.mall_flush_mb = std::max(0, env_int("AMOD_MALL_FLUSH_MB", 0));
  k.stream_minseg = std::max(0, env_int("AMOD_STREAM_MINSEG", 0));
  k.stream_diag = getenv("AMOD_STREAM_DIAG") != nullptr;
  k.stream_d2h = std::min(2, std::max(0, env_int("AMOD_STREAM_D2H", 1)));
  k.no_gap_scan = getenv("AMOD_NO_GAP_SCAN") != nullptr;
  k.stream_threads = env_int("AMOD_STREAM_THREADS", -1);
  k.stream_fullcopy = getenv("AMOD_STREAM_FULLCOPY") != nullptr;
  k.ema_per = env_int("AMOD_EMA_PER", -1);
  k.ema_warm = env_int("AMOD_EMA_WARM", -1);
  k.ema_rounds = env_int("AMOD_EMA_ROUNDS", -1);
}

int fail(amod_ctx *ctx, const std::string &msg, int code) {
  g_last_error = msg;
  if (ctx) ctx->err = msg;
  return code;
}

int validate(const amod_cfg *c) {
  if (!c) return 0;
  if (c->fft_size != amod::kFft) return 0;
  if (c->cp_len <= 0 || c->symbol_len != c->fft_size + c->cp_len) return 0;
  if (c->symbol_len > 768 || c->symbol_len % 4 != 0) return 0; // fine stage tap split / template buffer
  if (c->sub_start < 1 || c->sub_end >= c->fft_size / 2 || c->sub_start > c->sub_end) return 0;
  if (c->npilots < 0 || c->npilots > AMOD_MAX_PILOTS) return 0;
  if (c->modulation < AMOD_BPSK || c->modulation > AMOD_QAM16) return 0;
  if (c->repetition < 1) return 0;
  if (amod_num_data_subs(c) <= 0) return 0;
  return 1;
}

int build_crc(amod_ctx *ctx) {
  if (ctx->crc.p) return AMOD_SUCCESS;
  std::vector<uint32_t> h(4 * 256 + 32 * 1024 + 32 * 1024 + 1024 + amod::kCrcMats * 32 + 16 + 16 * 32);
  uint32_t *s4 = h.data(), *m1 = s4 + 1024, *m2 = m1 + 32 * 1024, *mb = m2 + 32 * 1024, *mat = mb + 1024;
  uint32_t *pre = mat + amod::kCrcMats * 32, *unpad = pre + 16;
  const uint32_t *t0 = crc_table();
  for (int i = 0; i < 256; ++i) s4[i] = t0[i];
  for (int k = 1; k < 4; ++k)
    for (int i = 0; i < 256; ++i) s4[k * 256 + i] = (s4[(k - 1) * 256 + i] >> 8) ^ t0[s4[(k - 1) * 256 + i] & 0xFF];
  for (int q = 0; q < 32; ++q) {
    shift_operator((int64_t)amod::kCrcChunk * q, m1 + q * 1024);
    shift_operator((int64_t)amod::kCrcChunk * 32 * q, m2 + q * 1024);
  }
  shift_operator(amod::kCrcBlock, mb);
  for (int b = 0; b < 32; ++b) { // matrices: column b = the register 1 << b after 16 q zero bytes
    uint32_t r = 1u << b;
    for (int q = 0; q < amod::kCrcMats; ++q) {
      mat[32 * q + b] = r;
      for (int i = 0; i < 16; ++i) r = crc_table()[r & 0xFF] ^ (r >> 8);
    }
  }
  // pre[k]: the register k zero bytes earlier that the k bytes advance to ~0. One zero
  // byte maps r to T[r & 0xFF] ^ (r >> 8); the top byte of T[x] is a bijection of x, so
  // the step inverts: x from the top byte, then r = ((r' ^ T[x]) << 8) | x
  {
    uint32_t inv_top[256];
    for (uint32_t x = 0; x < 256; ++x) inv_top[crc_table()[x] >> 24] = x;
    uint32_t r = 0xFFFFFFFFu;
    for (int k = 0; k < 16; ++k) {
      pre[k] = r;
      const uint32_t x = inv_top[r >> 24];
      r = ((r ^ crc_table()[x]) << 8) | x;
    }
    // unpad[k]: the inverse of k zero bytes as a GF(2) matrix (column b = the register that
    // k zero bytes advance to 1 << b), for k_demod's left-aligned CRC chunks
    for (int b = 0; b < 32; ++b) {
      uint32_t u = 1u << b;
      for (int k = 0; k < 16; ++k) {
        unpad[32 * k + b] = u;
        const uint32_t x = inv_top[u >> 24];
        u = ((u ^ crc_table()[x]) << 8) | x;
      }
    }
  }
  HIP_TRY(ctx->crc.ensure(h.size() * 4));
  HIP_TRY(hipMemcpy(ctx->crc.p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return AMOD_SUCCESS;
}

int get_tables(amod_ctx *ctx, const amod_cfg *c, amod::DevCfg &out) {
  int rc = build_crc(ctx);
  if (rc) return rc;
  auto key = cfg_key(*c);
  auto it = ctx->tables.find(key);
  if (it == ctx->tables.end()) {
    auto ts = std::make_unique<TableSet>();
    amod::DevCfg &d = ts->cfg;
    const int sym = c->symbol_len, nband = c->sub_end - c->sub_start + 1;
    d.cp = c->cp_len; d.sym = sym; d.sub_start = c->sub_start; d.sub_end = c->sub_end; d.nband = nband;
    d.npilots = c->npilots; d.ndata = amod_num_data_subs(c); d.bps = bps_of(c->modulation);
    d.mod = c->modulation; d.rep = c->repetition;
    for (int i = 0; i < c->npilots; ++i) d.pilots[i] = c->pilots[i];
    d.origin_idx = demap_exact(c->modulation, 0.0, 0.0);
    d.guard = ctx->knobs.guard_scale;
    d.stop_after = ctx->knobs.stop_after; // stage-cost diagnostics; results are not written
    // host images
    std::vector<float> pre1(sym), ce(sym), tmpl(3 * (size_t)sym);
    double known_full[amod::kFft] = {0};
    template_symbol(*c, 42.0, 2, pre1.data(), nullptr);
    template_symbol(*c, 44.0, 1, ce.data(), known_full);
    template_symbol(*c, 42.0, 2, tmpl.data(), nullptr);
    template_symbol(*c, 43.0, 1, tmpl.data() + sym, nullptr);
    template_symbol(*c, 44.0, 1, tmpl.data() + 2 * sym, nullptr);
    d.tx_tmax = 0.f;
    for (float v : tmpl) d.tx_tmax = std::max(d.tx_tmax, std::fabs(v));
    double te = 0.0;
    for (int i = 0; i < sym; ++i) te += (double)pre1[i] * (double)pre1[i];
    d.te = te; d.te_f = (float)te;
    // pre1 uses subcarriers of one parity, so its body repeats every 256 samples up
    // to a sign (even: +, odd: -): pre1[i + 256] = sign * pre1[i]. The fast fine stage
    // folds the correlation on it when the float32 template honours it to 1e-6.
    {
      const float sgn = (c->sub_start & 1) ? -1.f : 1.f;
      float tmax = 0.f, dmax = 0.f;
      for (int i = 0; i < sym; ++i) tmax = std::max(tmax, std::fabs(pre1[i]));
      for (int i = 0; i + 256 < sym; ++i) dmax = std::max(dmax, std::fabs(pre1[i + 256] - sgn * pre1[i]));
      d.fold = (sym - 512 <= 256 && dmax <= 1e-6f * tmax) ? (int)sgn : 0;
    }
    std::vector<float> known(nband);
    std::vector<int16_t> band_di(nband);
    int di = 0;
    for (int b = 0; b < nband; ++b) {
      const int k = c->sub_start + b;
      known[b] = (float)known_full[k];
      band_di[b] = is_pilot(*c, k) ? (int16_t)-1 : (int16_t)di++;
    }
    std::vector<float> tw1(2 * 8 * 64), tw2(2 * 8 * 8);
    for (int q = 0; q < 8; ++q)
      for (int l = 0; l < 64; ++l) {
        const double a = -2.0 * M_PI * (double)((l * q) % amod::kFft) / amod::kFft;
        tw1[2 * (q * 64 + l)] = (float)std::cos(a); tw1[2 * (q * 64 + l) + 1] = (float)std::sin(a);
      }
    for (int p = 0; p < 8; ++p)
      for (int l1 = 0; l1 < 8; ++l1) {
        const double a = -2.0 * M_PI * (double)((8 * l1 * p) % amod::kFft) / amod::kFft;
        tw2[2 * (p * 8 + l1)] = (float)std::cos(a); tw2[2 * (p * 8 + l1) + 1] = (float)std::sin(a);
      }
    const std::vector<double> twx = stage_twiddles(false), twi = stage_twiddles(true);
    std::vector<double> pts(2 * 16, 0.0);
    for (int i = 0; i < npoints(c->modulation); ++i) constellation(c->modulation, i, pts[2 * i], pts[2 * i + 1]);
    // one device allocation, 256-byte aligned pieces
    size_t off = 0;
    auto carve = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_pre1 = carve(sym * 4), o_tw1 = carve(tw1.size() * 4), o_tw2 = carve(tw2.size() * 4),
                 o_twx = carve(twx.size() * 8), o_known = carve(nband * 4), o_di = carve(nband * 2),
                 o_pts = carve(pts.size() * 8), o_twi = carve(twi.size() * 8), o_tmpl = carve(tmpl.size() * 4);
    if (ts->buf.ensure(off) != hipSuccess) return fail(ctx, "hipMalloc(tables)", AMOD_ERR_NOMEM);
    char *base = (char *)ts->buf.p;
    HIP_TRY(hipMemcpy(base + o_pre1, pre1.data(), sym * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_tw1, tw1.data(), tw1.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_tw2, tw2.data(), tw2.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_twx, twx.data(), twx.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_known, known.data(), nband * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_di, band_di.data(), nband * 2, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_pts, pts.data(), pts.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_twi, twi.data(), twi.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(base + o_tmpl, tmpl.data(), tmpl.size() * 4, hipMemcpyHostToDevice));
    d.t.pre1 = (const float *)(base + o_pre1);
    d.t.tw1 = (const float2 *)(base + o_tw1);
    d.t.tw2 = (const float2 *)(base + o_tw2);
    d.t.tw_exact = (const double2 *)(base + o_twx);
    d.t.known = (const float *)(base + o_known);
    d.t.band_di = (const int16_t *)(base + o_di);
    d.t.points = (const double2 *)(base + o_pts);
    d.t.tw_inv = (const double2 *)(base + o_twi);
    d.t.tmpl = (const float *)(base + o_tmpl);
    const uint32_t *crc = (const uint32_t *)ctx->crc.p;
    d.t.crc_s4 = crc;
    d.t.crc_m1 = crc + 1024;
    d.t.crc_m2 = crc + 1024 + 32 * 1024;
    d.t.crc_mb = crc + 1024 + 64 * 1024;
    d.t.crc_mat = crc + 1024 + 64 * 1024 + 1024;
    d.t.crc_pre = d.t.crc_mat + amod::kCrcMats * 32;
    d.t.crc_unpad = d.t.crc_pre + 16;
    it = ctx->tables.emplace(key, std::move(ts)).first;
  }
  out = it->second->cfg;
  return AMOD_SUCCESS;
}

int64_t max_bits_for(const amod_cfg *c, int64_t max_len) {
  return (max_len / c->symbol_len) * (int64_t)amod_num_data_subs(c) * bps_of(c->modulation);
}

constexpr int64_t kFastMaxLen = int64_t(1) << 18; // longest frame the fast path takes (k_detect moments in LDS)
constexpr int64_t kUpPiece = int64_t(16) << 20; // amod_decode_host: samples per uploaded piece (64 MB)

// capacities of one fast-path launch over frames of up to max_len samples
struct ChainDims {
  int64_t fast_len;
  int nb_cap, fine_cap, mcap;
};
ChainDims chain_dims(const amod_cfg *c, int64_t max_len) {
  ChainDims d;
  d.fast_len = std::min<int64_t>(std::max<int64_t>(max_len, 0), kFastMaxLen);
  d.nb_cap = 8 * (int)((d.fast_len + 3 + 255) / 256) + 8;
  d.fine_cap = (12 * c->cp_len + 1 + 7) & ~7; // every window the coarse stage lets through
  d.mcap = (int)std::max<int64_t>(0, d.fast_len / c->symbol_len - 3);
  return d;
}

// device buffers of the fast path for nframes frames (grow-only)
int ensure_chain(amod_ctx *ctx, int32_t nframes) {
  HIP_TRY(ctx->det.ensure(sizeof(amod::DetRec) * (size_t)std::max(nframes, 1)));
  return AMOD_SUCCESS;
}

// exact-list counters + lists for nframes frames (grow-only; a new buffer is not zeroed)
static hipError_t fb_grow(amod_ctx *ctx, int32_t nframes) {
  const size_t bytes = sizeof(int32_t) * (size_t)(64 + 5 * (size_t)std::max(nframes, 1));
  if (bytes <= ctx->fb.n) return hipSuccess;
  ctx->fb_zeroed = false;
  return ctx->fb.ensure(bytes);
}

int reserve(amod_ctx *ctx, const amod_cfg *c, int32_t nframes, int64_t max_len) {
  if (max_len < 0) { // device path: keep what amod_reserve set up, or size for dev_cap
    HIP_TRY(fb_grow(ctx, nframes));
    if (ctx->nslots > 0 && ctx->max_len >= ctx->dev_cap) return AMOD_SUCCESS;
    max_len = ctx->dev_cap;
  }
  const int64_t nslots = std::max<int64_t>(1, std::min<int64_t>({(int64_t)nframes, 512,
      std::max<int64_t>(1, (int64_t)(2ll << 30) / std::max<int64_t>(1, max_len * 4))}));
  HIP_TRY(fb_grow(ctx, nframes));
  // grow-only: a later, smaller reservation never shrinks a stride or the slot count that
  // earlier (longer) frames were sized for
  const int64_t words = (max_bits_for(c, max_len) + 31) / 32;
  const int64_t xs_stride = std::max<int64_t>(ctx->xs_stride, (max_len + 64) & ~int64_t(63));
  const int64_t bits_stride = std::max<int64_t>(ctx->bits_stride, ((2 * words + 32) + 63) & ~int64_t(63));
  const int64_t slots = std::max<int64_t>(ctx->nslots, nslots);
  HIP_TRY(ctx->xs.ensure(sizeof(float) * (size_t)(slots * xs_stride)));
  HIP_TRY(ctx->bits.ensure(sizeof(uint32_t) * (size_t)(slots * bits_stride)));
  ctx->xs_stride = xs_stride;
  ctx->bits_stride = bits_stride;
  ctx->nslots = (int)slots;
  ctx->max_len = std::max<int64_t>(ctx->max_len, max_len);
  return ensure_chain(ctx, nframes);
}

int decode_impl(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples, const int64_t *offsets,
                const int32_t *lengths, int32_t nframes, amod_result *results, uint8_t *payload,
                int64_t payload_stride, uint32_t options, hipStream_t stream, amod_debug *debug,
                int64_t max_len) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  if (!validate(cfg)) return fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  if (mode != AMOD_MODE_RECEIVED && mode != AMOD_MODE_CHUNK && mode != AMOD_MODE_LOOPBACK)
    return fail(ctx, "invalid mode", AMOD_ERR_ARG);
  if (mode == AMOD_MODE_LOOPBACK) options |= AMOD_OPT_FORCE_EXACT; // diagnostics: exact kernel only
  if (nframes < 0) return fail(ctx, "nframes < 0", AMOD_ERR_ARG);
  if (nframes == 0) return AMOD_SUCCESS;
  if (payload_stride < 16 || payload_stride % 16) return fail(ctx, "payload_stride must be a positive multiple of 16", AMOD_ERR_ARG);
  if (reinterpret_cast<uintptr_t>(samples) & 15) return fail(ctx, "samples must be 16-byte aligned", AMOD_ERR_ARG);
  HIP_TRY(hipSetDevice(ctx->device));
  amod::DevCfg d;
  int rc = get_tables(ctx, cfg, d);
  if (rc) return rc;
  d.mode = mode;
  rc = reserve(ctx, cfg, nframes, max_len);
  if (rc) return rc;
  hipStream_t s = stream ? stream : ctx->stream;
  amod::DevWork w{};
  w.samples = samples; w.off = offsets; w.len = lengths; w.nframes = nframes;
  w.res = results; w.payload = payload; w.stride = payload_stride; w.dbg = debug;
  int32_t *const fb_base = (int32_t *)ctx->fb.p;
  int32_t *fb = fb_base; // this decode's counter set; lists from fb_base + 64
  // exact-kernel work lists: A (fb[0]) filled by detection, B (fb[1]) by k_demod;
  // list C (fb[2]): frames whose detection the exact kernel replayed, for k_demod
  w.fb_count = fb; w.fb_list = fb_base + 64; w.fb_flags = fb_base + 64 + nframes;
  w.fb_zero = fb + 1; // (k_detect / k_chunk_prep: the counts of list B and the replay list, the claim counter)
  w.xs = (float *)ctx->xs.p; w.bits = (uint32_t *)ctx->bits.p;
  w.xs_stride = ctx->xs_stride; w.bits_stride = ctx->bits_stride;
  w.options = options;
  if (amod::soft_combine_applies(options, cfg->repetition, cfg->modulation)) {
    const int64_t per = ((max_bits_for(cfg, std::max<int64_t>(ctx->max_len, max_len)) + 64) + 63) & ~int64_t(63);
    if (ctx->soft_stride < per || ctx->soft_slots < ctx->nslots) {
      HIP_TRY(ctx->soft.ensure(sizeof(float) * (size_t)(per * std::max(1, ctx->nslots))));
      ctx->soft_stride = per;
      ctx->soft_slots = ctx->nslots;
    }
    w.soft = (float *)ctx->soft.p;
    w.soft_stride = ctx->soft_stride;
  }
  // fast-path capacities from the longest frame of this launch (host path) or the latest
  // reservation (device path); a frame's route depends only on it and on the frame
  const ChainDims dims = chain_dims(cfg, max_len >= 0 ? max_len : ctx->dev_cap);
  rc = ensure_chain(ctx, nframes);
  if (rc) return rc;
  w.nb_cap = dims.nb_cap; w.fine_cap = dims.fine_cap; w.mcap = dims.mcap; w.fast_len = dims.fast_len;
  if (ctx->knobs.demod_mcap > 0) w.mcap = std::min(w.mcap, ctx->knobs.demod_mcap); // experiments
  amod_demod_stream_words(d, w.mcap, &w.stream_words, &w.vote_off);
  w.det = (amod::DetRec *)ctx->det.p;
  if (!ctx->cu_count) {
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, ctx->device));
    ctx->cu_count = prop.multiProcessorCount;
  }
  if (ctx->knobs.stamps) { // diagnostics: per-frame s_memtime marks of the fast kernel
    HIP_TRY(ctx->stamps.ensure(sizeof(unsigned long long) * 32 * (size_t)nframes));
    HIP_TRY(hipMemsetAsync(ctx->stamps.p, 0, sizeof(unsigned long long) * 32 * (size_t)nframes, s));
    w.stamps = (unsigned long long *)ctx->stamps.p;
    ctx->nstamps = nframes;
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) ctx->fb_captured = true;
  if (!ctx->fb_zeroed) HIP_TRY(hipMemsetAsync(fb_base, 0, 256, s)); // after a reallocation or an aborted decode
  ctx->fb_zeroed = false; // until this decode's list-B launch is enqueued with its reset
  ctx->detect_ev = false;
  std::array<hipEvent_t, 6> ev{};
  if (ctx->profiling) {
    if (ctx->ev_free.empty()) {
      for (auto &e : ev) HIP_TRY(hipEventCreate(&e));
    } else {
      ev = ctx->ev_free.back();
      ctx->ev_free.pop_back();
    }
  }
  auto mark = [&](int i, hipStream_t on = nullptr) -> hipError_t {
    return ctx->profiling ? hipEventRecord(ev[i], on ? on : s) : hipSuccess;
  };
  // d.stop_after (diagnostics, AMOD_STOP_AFTER): <= 2 stops after detection
  const bool demod = d.stop_after >= 3;
  const int lds = 4 * 4 * w.stream_words; // k_demod: 4 waves per block
  const int soft = amod::soft_fast(options, d) ? 1 : 0; // k_demod's soft-combining instance
  if (ctx->demod_lds != lds || ctx->demod_mod != d.mod || ctx->demod_nband != d.nband || ctx->demod_soft != soft) {
    ctx->demod_lds = lds; ctx->demod_mod = d.mod; ctx->demod_nband = d.nband; ctx->demod_soft = soft;
    ctx->demod_bpc = amod_demod_blocks_per_cu(d, lds, soft != 0);
  }
  int64_t per_cu = ctx->demod_bpc;
  if (ctx->knobs.demod_bpc > 0) per_cu = ctx->knobs.demod_bpc; // diagnostics: grid size
  auto demod_blocks = [&](int n) { return (int)std::min<int64_t>(((int64_t)n + 3) / 4, (int64_t)ctx->cu_count * per_cu); };
  // Frames in chunks over two streams: k_detect of chunk c + 1 (HBM-bound) runs on `s`
  // while k_demod of chunk c (latency-bound FFT jobs) runs on the context's second
  // stream, so the demodulation hides under the next chunk's stream pass.
  int nchunk = 1;
  if (demod && !debug && nframes >= 2048) nchunk = kOverlapChunks;
  if (ctx->knobs.chunks > 0) nchunk = std::min(kMaxChunks, ctx->knobs.chunks);
  if (!demod || debug) nchunk = 1;
  nchunk = std::min(nchunk, std::max(1, nframes));
  // this decode's timeline slot (profiling; one-chunk decodes with a k_demod launch): set by
  // k_detect, list A's replica and the main k_demod launch only
  unsigned long long *tl = nullptr;
  int64_t tl_slot = -1, tl_waves = 0;
  if (ctx->profiling && demod && !debug && nchunk == 1 && !ctx->knobs.exact_serial) {
    tl_waves = 4 * (int64_t)demod_blocks(nframes); // k_demod: 4 waves per workgroup
    if (amod::kTlHead + tl_waves > ctx->tl_words) { // a new layout: the marks kept so far are void
      ctx->tl_words = amod::kTlHead + std::max<int64_t>(tl_waves, 4 * 4 * (int64_t)std::max(1, ctx->cu_count));
      HIP_TRY(ctx->tl.ensure(sizeof(unsigned long long) * (size_t)(ctx->tl_words * kTlSlots)));
      for (auto &e : ctx->tl_of) e.first = -1;
    }
    tl_slot = ctx->tl_next++ % kTlSlots;
    tl = (unsigned long long *)ctx->tl.p + ctx->tl_words * tl_slot;
  }
  w.tl = tl;
  amod::DevWork wb = w; // every field as w, list B
  wb.tl = nullptr;
  wb.fb_zero = nullptr;
  wb.fb_count = fb + 1; wb.fb_list = fb_base + 64 + 2 * nframes; wb.fb_flags = fb_base + 64 + 3 * nframes;
  // exact-kernel grid: persistent workgroups over the listed frames (usually none: the
  // launch then costs its dispatch, so two per CU, not one per slot)
  int xslots = std::min({ctx->nslots, nframes, 2 * std::max(1, ctx->cu_count)});
  if (ctx->knobs.xslots > 0) xslots = std::min(xslots, ctx->knobs.xslots); // experiments
  // list A's exact kernel, then (detection replay) k_demod over the frames it only
  // detected: a frame listed for COARSE / FINE / THRESH alone gets its preambleIdx from
  // the fp64 replica and its symbols from the fast path (AMOD_NO_REPLAY: diagnostics)
  const bool replay = demod && !debug && mode == AMOD_MODE_RECEIVED && !ctx->knobs.no_replay;
  auto exact_a = [&](hipStream_t st) -> int {
    amod::DevWork wa = w;
    wa.f0 = 0; wa.f1 = nframes;
    if (replay) { wa.rp_count = fb + 2; wa.rp_list = fb_base + 64 + 4 * nframes; }
    HIP_TRY(amod_launch_exact(d, wa, xslots, st, true));
    if (replay) {
      amod::DevWork wc = wb; // its guards list into B
      wc.f0 = 0; wc.f1 = nframes;
      wc.dm_count = fb + 2; wc.dm_list = fb_base + 64 + 4 * nframes;
      HIP_TRY(amod_launch_demod(d, wc, std::min(demod_blocks(nframes), std::max(1, ctx->cu_count)), st));
    }
    return AMOD_SUCCESS;
  };
  HIP_TRY(mark(0));
  if (nchunk == 1) {
    w.f0 = 0; w.f1 = nframes;
    HIP_TRY(amod_launch_detect(d, w, s));
    if (ctx->knobs.mall_flush_mb > 0) { // (experiments: k_demod's window reads from a cold Infinity Cache)
      const size_t fb_bytes = (size_t)ctx->knobs.mall_flush_mb << 20;
      HIP_TRY(ctx->flush.ensure(fb_bytes + 256));
      HIP_TRY(amod_launch_flush(ctx->flush.p, fb_bytes, (float *)((char *)ctx->flush.p + fb_bytes), s));
    }
    HIP_TRY(mark(1));
    if (demod) {
      // list A is complete: the exact replica of the frames detection listed (long
      // sequential recurrences) runs on the second stream, under k_demod
      // (AMOD_EXACT_SERIAL, diagnostics: after it, on the same stream)
      // Chunk mode: list A holds only frames routed before any demodulation (FORCE_EXACT,
      // longer than the fast-path workspace, soft combining off the fast path), usually
      // none, so it runs after k_demod on the same stream: an empty list then costs one
      // dispatch instead of a launch parked on the aux stream for all of k_demod and the
      // join; a batch with such frames decodes them after the fast ones.
      if (ctx->knobs.exact_serial || mode == AMOD_MODE_CHUNK) {
        wb.f0 = 0; wb.f1 = nframes;
        amod::DevWork wm = wb;
        if (!ctx->knobs.exact_serial) {
          wm.tl = tl;
          wm.claim = ctx->knobs.demod_static ? nullptr : fb + 3;
          wm.claim_rounds = ctx->knobs.claim_rounds;
          wm.claim_min = ctx->knobs.claim_min;
        }
        HIP_TRY(amod_launch_demod(d, wm, demod_blocks(nframes), s));
        HIP_TRY(mark(2));
        rc = exact_a(s);
        if (rc) return rc;
        HIP_TRY(mark(3));
      } else {
      HIP_TRY(hipEventRecord(ctx->chunk_ev[0], s));
      ctx->detect_ev = cap == hipStreamCaptureStatusNone;
      HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->chunk_ev[0], 0));
      rc = exact_a(ctx->aux);
      if (rc) return rc;
      HIP_TRY(mark(3, ctx->aux));
      HIP_TRY(hipEventRecord(ctx->chunk_ev[kMaxChunks], ctx->aux));
      wb.f0 = 0; wb.f1 = nframes;
      {
        // the exact kernel needs a wave slot and its registers on every SIMD it runs on:
        // with frames listed, k_demod leaves one workgroup per CU free
        amod::DevWork wm = wb;
        wm.tl = tl;
        wm.claim = ctx->knobs.demod_static ? nullptr : fb + 3; // the dynamic tail (zeroed by k_detect)
        wm.claim_rounds = ctx->knobs.claim_rounds;
        wm.claim_min = ctx->knobs.claim_min;
        const int nb = demod_blocks(nframes);
        if (per_cu >= 2 && nb >= (int)(ctx->cu_count * per_cu)) {
          wm.yield_count = fb;
          wm.yield_blocks = (int)(ctx->cu_count * (per_cu - 1));
        }
        HIP_TRY(amod_launch_demod(d, wm, nb, s));
      }
      HIP_TRY(mark(2));
      HIP_TRY(hipStreamWaitEvent(s, ctx->chunk_ev[kMaxChunks], 0)); // workspace slots are shared
      }
    } else {
      HIP_TRY(amod_launch_exact(d, w, xslots, s));
      HIP_TRY(mark(2));
      HIP_TRY(mark(3));
    }
  } else {
    for (int c = 0; c < nchunk; ++c) {
      w.f0 = wb.f0 = (int)((int64_t)nframes * c / nchunk);
      w.fb_zero = c == 0 ? fb + 1 : nullptr; // (the first chunk only: k_demod of chunk c - 1 appends)
      w.f1 = wb.f1 = (int)((int64_t)nframes * (c + 1) / nchunk);
      HIP_TRY(amod_launch_detect(d, w, s));
      HIP_TRY(hipEventRecord(ctx->chunk_ev[c], s));
      HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->chunk_ev[c], 0));
      HIP_TRY(amod_launch_demod(d, wb, demod_blocks(w.f1 - w.f0), ctx->aux));
    }
    HIP_TRY(mark(1)); // every k_detect done (on s)
    HIP_TRY(hipEventRecord(ctx->chunk_ev[kMaxChunks], ctx->aux));
    HIP_TRY(hipStreamWaitEvent(s, ctx->chunk_ev[kMaxChunks], 0));
    HIP_TRY(mark(2)); // (chunked diagnostics: k_demod ends with the join)
    rc = exact_a(s);
    if (rc) return rc;
    HIP_TRY(mark(3));
  }
  w.f0 = wb.f0 = 0; w.f1 = wb.f1 = nframes;
  HIP_TRY(mark(4));
  wb.fb_reset = fb; // list A's count, zeroed for the next decode (or replay)
  HIP_TRY(amod_launch_exact(d, wb, xslots, s)); // list B: frames k_demod listed
  // a captured decode does not run here: its launches (the reset included) exist only in
  // the graph, so the next eager decode must zero the counters itself
  ctx->fb_zeroed = xslots > 0 && cap == hipStreamCaptureStatusNone;
  HIP_TRY(mark(5));
  if (ctx->profiling) {
    ctx->ev_used.push_back(ev);
    ctx->tl_of.emplace_back(tl_slot, tl_waves);
  }
  return AMOD_SUCCESS;
}

// ----------------------------------------------------------------- TX -----
// modulateOFDM (modem.js:322-362) of a bit vector; appends symbols to out
void modulate(const amod_cfg &c, const std::vector<uint8_t> &bits, std::vector<float> &out) {
  const int bps = bps_of(c.modulation), per_sym = amod_num_data_subs(&c) * bps;
  const size_t nsym = (bits.size() + per_sym - 1) / per_sym;
  const int n = amod::kFft;
  for (size_t s = 0; s < nsym; ++s) {
    double re[amod::kFft] = {0}, im[amod::kFft] = {0};
    int di = 0;
    for (int k = c.sub_start; k <= c.sub_end; ++k) {
      if (is_pilot(c, k)) { re[k] = 1; im[k] = 0; continue; }
      int idx = 0;
      for (int b = 0; b < bps; ++b) {
        const size_t pos = s * per_sym + (size_t)di * bps + b;
        idx = (idx << 1) | (pos < bits.size() ? (bits[pos] & 1) : 0);
      }
      constellation(c.modulation, idx % npoints(c.modulation), re[k], im[k]);
      ++di;
    }
    const size_t o = out.size();
    out.resize(o + c.symbol_len);
    (void)n;
    symbol_from_spectrum(c, re, im, true, out.data() + o);
  }
}

int64_t assemble_frame(const amod_cfg &c, const std::vector<uint8_t> &payload, int pre, int post, float *out) {
  std::vector<uint8_t> bits;
  bits.reserve(payload.size() * 8 * c.repetition);
  for (uint8_t byte : payload)
    for (int b = 7; b >= 0; --b)
      for (int r = 0; r < c.repetition; ++r) bits.push_back((byte >> b) & 1);
  const int bps = bps_of(c.modulation), per_sym = amod_num_data_subs(&c) * bps;
  const int64_t nsym = ((int64_t)bits.size() + per_sym - 1) / per_sym;
  const int64_t total = pre + (3 + nsym) * (int64_t)c.symbol_len + post;
  if (!out) return total;
  std::fill(out, out + total, 0.0f);
  template_symbol(c, 42.0, 2, out + pre, nullptr);
  template_symbol(c, 43.0, 1, out + pre + c.symbol_len, nullptr);
  template_symbol(c, 44.0, 1, out + pre + 2 * c.symbol_len, nullptr);
  std::vector<float> data;
  modulate(c, bits, data);
  std::copy(data.begin(), data.end(), out + pre + 3 * c.symbol_len);
  double mx = 0.0;
  for (int64_t i = 0; i < total; ++i) mx = std::max(mx, std::fabs((double)out[i]));
  if (mx > 0) {
    const double s = 0.8 / mx;
    for (int64_t i = 0; i < total; ++i) out[i] = (float)((double)out[i] * s);
  }
  return total;
}

void put_be32(std::vector<uint8_t> &p, int32_t v) {
  p.push_back((uint8_t)((v >> 24) & 0xFF)); p.push_back((uint8_t)((v >> 16) & 0xFF));
  p.push_back((uint8_t)((v >> 8) & 0xFF)); p.push_back((uint8_t)(v & 0xFF));
}

std::vector<uint8_t> legacy_packet(const uint8_t *data, int32_t len, const uint8_t *name, int32_t name_len) {
  name_len = std::min(name_len, 255);
  std::vector<uint8_t> p;
  p.reserve(1 + name_len + 8 + len);
  p.push_back((uint8_t)name_len);
  p.insert(p.end(), name, name + name_len);
  put_be32(p, len);
  p.insert(p.end(), data, data + len);
  put_be32(p, (int32_t)amod_crc32(p.data(), p.size()));
  return p;
}

// buildMetadataPayload (modem.js:666-692): [0xFE][chunks:4][size:4][chunkSize:2][nameLen:1][name][CRC:4]
std::vector<uint8_t> meta_packet(int32_t total_chunks, int32_t total_size, int32_t chunk_size, const uint8_t *name,
                                 int32_t name_len) {
  name_len = std::min(name_len, 255);
  std::vector<uint8_t> p = {0xFE};
  put_be32(p, total_chunks);
  put_be32(p, total_size);
  p.push_back((uint8_t)((chunk_size >> 8) & 0xFF));
  p.push_back((uint8_t)(chunk_size & 0xFF));
  p.push_back((uint8_t)name_len);
  p.insert(p.end(), name, name + name_len);
  put_be32(p, (int32_t)amod_crc32(p.data(), p.size()));
  return p;
}

// buildDataChunkPayload (modem.js:694-714): [0xFF][seq:4][dataLen:2][data][CRC:4]
std::vector<uint8_t> chunk_packet(const uint8_t *data, int32_t len, int32_t seq) {
  std::vector<uint8_t> p = {0xFF};
  put_be32(p, seq);
  p.push_back((uint8_t)((len >> 8) & 0xFF));
  p.push_back((uint8_t)(len & 0xFF));
  p.insert(p.end(), data, data + len);
  put_be32(p, (int32_t)amod_crc32(p.data(), p.size()));
  return p;
}

int silence_len(const amod_cfg &c, double seconds_std, double seconds_ac) {
  return (int)((double)c.sample_rate * (c.cp_len >= 128 ? seconds_ac : seconds_std));
}
int rounded_silence(const amod_cfg &c, double seconds) {
  return (int)std::floor((double)c.sample_rate * seconds + 0.5);
}

} // namespace

// =============================================================== C ABI =====
extern "C" {

int amod_abi_version(void) { return AMOD_ABI_VERSION; }

int amod_close(amod_ctx *ctx);
const amod::Knobs *amod_ctx_knobs(const amod_ctx *ctx) { return ctx ? &ctx->knobs : nullptr; }
hipEvent_t amod_ctx_detect_event(const amod_ctx *ctx) { return ctx && ctx->detect_ev ? ctx->chunk_ev[0] : nullptr; }

int amod_ctx_device(const amod_ctx *ctx) { return ctx ? ctx->device : 0; }
hipStream_t amod_ctx_stream(const amod_ctx *ctx) { return ctx ? ctx->stream : nullptr; }
int amod_ctx_fail(amod_ctx *ctx, const char *msg, int code) { return fail(ctx, msg, code); }
void **amod_ctx_ext(amod_ctx *ctx, int slot, void (*free_fn)(void *)) {
  if (!ctx || slot < 0 || slot >= 4) return nullptr;
  if (free_fn) ctx->ext_free[slot] = free_fn;
  return &ctx->ext[slot];
}
int amod_cfg_valid(const amod_cfg *cfg) { return validate(cfg); }

int amod_open(int device, amod_ctx **out) {
  if (!out) return fail(nullptr, "null out", AMOD_ERR_ARG);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(nullptr, "no HIP device", AMOD_ERR_NODEV);
  if (device < 0 || device >= n) return fail(nullptr, "device index out of range", AMOD_ERR_NODEV);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(nullptr, std::string("device is ") + prop.gcnArchName + ", libamodem is built for gfx950", AMOD_ERR_NODEV);
  HIP_TRY(hipSetDevice(device));
  auto *ctx = new amod_ctx();
  ctx->device = device;
  for (DevBuf *b : {&ctx->fb, &ctx->xs, &ctx->bits, &ctx->soft, &ctx->det}) {
    b->keep = &ctx->fb_captured;
    b->retired = &ctx->retired;
  }
  read_knobs(ctx->knobs);
  // The second stream, created here at the device's highest priority: it then draws its
  // hardware queue from the high-priority pool, never the caller's stream's queue, so
  // list A's replica (enqueued on it before k_demod) runs beside k_demod instead of
  // ahead of it on a shared queue (a lazily created default-
  // priority stream landed on the caller's queue in one of GPU_MAX_HW_QUEUES' rotations)
  int prio_least = 0, prio_greatest = 0;
  bool ok = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) == hipSuccess &&
            hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) == hipSuccess &&
            hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking,
                                        ctx->knobs.aux_priority ? prio_greatest : prio_least) == hipSuccess;
  for (auto &e : ctx->chunk_ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    amod_close(ctx);
    return fail(nullptr, "hipStreamCreate / hipEventCreate failed", AMOD_ERR_HIP);
  }
  *out = ctx;
  return AMOD_SUCCESS;
}

int amod_close(amod_ctx *ctx) {
  if (!ctx) return AMOD_SUCCESS;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
  }
  if (ctx->aux) (void)hipStreamSynchronize(ctx->aux);
  for (int i = 0; i < 4; ++i)
    if (ctx->ext[i] && ctx->ext_free[i]) ctx->ext_free[i](ctx->ext[i]);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  for (auto &e : ctx->chunk_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &ev : ctx->ev_used) for (auto &e : ev) (void)hipEventDestroy(e);
  if (ctx->up) {
    (void)hipStreamSynchronize(ctx->up);
    (void)hipStreamDestroy(ctx->up);
  }
  for (hipEvent_t e : ctx->up_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->dn_ev) (void)hipEventDestroy(e);
  for (void *p : ctx->retired) (void)hipFree(p);
  for (auto &ev : ctx->ev_free) for (auto &e : ev) (void)hipEventDestroy(e);
  delete ctx;
  return AMOD_SUCCESS;
}

const char *amod_last_error(const amod_ctx *ctx) {
  if (ctx && !ctx->err.empty()) return ctx->err.c_str();
  return g_last_error.c_str();
}

int amod_config_preset(const char *name, int32_t modulation, int32_t repetition, amod_cfg *out) {
  if (!out) return fail(nullptr, "null out", AMOD_ERR_ARG);
  if (modulation < AMOD_BPSK || modulation > AMOD_QAM16) return fail(nullptr, "bad modulation", AMOD_ERR_ARG);
  std::memset(out, 0, sizeof *out);
  static const int std_p[] = {15, 29, 43, 57, 71, 85, 99, 113, 127, 141, 155, 169, 183, 197, 211, 225};
  static const int ac_p[] = {25, 35, 45, 55, 65, 75, 85};
  static const int nb_p[] = {37, 45, 53};
  const int *p = std_p;
  int np = 16;
  out->fft_size = 512;
  out->sample_rate = 44100;
  const std::string n = name ? name : "";
  if (n == "acoustic") { out->cp_len = 128; out->sub_start = 23; out->sub_end = 93; p = ac_p; np = 7; }
  else if (n == "narrowband") { out->cp_len = 256; out->sub_start = 35; out->sub_end = 58; p = nb_p; np = 3; }
  else { out->cp_len = 64; out->sub_start = 12; out->sub_end = 232; }
  out->symbol_len = out->fft_size + out->cp_len;
  out->npilots = np;
  for (int i = 0; i < np; ++i) out->pilots[i] = p[i];
  out->modulation = modulation;
  out->repetition = repetition < 1 ? 1 : repetition;
  return AMOD_SUCCESS;
}

int32_t amod_num_data_subs(const amod_cfg *c) {
  if (!c) return 0;
  int32_t n = 0;
  for (int k = c->sub_start; k <= c->sub_end; ++k) n += !is_pilot(*c, k);
  return n;
}

int32_t amod_estimate_frame_samples(const amod_cfg *c, int32_t payload_bytes) {
  if (!c) return 0;
  const double per_sym = (double)amod_num_data_subs(c) * bps_of(c->modulation);
  const double total = (double)payload_bytes * 8.0 * (double)std::max(1, c->repetition);
  return (3 + (int32_t)std::ceil(total / per_sym)) * c->symbol_len;
}

int64_t amod_payload_stride(const amod_cfg *c, int64_t max_len) {
  if (!c || max_len < 0) return 16;
  const int64_t bytes = max_bits_for(c, max_len) / 8 + 16;
  return (bytes + 15) & ~int64_t(15);
}

int amod_reserve(amod_ctx *ctx, const amod_cfg *cfg, int32_t nframes, int64_t max_len) {
  if (!ctx || !validate(cfg)) return fail(ctx, "invalid argument", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  amod::DevCfg d;
  int rc = get_tables(ctx, cfg, d);
  if (rc) return rc;
  if (max_len >= 0) ctx->dev_cap = max_len; // the device path's fast-path capacity from now on
  return reserve(ctx, cfg, nframes, max_len);
}

int amod_decode_device(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                       const int64_t *offsets, const int32_t *lengths, int32_t nframes, amod_result *results,
                       uint8_t *payload, int64_t payload_stride, uint32_t options, void *stream) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  return decode_impl(ctx, cfg, mode, samples, offsets, lengths, nframes, results, payload, payload_stride, options,
                     (hipStream_t)stream, nullptr, -1);
}

int amod_decode_device_debug(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                             const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                             amod_result *results, uint8_t *payload, int64_t payload_stride, uint32_t options,
                             void *stream, amod_debug *debug) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  return decode_impl(ctx, cfg, mode, samples, offsets, lengths, nframes, results, payload, payload_stride, options,
                     (hipStream_t)stream, debug, -1);
}

namespace {
int decode_host_impl(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples, int64_t nsamples,
                     const int64_t *offsets, const int32_t *lengths, int32_t nframes, amod_result *results,
                     uint8_t *payload, int64_t payload_stride, uint32_t options, amod_progress_fn progress,
                     void *user) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  if (nframes < 0 || nsamples < 0) return fail(ctx, "negative size", AMOD_ERR_ARG);
  for (int32_t i = 0; i < nframes; ++i)
    if (offsets[i] < 0 || lengths[i] < 0 || offsets[i] + lengths[i] > nsamples)
      return fail(ctx, "frame " + std::to_string(i) + " lies outside the sample buffer", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (nframes == 0) return AMOD_SUCCESS;
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(ctx->h_samples.ensure(sizeof(float) * (size_t)(nsamples + 4)));
  HIP_TRY(ctx->h_off.ensure(sizeof(int64_t) * (size_t)nframes));
  HIP_TRY(ctx->h_len.ensure(sizeof(int32_t) * (size_t)nframes));
  HIP_TRY(ctx->h_res.ensure(sizeof(amod_result) * (size_t)nframes));
  HIP_TRY(ctx->h_payload.ensure((size_t)payload_stride * (size_t)nframes));
  hipStream_t s = ctx->stream;
  if (!ctx->up) HIP_TRY(hipStreamCreateWithFlags(&ctx->up, hipStreamNonBlocking));
  HIP_TRY(hipMemcpyAsync(ctx->h_off.p, offsets, sizeof(int64_t) * nframes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(ctx->h_len.p, lengths, sizeof(int32_t) * nframes, hipMemcpyHostToDevice, s));
  // the fast kernel writes only the decoded prefix of each slot: hand back zeros past it
  HIP_TRY(hipMemsetAsync(ctx->h_payload.p, 0, (size_t)payload_stride * (size_t)nframes, s));
  // The samples go up in pieces on the upload stream while the context stream decodes the
  // frames whose samples have all landed: frames in index order, when their ends never
  // decrease (a batch cut from one recording), else every frame after the last piece. A
  // pageable copy returns once its piece is staged, so the decodes enqueued after it run
  // on the GPU during the next piece's upload.
  bool mono = true;
  for (int32_t i = 1; i < nframes && mono; ++i) mono = offsets[i] + lengths[i] >= offsets[i - 1] + lengths[i - 1];
  int64_t piece = kUpPiece;
  if (ctx->knobs.up_piece > 0) piece = std::max<int64_t>(1024, ctx->knobs.up_piece); // tests: many pieces
  const int64_t npiece = (nsamples + piece - 1) / piece;
  while ((int64_t)ctx->up_ev.size() < std::max<int64_t>(npiece, 1)) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->up_ev.push_back(e);
  }
  HIP_TRY(hipEventRecord(ctx->up_ev[0], s)); // the upload stream starts after the memset's stream order
  HIP_TRY(hipStreamWaitEvent(ctx->up, ctx->up_ev[0], 0));
  // one workspace reservation and one fast-path capacity for the whole call (its longest
  // frame): every piece's launch routes its frames as a one-piece call would, and no
  // piece's reservation grows a buffer (hipFree would synchronise the upload pipeline)
  int64_t call_max = 0;
  for (int32_t i = 0; i < nframes; ++i) call_max = std::max<int64_t>(call_max, lengths[i]);
  {
    amod::DevCfg d;
    int rc = get_tables(ctx, cfg, d);
    if (rc == AMOD_SUCCESS) rc = reserve(ctx, cfg, nframes, call_max);
    if (rc) {
      (void)hipStreamSynchronize(ctx->up);
      return rc;
    }
  }
  if (!progress && (npiece <= 1 || !mono)) {
    // one launch and nobody to tell about prefixes: the samples go up, one decode, the
    // records and payload rows straight back into the caller's buffers (no helper thread,
    // no pinned mirrors)
    for (int64_t p = 0; p < npiece; ++p) {
      const int64_t lo = p * piece, n = std::min(piece, nsamples - lo);
      HIP_TRY(hipMemcpyAsync((float *)ctx->h_samples.p + lo, samples + lo, sizeof(float) * n, hipMemcpyHostToDevice,
                             ctx->up));
    }
    HIP_TRY(hipEventRecord(ctx->up_ev[0], ctx->up));
    HIP_TRY(hipStreamWaitEvent(s, ctx->up_ev[0], 0));
    const int rc = decode_impl(ctx, cfg, mode, (const float *)ctx->h_samples.p, (const int64_t *)ctx->h_off.p,
                               (const int32_t *)ctx->h_len.p, nframes, (amod_result *)ctx->h_res.p,
                               (uint8_t *)ctx->h_payload.p, payload_stride, options, s, nullptr, call_max);
    if (rc) {
      (void)hipStreamSynchronize(ctx->up);
      (void)hipStreamSynchronize(s);
      return rc;
    }
    HIP_TRY(hipMemcpyAsync(results, ctx->h_res.p, sizeof(amod_result) * (size_t)nframes, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(payload, ctx->h_payload.p, (size_t)payload_stride * (size_t)nframes,
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return AMOD_SUCCESS;
  }
  HIP_TRY(ctx->pin_res.ensure(sizeof(amod_result) * (size_t)nframes));
  HIP_TRY(ctx->pin_payload.ensure((size_t)payload_stride * (size_t)nframes));
  // every launch's frames [a, b) come back on the context stream right after it (DMA into
  // the pinned mirrors); a helper thread waits for each piece's copy, moves it into the
  // caller's buffers and reports it, so the calling thread keeps staging the uploads (the
  // copies into fresh pageable memory fault page by page: on the calling thread they
  // delayed the next pieces' uploads)
  struct Back { hipEvent_t ev; int32_t a, b; };
  std::mutex bmu;
  std::condition_variable bcv;
  std::vector<Back> back;
  bool bclosed = false;
  hipError_t berr = hipSuccess;
  std::thread deliverer([&] {
    (void)hipSetDevice(ctx->device);
    for (size_t i = 0;; ++i) {
      Back k;
      {
        std::unique_lock<std::mutex> lk(bmu);
        bcv.wait(lk, [&] { return bclosed || i < back.size(); });
        if (i >= back.size()) return;
        k = back[i];
      }
      const hipError_t e = hipEventSynchronize(k.ev);
      if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(bmu);
        berr = e;
        return;
      }
      std::memcpy(results + k.a, (const amod_result *)ctx->pin_res.p + k.a, sizeof(amod_result) * (size_t)(k.b - k.a));
      std::memcpy(payload + (int64_t)k.a * payload_stride,
                  (const uint8_t *)ctx->pin_payload.p + (int64_t)k.a * payload_stride,
                  (size_t)payload_stride * (size_t)(k.b - k.a));
      if (progress) progress(user, k.b);
    }
  });
  auto finish = [&](bool drain) -> hipError_t { // stop the helper (after the queued pieces when drain)
    if (!deliverer.joinable()) return berr;
    {
      std::lock_guard<std::mutex> lk(bmu);
      if (!drain) back.resize(0);
      bclosed = true;
    }
    bcv.notify_one();
    deliverer.join();
    return berr;
  };
  struct Joiner { // every return stops the helper first, then waits out the streams (an
                  // upload or a copy into the pinned mirrors may still be in flight after an
                  // early return through HIP_TRY; the next call reuses those buffers)
    std::function<void()> f;
    ~Joiner() { f(); }
  } joiner{[&] {
    (void)finish(false);
    (void)hipStreamSynchronize(ctx->up);
    (void)hipStreamSynchronize(s);
  }};
  int32_t a = 0; // the first frame not yet enqueued
  for (int64_t p = 0; p <= npiece; ++p) {
    int64_t covered = nsamples;
    if (p < npiece) {
      const int64_t lo = p * piece, n = std::min(piece, nsamples - lo);
      HIP_TRY(hipMemcpyAsync((float *)ctx->h_samples.p + lo, samples + lo, sizeof(float) * n, hipMemcpyHostToDevice,
                             ctx->up));
      HIP_TRY(hipEventRecord(ctx->up_ev[p], ctx->up));
      HIP_TRY(hipStreamWaitEvent(s, ctx->up_ev[p], 0));
      covered = lo + n;
      if (!mono && p + 1 < npiece) continue;
    }
    int32_t b = a;
    while (b < nframes && (p == npiece || offsets[b] + lengths[b] <= covered)) ++b;
    if (b == a) continue;
    const int rc = decode_impl(ctx, cfg, mode, (const float *)ctx->h_samples.p, (const int64_t *)ctx->h_off.p + a,
                               (const int32_t *)ctx->h_len.p + a, b - a, (amod_result *)ctx->h_res.p + a,
                               (uint8_t *)ctx->h_payload.p + (int64_t)a * payload_stride, payload_stride, options, s,
                               nullptr, call_max);
    hipError_t e = rc ? hipSuccess : hipErrorUnknown;
    if (!rc) {
      const size_t nb = back.size(); // (only this thread appends)
      if (nb == ctx->dn_ev.size()) {
        hipEvent_t ev;
        e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e == hipSuccess) ctx->dn_ev.push_back(ev);
      } else {
        e = hipSuccess;
      }
      if (e == hipSuccess)
        e = hipMemcpyAsync((amod_result *)ctx->pin_res.p + a, (const amod_result *)ctx->h_res.p + a,
                           sizeof(amod_result) * (size_t)(b - a), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess)
        e = hipMemcpyAsync((uint8_t *)ctx->pin_payload.p + (int64_t)a * payload_stride,
                           (const uint8_t *)ctx->h_payload.p + (int64_t)a * payload_stride,
                           (size_t)payload_stride * (size_t)(b - a), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipEventRecord(ctx->dn_ev[nb], s);
      if (e == hipSuccess) {
        {
          std::lock_guard<std::mutex> lk(bmu);
          back.push_back(Back{ctx->dn_ev[nb], a, b});
        }
        bcv.notify_one();
      }
    }
    if (rc) return rc; // (the joiner stops the helper and drains both streams)
    HIP_TRY(e);
    a = b;
  }
  HIP_TRY(finish(true));
  return AMOD_SUCCESS;
}
} // namespace

int amod_decode_host(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples, int64_t nsamples,
                     const int64_t *offsets, const int32_t *lengths, int32_t nframes, amod_result *results,
                     uint8_t *payload, int64_t payload_stride, uint32_t options) {
  return decode_host_impl(ctx, cfg, mode, samples, nsamples, offsets, lengths, nframes, results, payload,
                          payload_stride, options, nullptr, nullptr);
}

int amod_decode_host_progress(amod_ctx *ctx, const amod_cfg *cfg, int32_t mode, const float *samples,
                              int64_t nsamples, const int64_t *offsets, const int32_t *lengths, int32_t nframes,
                              amod_result *results, uint8_t *payload, int64_t payload_stride, uint32_t options,
                              amod_progress_fn progress, void *user) {
  return decode_host_impl(ctx, cfg, mode, samples, nsamples, offsets, lengths, nframes, results, payload,
                          payload_stride, options, progress, user);
}

int amod_synchronize(amod_ctx *ctx) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return AMOD_SUCCESS;
}

int amod_set_profiling(amod_ctx *ctx, int enable) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->profiling = enable != 0;
  return AMOD_SUCCESS;
}

int amod_kernel_stages(amod_ctx *ctx, double *ms, int32_t nslots, int64_t *n) {
  if (!ctx || nslots < 0 || (nslots && !ms)) return fail(ctx, "invalid argument", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  // the slots: {from event, to event} (amod.h AMOD_STAGE_*)
  static const int span[AMOD_STAGE_COUNT][2] = {{0, 1}, {1, 2}, {4, 5}, {1, 3}, {2, 4}, {1, 4}};
  double acc[AMOD_STAGE_COUNT] = {0};
  // the timeline marks of the (at most kTlSlots) latest profiled decodes
  std::vector<unsigned long long> tlh;
  if (ctx->tl.p && !ctx->ev_used.empty()) {
    HIP_TRY(hipEventSynchronize(ctx->ev_used.back()[5]));
    tlh.resize((size_t)(ctx->tl_words * kTlSlots));
    HIP_TRY(hipMemcpy(tlh.data(), ctx->tl.p, sizeof(unsigned long long) * tlh.size(), hipMemcpyDeviceToHost));
    const size_t n = ctx->tl_of.size(), from = n > (size_t)kTlSlots ? n - kTlSlots : 0;
    for (size_t i = from; i < n; ++i) {
      const int64_t sl = ctx->tl_of[i].first, nw = ctx->tl_of[i].second;
      if (sl < 0) continue;
      const unsigned long long *m = tlh.data() + ctx->tl_words * sl;
      const unsigned long long a_start = m[0];
      unsigned long long d_end = 0;
      for (int64_t q = 0; q < nw; ++q) d_end = std::max(d_end, m[amod::kTlHead + q]);
      if (a_start == ~0ull || d_end == 0) continue; // list A took no frame / no k_demod wave ran
      ctx->ov_listed += 1;
      const double lead = ((double)(long long)(d_end - a_start)) / 100.0; // 100 MHz real-time clock
      ctx->ov_beside += a_start < d_end;
      ctx->ov_lead_us += lead;
    }
  }
  ctx->tl_of.clear();
  for (auto &ev : ctx->ev_used) {
    HIP_TRY(hipEventSynchronize(ev[5]));
    for (int i = 0; i < AMOD_STAGE_COUNT; ++i) {
      float t = 0;
      HIP_TRY(hipEventElapsedTime(&t, ev[span[i][0]], ev[span[i][1]]));
      acc[i] += t;
    }
    ctx->ev_free.push_back(ev);
  }
  for (int i = 0; i < nslots; ++i) ms[i] = i < AMOD_STAGE_COUNT ? acc[i] : 0.0;
  if (n) *n = (int64_t)ctx->ev_used.size();
  ctx->ev_used.clear();
  return AMOD_SUCCESS;
}

int amod_aux_overlap(amod_ctx *ctx, int64_t *listed, int64_t *beside, double *lead_us) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (listed) *listed = ctx->ov_listed;
  if (beside) *beside = ctx->ov_beside;
  if (lead_us) *lead_us = ctx->ov_lead_us;
  ctx->ov_listed = ctx->ov_beside = 0;
  ctx->ov_lead_us = 0.0;
  return AMOD_SUCCESS;
}

int amod_kernel_breakdown(amod_ctx *ctx, double *ms, int64_t *n) {
  double st[AMOD_STAGE_COUNT];
  const int rc = amod_kernel_stages(ctx, st, AMOD_STAGE_COUNT, n);
  if (rc) return rc;
  if (ms) { ms[0] = st[AMOD_STAGE_DETECT]; ms[1] = st[AMOD_STAGE_DEMOD_PATH]; ms[2] = st[AMOD_STAGE_EXACT_B]; }
  return AMOD_SUCCESS;
}

int amod_kernel_times(amod_ctx *ctx, double *fast_ms, int64_t *fast_n, double *exact_ms, int64_t *exact_n) {
  double ms[3];
  int64_t n = 0;
  const int rc = amod_kernel_breakdown(ctx, ms, &n);
  if (rc) return rc;
  if (fast_ms) *fast_ms = ms[0] + ms[1];
  if (exact_ms) *exact_ms = ms[2];
  if (fast_n) *fast_n = n;
  if (exact_n) *exact_n = n;
  return AMOD_SUCCESS;
}

int amod_analyze_loopback(amod_ctx *ctx, const amod_cfg *cfg, const float *samples, int64_t nsamples,
                          amod_result *res, amod_debug *dbg, uint8_t *bytes, int64_t cap) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  if (!res || !dbg || nsamples < 0 || nsamples > INT32_MAX || (nsamples && !samples) || cap < 0 || (cap && !bytes))
    return fail(ctx, "invalid argument", AMOD_ERR_ARG);
  if (!validate(cfg)) return fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  const int64_t stride = amod_payload_stride(cfg, nsamples);
  HIP_TRY(ctx->h_samples.ensure(sizeof(float) * (size_t)(nsamples + 4)));
  HIP_TRY(ctx->h_off.ensure(sizeof(int64_t)));
  HIP_TRY(ctx->h_len.ensure(sizeof(int32_t)));
  HIP_TRY(ctx->h_res.ensure(sizeof(amod_result)));
  HIP_TRY(ctx->h_payload.ensure((size_t)stride));
  HIP_TRY(ctx->h_dbg.ensure(sizeof(amod_debug)));
  hipStream_t s = ctx->stream;
  const int64_t off0 = 0;
  const int32_t len0 = (int32_t)nsamples;
  if (nsamples) HIP_TRY(hipMemcpyAsync(ctx->h_samples.p, samples, sizeof(float) * nsamples, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(ctx->h_off.p, &off0, sizeof off0, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(ctx->h_len.p, &len0, sizeof len0, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(ctx->h_dbg.p, 0, sizeof(amod_debug), s));
  HIP_TRY(hipMemsetAsync(ctx->h_payload.p, 0, (size_t)stride, s));
  int rc = decode_impl(ctx, cfg, AMOD_MODE_LOOPBACK, (const float *)ctx->h_samples.p, (const int64_t *)ctx->h_off.p,
                       (const int32_t *)ctx->h_len.p, 1, (amod_result *)ctx->h_res.p, (uint8_t *)ctx->h_payload.p,
                       stride, 0, s, (amod_debug *)ctx->h_dbg.p, nsamples);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(res, ctx->h_res.p, sizeof(amod_result), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(dbg, ctx->h_dbg.p, sizeof(amod_debug), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const int64_t nb = std::min<int64_t>(std::max<int32_t>(res->nbytes, 0), std::min<int64_t>(cap, stride));
  if (nb > 0) HIP_TRY(hipMemcpy(bytes, ctx->h_payload.p, (size_t)nb, hipMemcpyDeviceToHost));
  return AMOD_SUCCESS;
}

int64_t amod_debug_stamps(amod_ctx *ctx, uint64_t *out, int64_t cap) {
  if (!ctx || !ctx->stamps.p) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  const int64_t n = std::min<int64_t>(cap, 32 * ctx->nstamps);
  if (hipMemcpy(out, ctx->stamps.p, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return n;
}

uint32_t amod_crc32(const uint8_t *d, size_t n) {
  const uint32_t *t = crc_table();
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = t[(c ^ d[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

int amod_preamble1(const amod_cfg *cfg, float *out) {
  if (!validate(cfg) || !out) return fail(nullptr, "invalid argument", AMOD_ERR_ARG);
  template_symbol(*cfg, 42.0, 2, out, nullptr);
  return AMOD_SUCCESS;
}

int64_t amod_tx_legacy(const amod_cfg *cfg, const uint8_t *data, int32_t len, const uint8_t *name, int32_t name_len,
                       float *out) {
  if (!validate(cfg) || len < 0 || name_len < 0) return AMOD_ERR_ARG;
  const auto p = legacy_packet(data, len, name, name_len);
  return assemble_frame(*cfg, p, silence_len(*cfg, 0.3, 0.5), silence_len(*cfg, 0.2, 0.5), out);
}

int64_t amod_tx_meta(const amod_cfg *cfg, int32_t total_chunks, int32_t total_size, int32_t chunk_size,
                     const uint8_t *name, int32_t name_len, float *out) {
  if (!validate(cfg) || name_len < 0) return AMOD_ERR_ARG;
  const auto p = meta_packet(total_chunks, total_size, chunk_size, name, name_len);
  int32_t pre, post;
  amod_tx_silence(cfg, AMOD_TX_META, &pre, &post);
  return assemble_frame(*cfg, p, pre, post, out);
}

int64_t amod_tx_chunk(const amod_cfg *cfg, const uint8_t *data, int32_t len, int32_t seq, float *out) {
  if (!validate(cfg) || len < 0) return AMOD_ERR_ARG;
  const auto p = chunk_packet(data, len, seq);
  int32_t pre, post;
  amod_tx_silence(cfg, AMOD_TX_CHUNK, &pre, &post);
  return assemble_frame(*cfg, p, pre, post, out);
}

int amod_tx_silence(const amod_cfg *cfg, int32_t kind, int32_t *pre, int32_t *post) {
  if (!validate(cfg) || !pre || !post) return AMOD_ERR_ARG;
  switch (kind) {
  case AMOD_TX_LEGACY: *pre = silence_len(*cfg, 0.3, 0.5); *post = silence_len(*cfg, 0.2, 0.5); break;
  case AMOD_TX_META: *pre = rounded_silence(*cfg, cfg->cp_len >= 128 ? 0.5 : 0.3); *post = rounded_silence(*cfg, 0.02); break;
  case AMOD_TX_CHUNK: *pre = rounded_silence(*cfg, 0.05); *post = rounded_silence(*cfg, 0.02); break;
  default: return AMOD_ERR_ARG;
  }
  return AMOD_SUCCESS;
}

int64_t amod_packet_legacy(const uint8_t *data, int32_t len, const uint8_t *name, int32_t name_len, uint8_t *out) {
  if (len < 0 || name_len < 0) return AMOD_ERR_ARG;
  const auto p = legacy_packet(data, len, name, name_len);
  if (out) std::copy(p.begin(), p.end(), out);
  return (int64_t)p.size();
}

int64_t amod_packet_meta(int32_t total_chunks, int32_t total_size, int32_t chunk_size, const uint8_t *name,
                         int32_t name_len, uint8_t *out) {
  if (name_len < 0) return AMOD_ERR_ARG;
  const auto p = meta_packet(total_chunks, total_size, chunk_size, name, name_len);
  if (out) std::copy(p.begin(), p.end(), out);
  return (int64_t)p.size();
}

int64_t amod_packet_chunk(const uint8_t *data, int32_t len, int32_t seq, uint8_t *out) {
  if (len < 0) return AMOD_ERR_ARG;
  const auto p = chunk_packet(data, len, seq);
  if (out) std::copy(p.begin(), p.end(), out);
  return (int64_t)p.size();
}

int64_t amod_tx_frame_samples(const amod_cfg *cfg, int64_t pkt_len, int32_t pre, int32_t post) {
  if (!validate(cfg) || pkt_len < 0 || pre < 0 || post < 0) return AMOD_ERR_ARG;
  const int64_t per_sym = (int64_t)amod_num_data_subs(cfg) * bps_of(cfg->modulation);
  const int64_t nsym = (pkt_len * 8 * cfg->repetition + per_sym - 1) / per_sym;
  return pre + (3 + nsym) * (int64_t)cfg->symbol_len + post;
}

int amod_tx_device(amod_ctx *ctx, const amod_cfg *cfg, const uint8_t *packets, const int64_t *pkt_off,
                   const int32_t *pkt_len, const int32_t *pre, const int32_t *post, int32_t nframes, float *out,
                   const int64_t *out_off, void *stream) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  if (!validate(cfg)) return fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  if (nframes < 0) return fail(ctx, "nframes < 0", AMOD_ERR_ARG);
  if (nframes == 0) return AMOD_SUCCESS;
  if (!packets || !pkt_off || !pkt_len || !pre || !post || !out || !out_off)
    return fail(ctx, "null device pointer", AMOD_ERR_ARG);
  HIP_TRY(hipSetDevice(ctx->device));
  amod::DevCfg d;
  const int rc = get_tables(ctx, cfg, d);
  if (rc) return rc;
  amod::DevTxWork w{packets, pkt_off, pkt_len, pre, post, out, out_off, nframes};
  HIP_TRY(amod_launch_tx(d, w, stream ? (hipStream_t)stream : ctx->stream));
  return AMOD_SUCCESS;
}

int64_t amod_tx_host(amod_ctx *ctx, const amod_cfg *cfg, const uint8_t *packets, int64_t nbytes,
                     const int64_t *pkt_off, const int32_t *pkt_len, const int32_t *pre, const int32_t *post,
                     int32_t nframes, float *out, int64_t *out_off) {
  if (!ctx) return fail(nullptr, "null context", AMOD_ERR_ARG);
  if (!validate(cfg)) return fail(ctx, "invalid amod_cfg", AMOD_ERR_ARG);
  if (nframes < 0 || nbytes < 0) return fail(ctx, "negative size", AMOD_ERR_ARG);
  std::vector<int64_t> oo(nframes);
  int64_t total = 0;
  for (int32_t i = 0; i < nframes; ++i) {
    if (pkt_off[i] < 0 || pkt_len[i] < 0 || pkt_off[i] + pkt_len[i] > nbytes)
      return fail(ctx, "packet " + std::to_string(i) + " lies outside the packet buffer", AMOD_ERR_ARG);
    const int64_t n = amod_tx_frame_samples(cfg, pkt_len[i], pre[i], post[i]);
    if (n < 0) return fail(ctx, "invalid silence length", AMOD_ERR_ARG);
    oo[i] = total;
    total += n;
  }
  if (!out) return total;
  if (out_off) std::copy(oo.begin(), oo.end(), out_off);
  if (nframes == 0) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(ctx->tx_pkt.ensure((size_t)std::max<int64_t>(nbytes, 1)));
  HIP_TRY(ctx->tx_meta.ensure((size_t)nframes * (2 * sizeof(int64_t) + 3 * sizeof(int32_t))));
  HIP_TRY(ctx->tx_out.ensure(sizeof(float) * (size_t)total));
  int64_t *d_po = (int64_t *)ctx->tx_meta.p, *d_oo = d_po + nframes;
  int32_t *d_pl = (int32_t *)(d_oo + nframes), *d_pre = d_pl + nframes, *d_post = d_pre + nframes;
  hipStream_t s = ctx->stream;
  if (nbytes) HIP_TRY(hipMemcpyAsync(ctx->tx_pkt.p, packets, (size_t)nbytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_po, pkt_off, sizeof(int64_t) * nframes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_oo, oo.data(), sizeof(int64_t) * nframes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_pl, pkt_len, sizeof(int32_t) * nframes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_pre, pre, sizeof(int32_t) * nframes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d_post, post, sizeof(int32_t) * nframes, hipMemcpyHostToDevice, s));
  amod::DevCfg d;
  const int rc = get_tables(ctx, cfg, d);
  if (rc) return rc;
  amod::DevTxWork w{(const uint8_t *)ctx->tx_pkt.p, d_po, d_pl, d_pre, d_post, (float *)ctx->tx_out.p, d_oo, nframes};
  HIP_TRY(amod_launch_tx(d, w, s));
  HIP_TRY(hipMemcpyAsync(out, ctx->tx_out.p, sizeof(float) * (size_t)total, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return total;
}

int64_t amod_synth_legacy_packets(int32_t nframes, int32_t first, int32_t payload_len, const uint8_t *name,
                                  int32_t name_len, uint8_t *out, int64_t *offsets, int32_t *lengths) {
  if (nframes < 0 || payload_len < 0 || name_len < 0) return AMOD_ERR_ARG;
  std::vector<uint8_t> data(payload_len);
  const int64_t plen = (int64_t)legacy_packet(data.data(), payload_len, name, name_len).size();
  if (!out) return plen * nframes;
  for (int32_t i = 0; i < nframes; ++i) {
    amod_synth_payload(0x9E3779B9u ^ (uint32_t)(first + i), payload_len, data.data());
    const auto p = legacy_packet(data.data(), payload_len, name, name_len);
    std::copy(p.begin(), p.end(), out + plen * i);
    offsets[i] = plen * i;
    lengths[i] = (int32_t)plen;
  }
  return plen * nframes;
}

int64_t amod_tx_test_signal(const amod_cfg *cfg, float *out) {
  uint8_t d[16];
  for (int i = 0; i < 16; ++i) d[i] = (uint8_t)i;
  return amod_tx_legacy(cfg, d, 16, (const uint8_t *)"test", 4, out);
}

void amod_synth_payload(uint32_t seed, int32_t len, uint8_t *out) {
  uint32_t s = seed;
  for (int32_t i = 0; i < len; ++i) {
    if ((i & 3) == 0) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; }
    out[i] = (uint8_t)((s >> (8 * (i & 3))) & 0xFF);
  }
}

int64_t amod_synth_legacy_batch(const amod_cfg *cfg, int32_t nframes, int32_t first, int32_t payload_len,
                                const uint8_t *name, int32_t name_len, float *out, int64_t *offsets,
                                int32_t *lengths, int32_t threads) {
  if (!validate(cfg) || nframes < 0 || payload_len < 0) return AMOD_ERR_ARG;
  // every frame has the same length (same payload size and name)
  std::vector<uint8_t> tmp(payload_len);
  const auto probe = legacy_packet(tmp.data(), payload_len, name, name_len);
  const int64_t flen = amod_tx_legacy(cfg, tmp.data(), payload_len, name, name_len, nullptr);
  (void)probe;
  const int64_t total = flen * nframes;
  if (!out) return total;
  for (int32_t i = 0; i < nframes; ++i) { offsets[i] = flen * i; lengths[i] = (int32_t)flen; }
  int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = std::min<int>(nt, std::max(1, nframes));
  std::atomic<int32_t> next{0};
  auto work = [&] {
    std::vector<uint8_t> data(payload_len);
    for (;;) {
      const int32_t i = next.fetch_add(1);
      if (i >= nframes) break;
      amod_synth_payload(0x9E3779B9u ^ (uint32_t)(first + i), payload_len, data.data());
      amod_tx_legacy(cfg, data.data(), payload_len, name, name_len, out + flen * i);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto &t : pool) t.join();
  return total;
}

} // extern "C"
