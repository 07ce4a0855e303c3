// k_decode_exact.hip — exact-replica path of the receive chain (gfx950).
//
// Replays modem.js in IEEE double, operation for operation (this file is built
// with -ffp-contract=off; fp64 add/mul/div/sqrt are correctly rounded), so every
// intermediate equals the reference bit for bit:
//   mean        sequential sum (preprocessSignal 215-217), one lane over LDS chunks
//   Schmidl-Cox sliding recurrence (detectPreamble 292-316): the per-position
//               increments and the metrics are independent of the running sums, so all
//               lanes compute them; one lane runs only the three sequential additions
//   fine timing one lane per candidate offset, sequential 576-tap sums (576-587)
//   FFT         radix-2 DIT stages with the reference's per-stage twiddle
//               recurrence tabulated on the host (fftIterative 26-47); each stage's
//               butterflies are independent, so 256 lanes run them in parallel
//               without changing a single rounding
//   equaliser / pilot phase / demap  as demodulateOFDM 386-413 (joint argmin)
// It runs for frames the fast kernel routes here (guard band hit, NaN/Inf, too
// long for LDS, or AMOD_OPT_FORCE_EXACT), one 256-thread workgroup per frame.
#include "amodem_internal.h"

namespace amod {
namespace {

constexpr int XT = 256;     // threads per workgroup
constexpr int CH = 3072;    // sample chunk staged in LDS (XSmem <= 40 KB: four workgroups per CU)

constexpr int SCH = kFft * 2; // Schmidl-Cox positions per chunk (3 x SCH doubles overlay the FFT arrays)
#ifndef AMOD_SEG_G
#define AMOD_SEG_G 1024
#endif
constexpr int kSegG = AMOD_SEG_G; // samples per certified segment of the mean (at least)

struct alignas(16) XSmem { // (static_assert below: four per CU fit the 160 KB of LDS)
  float chunk[CH + 520];
  union {
    struct {
      double re[kFft], im[kFft];
      double hr[kFft], hi[kFft];
      double er[kFft], ei[kFft];
    };
    double sc[3 * SCH]; // detectPreamble: per-position increments, then states (p, ra, rb)
  };
  double rd[XT / 64 + 4];
  float rf[XT / 64];
  int ri[XT / 64 + 4];
  uint32_t ru[16];
  double mean, mx, best, phase;
  float xmn, xmx;
  int coarse, start, status, nonfin;
};

static_assert(sizeof(XSmem) <= 40 * 1024, "list A's exact workgroup must fit beside three k_demod ones");

__device__ __forceinline__ double or_zero(float v) { return (v != v || v == 0.0f) ? 0.0 : (double)v; } // `x || 0`
__device__ __forceinline__ int rev9(int i) { return (int)(__brev((unsigned)i) >> 23); }

// fft(re, 0) of 512 real samples src[0..511] (modem.js:6-13, 26-66), result in sm.re/sm.im
__device__ void fft_exact(const float *src, XSmem &sm, const double2 *tw) {
  const int tid = threadIdx.x;
  for (int j = tid; j < kFft; j += XT) { sm.re[j] = or_zero(src[rev9(j)]); sm.im[j] = 0.0; }
  __syncthreads();
  for (int half = 1; half < kFft; half <<= 1) {
    const int t = tid; // 256 butterflies per stage
    const int blk = t / half, j = t - blk * half;
    const int a = blk * 2 * half + j, b = a + half;
    const double2 w = tw[half - 1 + j];
    const double t_re = w.x * sm.re[b] - w.y * sm.im[b];
    const double t_im = w.x * sm.im[b] + w.y * sm.re[b];
    sm.re[b] = sm.re[a] - t_re;
    sm.im[b] = sm.im[a] - t_im;
    sm.re[a] = sm.re[a] + t_re;
    sm.im[a] = sm.im[a] + t_im;
    __syncthreads();
  }
}

// Make this workgroup's global stores (plain or atomic) visible to its own later
// plain loads: drain them to L2, barrier, then drop this CU's L1 copies.
__device__ __forceinline__ void wg_global_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// fn(i, p[i]) for this thread's strided indices i = tid + k XT < N, in ascending order,
// eight loads in flight per thread (one workgroup streams a whole frame)
template <typename F> __device__ __forceinline__ void strided8(const float *__restrict__ p, int N, F &&fn) {
  int i = threadIdx.x;
  for (; i + 7 * XT < N; i += 8 * XT) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[i + u * XT];
#pragma unroll
    for (int u = 0; u < 8; ++u) fn(i + u * XT, v[u]);
  }
  for (; i < N; i += XT) fn(i, p[i]);
}

// fn(i, p[i]) for every i < N, as aligned float4 loads (a frame starts anywhere): one
// workgroup streams a whole frame with 4 x 16 B in flight per thread. Each thread sees its
// samples in no particular order (its callers only take order-free sums and extremes, or
// write sample i itself).
template <typename F> __device__ __forceinline__ void stream4(const float *__restrict__ p, int N, F &&fn) {
  const int ph = (int)((reinterpret_cast<uintptr_t>(p) >> 2) & 3);
  const float4 *const b = reinterpret_cast<const float4 *>(p - ph);
  const int nvec = (N + ph + 3) >> 2;
  auto use = [&](int v, const float4 t) {
    const int i0 = 4 * v - ph;
    if (i0 >= 0 && i0 + 3 < N) { fn(i0, t.x); fn(i0 + 1, t.y); fn(i0 + 2, t.z); fn(i0 + 3, t.w); }
    else {
      if (i0 >= 0 && i0 < N) fn(i0, t.x);
      if (i0 + 1 >= 0 && i0 + 1 < N) fn(i0 + 1, t.y);
      if (i0 + 2 >= 0 && i0 + 2 < N) fn(i0 + 2, t.z);
      if (i0 + 3 < N) fn(i0 + 3, t.w);
    }
  };
  int v = threadIdx.x;
  for (; v + 3 * XT < nvec; v += 4 * XT) {
    float4 t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = b[v + u * XT];
#pragma unroll
    for (int u = 0; u < 4; ++u) use(v + u * XT, t[u]);
  }
  for (; v < nvec; v += XT) use(v, b[v]);
}

__device__ __forceinline__ double js_max(double a, double b) { // Math.max, NaN-propagating
  if (a != a || b != b) return __builtin_nan("");
  return b > a ? b : a;
}

// detectPreambleCrossCorr (modem.js:235-284) on the preprocessed samples xs: a strided
// coarse search then a +-step fine search, each offset's sums sequential in fp64 on one
// lane; first strict maximum like the reference loops. Whole workgroup; returns the index
// or -1.
__device__ int crosscorr_detect(const float *xs, int N, const DevCfg &cfg, XSmem &sm) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pLen = cfg.sym;
  if (N < pLen || cfg.te < 1e-10) return -1;
  const int end = N - pLen;
  const int step = max(1, pLen / 10);
  int best_idx = -1;
  double best = 0.0;
  auto scan = [&](int d0, int d1, int dstep, double &b, int &bi) {
    double bm = b;
    int bx = 0x7fffffff;
    for (int d = d0 + tid * dstep; d <= d1; d += XT * dstep) {
      double corr = 0.0, se = 0.0;
      for (int i = 0; i < pLen; ++i) {
        const double sv = xs[d + i];
        corr += sv * (double)cfg.t.pre1[i];
        se += sv * sv;
      }
      const double den = sqrt(se * cfg.te);
      if (den > 0.001) {
        const double m = corr / den;
        if (m > bm) { bm = m; bx = d; }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double om = __shfl_xor(bm, o, 64);
      const int oi = __shfl_xor(bx, o, 64);
      if (om > bm || (om == bm && oi < bx)) { bm = om; bx = oi; }
    }
    __syncthreads();
    if (lane == 0) { sm.rd[wave] = bm; sm.ri[wave] = bx; }
    __syncthreads();
    double B = sm.rd[0];
    int I = sm.ri[0];
    for (int i = 1; i < XT / 64; ++i)
      if (sm.rd[i] > B || (sm.rd[i] == B && sm.ri[i] < I)) { B = sm.rd[i]; I = sm.ri[i]; }
    if (I != 0x7fffffff) { b = B; bi = I; } // some offset beat the running best
  };
  scan(0, end, step, best, best_idx);
  if (best_idx < 0 || best < 0.15) return -1;
  const int f0 = max(0, best_idx - step), f1 = min(end, best_idx + step);
  best = 0.0;
  scan(f0, f1, 1, best, best_idx);
  return best > 0.15 ? best_idx : -1;
}

// diagnostics only (AMOD_STAMPS): shader-clock marks 8-14 of an exact frame
#define XSTAMP(k)                                                                        \
  do {                                                                                  \
    if (w.stamps && tid == 0) w.stamps[(int64_t)f * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// the exact replica of one listed frame per workgroup iteration (kernels below)
__device__ __forceinline__ void exact_body(const DevCfg &cfg, const DevWork &w) {
  __shared__ XSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // listed frames are latency-bound chains (sequential recurrences) that run beside the
  // throughput-bound k_demod: their waves issue first on a shared SIMD
  __builtin_amdgcn_s_setprio(3);
  const int count = *w.fb_count;
  // list B (the decode's last launch) zeroes list A's count for the next decode (or graph
  // replay): every launch that appends to or reads it ran before this one
  if (w.fb_reset && blockIdx.x == 0 && tid == 0) *w.fb_reset = 0;
  const int SYM = cfg.sym, CP = cfg.cp;
  for (int item = blockIdx.x; item < count; item += gridDim.x) {
    const int f = w.fb_list[item];
    const int flags0 = w.fb_flags[item];
    const float *xr = w.samples + w.off[f];
    const int N = w.len[f];
    float *xs = w.xs + (int64_t)blockIdx.x * w.xs_stride;
    uint32_t *bits = w.bits + (int64_t)blockIdx.x * w.bits_stride;
    amod_debug *D = w.dbg ? w.dbg + f : nullptr;
    amod_result r;
    init_result(r);
    r.flags = flags0 | AMOD_FLAG_EXACT;
    XSTAMP(8);
    if (w.tl && tid == 0 && item == (int)blockIdx.x) atomicMin(w.tl, (unsigned long long)wall_clock64());
    if (w.stamps && tid == 0) w.stamps[(int64_t)f * 32 + 1] = __builtin_amdgcn_s_memrealtime(); // (100 MHz)
    {
      const int64_t need_bits = (int64_t)(N / SYM) * cfg.ndata * cfg.bps;
      if ((int64_t)N > w.xs_stride || 2 * ((need_bits + 31) / 32) + 16 > w.bits_stride) {
        if (tid == 0) { r.status = AMOD_E_CAPACITY; w.res[f] = r; }
        __syncthreads();
        continue;
      }
    }
    int status = AMOD_OK;
    int start = 0;
    const float *sig = xr; // samples the demodulator reads

    const bool loop = cfg.mode == AMOD_MODE_LOOPBACK; // analyzeLoopback's receive core
    // A frame the fast path listed only for demodulation-stage guards (k_demod: decision
    // margins, pilot |eqRe|, |H|^2, a parse past the demodulated symbols) or for opt-in
    // soft combining already has a proven preambleIdx: the replica runs preprocess +
    // demodulation only.
    const bool demod_only = cfg.mode == AMOD_MODE_RECEIVED && w.det && flags0 != 0 &&
        (flags0 & ~(AMOD_FLAG_DEMAP | AMOD_FLAG_PHASE | AMOD_FLAG_CHANNEL | AMOD_FLAG_SPAN | AMOD_FLAG_SOFT |
                    AMOD_FLAG_REPLAY)) == 0;
    // A frame listed only for detection-stage guards (and not for soft combining) replays
    // the detection here and goes back to k_demod (w.rp_count: the caller launches it)
    const bool replay = w.rp_count && w.det && !D && cfg.mode == AMOD_MODE_RECEIVED && flags0 != 0 &&
        (flags0 & ~(AMOD_FLAG_COARSE | AMOD_FLAG_FINE | AMOD_FLAG_THRESH)) == 0 &&
        !(soft_combine_applies(w.options, cfg.rep, cfg.mod) && !soft_fast(w.options, cfg));
    if (cfg.mode != AMOD_MODE_CHUNK) {
      // ---- preprocessSignal: the mean is a sequential double sum (modem.js:215-217).
      // Every partial sum of floats is a multiple of 2^emin (the smallest sample ulp) and
      // at most sum|x| in magnitude; when sum|x| < 2^(emin + 53) no partial sum rounds, in
      // any order, so the parallel sum is bit-equal to the sequential one. Otherwise (or
      // with non-finite samples) the sum runs sequentially.
      // (one pass: the parallel sum and its certificate, and the extremes, from which
      // the peak below follows without a pass of its own)
      double ps = 0.0, pa = 0.0;
      int emin = 1 << 20, nonfin = 0;
      float xmn = INFINITY, xmx = -INFINITY;
      stream4(xr, N, [&](int, float x) {
        ps += (double)x;
        pa += fabs((double)x);
        xmn = fminf(xmn, x);
        xmx = fmaxf(xmx, x);
        const uint32_t e = (__float_as_uint(x) >> 23) & 0xFFu;
        if (e == 0xFFu) nonfin = 1;
        else if (x != 0.0f) emin = min(emin, e == 0 ? -149 : (int)e - 150);
      });
      for (int o = 32; o > 0; o >>= 1) {
        ps += __shfl_xor(ps, o, 64);
        pa += __shfl_xor(pa, o, 64);
        emin = min(emin, __shfl_xor(emin, o, 64));
        nonfin |= __shfl_xor(nonfin, o, 64);
        xmn = fminf(xmn, __shfl_xor(xmn, o, 64));
        xmx = fmaxf(xmx, __shfl_xor(xmx, o, 64));
      }
      if (lane == 0) { sm.rd[wave] = ps; sm.ri[wave] = emin; sm.ri[XT / 64 + wave] = nonfin; }
      if (lane == 0) { sm.er[wave] = pa; sm.rf[wave] = xmn; sm.ei[wave] = (double)xmx; }
      __syncthreads();
      bool exact_par = true;
      if (tid == 0) {
        double S = 0.0, PA = 0.0;
        int EM = 1 << 20, NF = 0;
        float MN = INFINITY, MX = -INFINITY;
        for (int i = 0; i < XT / 64; ++i) {
          S += sm.rd[i]; PA += sm.er[i]; EM = min(EM, sm.ri[i]); NF |= sm.ri[XT / 64 + i];
          MN = fminf(MN, sm.rf[i]); MX = fmaxf(MX, (float)sm.ei[i]);
        }
        sm.xmn = MN; sm.xmx = MX; sm.nonfin = NF;
        // non-finite samples: NaN, or +-Inf, whatever the order (finite sums stay finite)
        exact_par = NF || EM >= (1 << 19) || PA * (1.0 + 0x1p-40) < ldexp(1.0, EM + 53);
        sm.mean = S / (double)N;
        sm.status = exact_par;
      }
      __syncthreads();
      exact_par = sm.status != 0;
      __syncthreads();
      XSTAMP(13);
      if (!exact_par) {
        // Segments of G >= kSegG samples, certified one by one along the sequential order. A
        // segment whose sum|x| < 2^(em + 53) (em: its smallest sample ulp exponent) has
        // exact internal sums in any order, so its total comes out exact from one thread's
        // running sum. With S the running (sequential) sum at its start and q the smaller
        // of em and the exponent of S's lowest set bit, every partial sum S + P_j is a
        // multiple of 2^q no larger than |S| + sum|x| in magnitude; below 2^(q + 53) none
        // of them rounds and S + total is the sequential result. A segment failing either
        // test (a sample far below the running sum's ulp, or a partial sum that could
        // round) is summed sample by sample. One thread per segment (the frame is
        // L2-resident after the pass above): no cross-lane scans.
        constexpr int SEGCAP = SCH;
        double *const seg_s = sm.sc, *const seg_a = sm.sc + SEGCAP, *const seg_e = sm.sc + 2 * SEGCAP;
        const int G = kSegG * max(1, (N + kSegG * SEGCAP - 1) / (kSegG * SEGCAP));
        const int nseg = (N + G - 1) / G;
        for (int sg = tid; sg < nseg; sg += XT) {
          const int b0 = sg * G, e1 = min(N, b0 + G);
          double ss = 0.0, sa = 0.0;
          int em = 1 << 20;
          auto add = [&](float x) {
            ss += (double)x;
            sa += fabs((double)x);
            const uint32_t e = (__float_as_uint(x) >> 23) & 0xFFu;
            if (x != 0.0f) em = min(em, e == 0 ? -149 : (int)e - 150);
          };
          int i = b0;
          for (; i + 8 <= e1; i += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = xr[i + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) add(v[u]);
          }
          for (; i < e1; ++i) add(xr[i]);
          seg_s[sg] = ss; seg_a[sg] = sa; seg_e[sg] = (double)em;
        }
        __syncthreads();
        if (wave == 0) { // the chain along the segments: wave-uniform S on every lane
          double S = 0.0;
          for (int sg = 0; sg < nseg; ++sg) {
            const int em = (int)seg_e[sg];
            if (em >= (1 << 19)) continue; // all zeros
            // S is a multiple of 2^(exponent of its lowest set bit)
            int qs = 1 << 20;
            if (S != 0.0) {
              const uint64_t b = (uint64_t)__double_as_longlong(S);
              const int be = (int)((b >> 52) & 0x7FF);
              const uint64_t m = (b & 0xFFFFFFFFFFFFFull) | (be ? (1ull << 52) : 0ull);
              qs = (be ? be : 1) - 1075 + __builtin_ctzll(m);
            }
            const int q = min(em, qs);
            // (sum|x| in fp64 over G terms: relative error below G 2^-53)
            const double slack = 1.0 + ldexp((double)G, -52);
            const bool inner = seg_a[sg] * slack < ldexp(1.0, em + 53);
            const double reach = (fabs(S) + seg_a[sg]) * slack;
            if (inner && reach < ldexp(1.0, q + 53)) {
              S += seg_s[sg];
            } else { // sample by sample: 64 coalesced loads, then lane by lane in order
              const int e1 = min(N, (sg + 1) * G);
              for (int b0 = sg * G; b0 < e1; b0 += 64) {
                const float v = b0 + lane < e1 ? xr[b0 + lane] : 0.f;
                const int nj = min(64, e1 - b0);
                for (int j = 0; j < nj; ++j) S += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
              }
            }
          }
          if (lane == 0) sm.mean = S / (double)N;
        }
      }
      __syncthreads();
      XSTAMP(14);
      const double mean = sm.mean;
      double mx = 0.0;
      if (!sm.nonfin) {
        // finite samples: max |f32(x - mean)| is reached at an extreme (fl64(x - mean) and
        // the f32 rounding are monotone in x), so the peak is known before the one pass
        // that writes the normalised samples
        if (tid == 0) {
          const double m = N == 0 ? 0.0 : js_max(js_max(0.0, fabs((double)(float)((double)sm.xmx - mean))),
                                                 fabs((double)(float)((double)sm.xmn - mean)));
          sm.mx = m;
          if (D) { D->mean = mean; D->mx = m; }
        }
        __syncthreads();
        mx = sm.mx;
        // a replayed detection reads the normalised samples only up to its fine window
        // (the recurrence stops at the proven hull's end; k_demod reads the raw samples)
        int nn = N;
        if (replay) {
          const DetRec dr = w.det[f];
          if (dr.sc_lo >= 0 && dr.sc_hi >= dr.sc_lo) nn = (int)min<int64_t>(N, (int64_t)dr.sc_hi + kFft + 3 * CP + SYM + 1);
        }
        if (mx > 1e-6) stream4(xr, nn, [&](int i, float x) { xs[i] = (float)((double)(float)((double)x - mean) / mx); });
        else stream4(xr, nn, [&](int i, float x) { xs[i] = (float)((double)x - mean); });
      } else { // NaN / Inf: Math.max's NaN propagation over every sample, then the division
        stream4(xr, N, [&](int i, float x) {
          const float o = (float)((double)x - mean);
          xs[i] = o;
          mx = js_max(mx, fabs((double)o));
        });
        for (int o = 32; o > 0; o >>= 1) mx = js_max(mx, __shfl_xor(mx, o, 64));
        if (lane == 0) sm.rd[wave] = mx;
        __syncthreads();
        if (tid == 0) {
          double m = 0.0;
          for (int i = 0; i < XT / 64; ++i) m = js_max(m, sm.rd[i]);
          sm.mx = m;
          if (D) { D->mean = mean; D->mx = m; }
        }
        wg_global_sync(); // (the pass below reads samples other threads wrote)
        mx = sm.mx;
        if (mx > 1e-6) stream4(xs, N, [&](int i, float o) { xs[i] = (float)((double)o / mx); }); // own indices only
      }
      wg_global_sync();
      sig = xs;
      XSTAMP(9);

      // ---- detectPreamble: sequential recurrence, one lane
      const int half = kFft / 2;
      int coarse = -1;
      double best = 0.0;
      if (demod_only) {
        // the fast path's detection record: preambleIdx proven by its guards
        const DetRec dr = w.det[f];
        r.flags |= dr.flags; // a replayed detection's flags (0 for k_detect's records)
        r.coarse_idx = dr.coarse;
        r.fine_metric = dr.fbest;
        r.preamble_idx = start = dr.start;
      } else if (N >= 2 * half) {
        // chunk of positions [c0, c0 + n): (1) every lane forms the increments
        // fl(fl(mid bIn) - fl(aOut mid)) etc. of the updates at those positions, (2) lane 0
        // replaces each increment by the running state at that position and adds it (the
        // only sequential step: three independent fp64 additions), (3) every lane forms
        // the metric p^2 / (ra rb) of its positions, first strict maximum per lane;
        // lanes then combine by (metric, lowest index) = the reference's first maximum
        const int end = N - 2 * half;
        // a frame the coarse stage listed with a proven hull [sc_lo, sc_hi] of the argmax:
        // the recurrence runs to sc_hi, metrics are compared there only
        int d_lo = 0, d_hi = end;
        if (w.det && cfg.mode == AMOD_MODE_RECEIVED && !loop) {
          const DetRec dr = w.det[f];
          if (dr.sc_lo >= 0 && dr.sc_hi >= dr.sc_lo) { d_lo = dr.sc_lo; d_hi = min(dr.sc_hi, end); }
        }
        if (w.stamps && tid == 0) // (diagnostics: the recurrence's range, slot 7)
          w.stamps[(int64_t)f * 32 + 7] = ((unsigned long long)(uint32_t)d_lo << 32) | (uint32_t)d_hi;
        // lanes 0, 1, 2 carry the three independent recurrences p, ra, rb (each lane its
        // own array of increments -> states), so one instruction stream advances all three
        double acc = 0.0;
        double bm = 0.0;                     // > best = 0 like the reference's first test
        int bi = -1;
        double *const tp = sm.sc, *const tra = sm.sc + SCH, *const trb = sm.sc + 2 * SCH;
        if (tid < 3) { // P(0), Ra(0), Rb(0) (modem.js:292-298), one sum per lane
          for (int m = 0; m < half; ++m) {
            const double a = xs[m], b = xs[m + half];
            acc += tid == 0 ? a * b : (tid == 1 ? a * a : b * b);
          }
        }
        // positions [0, P1) before the hull: only the running sums matter, in a pipeline of
        // half-chunks (HB positions): wave 0's lanes 0-2 add the increments of half h while
        // waves 1-3 form those of half h + 1 in the other half of the buffer
        constexpr int HB = SCH / 2;
        const int P1 = (d_lo / HB) * HB;
        if (P1 > 0) {
          const int nh = P1 / HB;
          // increments of half h's positions from samples (a_out, mid, b_in), into buffer h & 1
          auto put = [&](int h, int k, float a_out_f, float mid_f, float b_in_f) {
            double *const bp = sm.sc + (h & 1) * 3 * HB;
            const int d = h * HB + k;
            double ip = 0.0, ia = 0.0, ib = 0.0;
            if (d < end) {
              const double a_out = a_out_f, mid = mid_f, b_in = b_in_f;
              ip = mid * b_in - a_out * mid;
              ia = mid * mid - a_out * a_out;
              ib = b_in * b_in - mid * mid;
            }
            bp[k] = ip; bp[HB + k] = ia; bp[2 * HB + k] = ib;
          };
          auto ld = [&](int d) { return d < N ? xs[d] : 0.f; };
          for (int k = tid; k < HB; k += XT) put(0, k, ld(k), ld(k + half), ld(k + 2 * half));
          // waves 1-3: thread tt forms positions tt, tt + 192, tt + 384 of a half; its samples
          // for half h + 2 are loaded while half h + 1's increments are formed from registers
          constexpr int PT = (HB + XT - 65) / (XT - 64);
          const int tt = tid - 64;
          float ra[PT], rm[PT], rb[PT];
          auto load_half = [&](int h) {
#pragma unroll
            for (int j = 0; j < PT; ++j) {
              const int k = tt + (XT - 64) * j, d = h * HB + k;
              const bool v = k < HB;
              ra[j] = v ? ld(d) : 0.f; rm[j] = v ? ld(d + half) : 0.f; rb[j] = v ? ld(d + 2 * half) : 0.f;
            }
          };
          if (wave > 0 && nh > 1) load_half(1);
          __syncthreads();
          for (int h = 0; h < nh; ++h) {
            if (wave == 0) {
              if (lane < 3) {
                const double2 *const v = reinterpret_cast<const double2 *>(sm.sc + (h & 1) * 3 * HB + lane * HB);
                // (the next eight pairs are read while these are added: the adds are the chain)
                double2 t[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) t[j] = v[j];
                for (int k = 0; k < HB / 2; k += 8) {
                  double2 u[8];
                  const int kn = k + 8 < HB / 2 ? k + 8 : k;
#pragma unroll
                  for (int j = 0; j < 8; ++j) u[j] = v[kn + j];
#pragma unroll
                  for (int j = 0; j < 8; ++j) { acc += t[j].x; acc += t[j].y; }
#pragma unroll
                  for (int j = 0; j < 8; ++j) t[j] = u[j];
                }
              }
            } else {
              if (h + 1 < nh) {
#pragma unroll
                for (int j = 0; j < PT; ++j) {
                  const int k = tt + (XT - 64) * j;
                  if (k < HB) put(h + 1, k, ra[j], rm[j], rb[j]);
                }
              }
              if (h + 2 < nh) load_half(h + 2);
            }
            __syncthreads();
          }
        }
        for (int c0 = P1; c0 <= d_hi; c0 += SCH) {
          const int n = min(SCH, d_hi + 1 - c0);
          const int ns = n + 2 * half; // samples [c0, c0 + n + 512) <= N
          for (int i = tid; i < ns; i += XT) sm.chunk[i] = c0 + i < N ? xs[c0 + i] : 0.f;
          __syncthreads();
          for (int k = tid; k < n; k += XT) {
            double ip = 0.0, ia = 0.0, ib = 0.0;
            if (c0 + k < end) {
              const double a_out = sm.chunk[k], mid = sm.chunk[k + half], b_in = sm.chunk[k + 2 * half];
              ip = mid * b_in - a_out * mid;
              ia = mid * mid - a_out * a_out;
              ib = b_in * b_in - mid * mid;
            }
            tp[k] = ip; tra[k] = ia; trb[k] = ib;
          }
          __syncthreads();
          const bool keep = c0 + n > d_lo; // some position of this chunk is compared
          if (tid < 3) {
            double2 *const v = reinterpret_cast<double2 *>(sm.sc + tid * SCH);
            int k = 0;
            if (!keep) { // states not needed: the running sum only
              for (; k + 8 <= n; k += 8) {
                double2 t[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) t[j] = v[(k >> 1) + j];
#pragma unroll
                for (int j = 0; j < 4; ++j) { acc += t[j].x; acc += t[j].y; }
              }
            } else {
              for (; k + 8 <= n; k += 8) {
                double2 t[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) t[j] = v[(k >> 1) + j];
#pragma unroll
                for (int j = 0; j < 4; ++j) { // state at the position, then its update
                  const double s0 = acc;
                  acc += t[j].x; // zero past `end`: adding +0.0 changes nothing
                  const double s1 = acc;
                  acc += t[j].y;
                  v[(k >> 1) + j] = make_double2(s0, s1);
                }
              }
            }
            double *const vs = sm.sc + tid * SCH;
            for (; k < n; ++k) {
              const double t = vs[k];
              vs[k] = acc;
              acc += t;
            }
          }
          __syncthreads();
          for (int k = tid; keep && k < n; k += XT) {
            if (c0 + k < d_lo) continue;
            const double pp = tp[k], a = tra[k], b = trb[k];
            if (a > 0.01 && b > 0.01) {
              const double metric = (pp * pp) / (a * b);
              if (metric > bm) { bm = metric; bi = c0 + k; }
            }
          }
          __syncthreads();
        }
        for (int o = 32; o > 0; o >>= 1) {
          const double om = __shfl_xor(bm, o, 64);
          const int oi = __shfl_xor(bi, o, 64);
          if (om > bm || (om == bm && oi >= 0 && (bi < 0 || oi < bi))) { bm = om; bi = oi; }
        }
        if (lane == 0) { sm.rd[wave] = bm; sm.ri[wave] = bi; }
        __syncthreads();
        if (tid == 0) {
          best = 0.0; coarse = -1;
          for (int i = 0; i < XT / 64; ++i)
            if (sm.rd[i] > best || (sm.rd[i] == best && sm.ri[i] >= 0 && (coarse < 0 || sm.ri[i] < coarse))) {
              best = sm.rd[i]; coarse = sm.ri[i];
            }
        }
        if (tid == 0) { sm.best = best; sm.coarse = best > 0.5 ? coarse : -1; }
      } else if (tid == 0) {
        sm.best = 0.0; sm.coarse = -1;
      }
      __syncthreads();
      XSTAMP(10);
      if (!demod_only) {
      coarse = sm.coarse;
      if (loop && coarse < 0) coarse = crosscorr_detect(xs, N, cfg, sm); // modem.js:982-985
      r.coarse_idx = coarse;
      if (D && tid == 0) { D->coarse_metric = sm.best; D->coarse_lo = coarse; D->coarse_hi = coarse; }
      if (coarse < 0) {
        status = AMOD_E_PREAMBLE;
      } else {
        // ---- fine timing: one lane per offset, sequential sums (modem.js:567-588)
        const int R = CP * 3;
        const int lo = max(0, coarse - R), hi = min(N - SYM, coarse + R);
        double bm = -__builtin_inf();
        int bi = 0x7fffffff;
        // the window [lo, hi + SYM) staged in LDS (the S-C chunk buffer is free now); f32 x
        // f32 products are exact in double, so fma(s, q, corr) is the reference's
        // corr + s * q with its one rounding
        const int wn = hi + SYM - lo;
        const bool staged = wn > 0 && wn + SYM <= CH + 520 && (SYM & 7) == 0;
        auto offset = [&](const float *win, const float *q, int d) {
          double corr = 0.0, se = 0.0;
          if (staged) { // LDS: the next eight samples and coefficients are read under these
            float a[8], c[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) { a[j] = win[j]; c[j] = q[j]; }
            for (int i = 0; i < SYM; i += 8) {
              float an[8], cn[8];
              const int in = i + 8 < SYM ? i + 8 : i;
#pragma unroll
              for (int j = 0; j < 8; ++j) { an[j] = win[in + j]; cn[j] = q[in + j]; }
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const double sv = a[j];
                corr = __builtin_fma(sv, (double)c[j], corr);
                se = __builtin_fma(sv, sv, se);
              }
#pragma unroll
              for (int j = 0; j < 8; ++j) { a[j] = an[j]; c[j] = cn[j]; }
            }
          } else {
            for (int i = 0; i < SYM; ++i) {
              const double sv = win[i];
              corr = __builtin_fma(sv, (double)q[i], corr);
              se = __builtin_fma(sv, sv, se);
            }
          }
          const double den = sqrt(se * cfg.te);
          if (den > 0.001) {
            const double m = corr / den;
            if (m > bm) { bm = m; bi = d; }
          }
        };
        if (staged) {
          for (int i = tid; i < wn; i += XT) sm.chunk[i] = xs[lo + i];
          for (int i = tid; i < SYM; i += XT) sm.chunk[wn + i] = cfg.t.pre1[i];
          __syncthreads();
          for (int d = lo + tid; d <= hi; d += XT) offset(sm.chunk + (d - lo), sm.chunk + wn, d);
        } else {
          for (int d = lo + tid; d <= hi; d += XT) offset(xs + d, cfg.t.pre1, d);
        }
        // argmax over lanes: highest metric, then lowest offset (strict '>' in order)
        for (int o = 32; o > 0; o >>= 1) {
          const double om = __shfl_xor(bm, o, 64);
          const int oi = __shfl_xor(bi, o, 64);
          if (om > bm || (om == bm && oi < bi)) { bm = om; bi = oi; }
        }
        if (lane == 0) { sm.rd[wave] = bm; sm.ri[wave] = bi; }
        __syncthreads();
        if (tid == 0) {
          double B = -__builtin_inf();
          int I = 0x7fffffff;
          for (int i = 0; i < XT / 64; ++i)
            if (sm.rd[i] > B || (sm.rd[i] == B && sm.ri[i] < I)) { B = sm.rd[i]; I = sm.ri[i]; }
          sm.best = B;
          sm.start = I == 0x7fffffff ? coarse : I;
          if (D) { D->fine_metric = B; D->fine_idx = sm.start; }
        }
        __syncthreads();
        start = sm.start;
        r.fine_metric = (float)sm.best;
        if (loop) {  // no correlation cut-off; the data part may be empty (modem.js:1012-1045)
          if (start + 3 * SYM > N) status = AMOD_E_SHORT_CE;
        } else if (sm.best < 0.1) status = AMOD_E_LOW_CORR;
        else if (start + 3 * SYM > N) status = AMOD_E_SHORT_CE;
        else if (start + 3 * SYM >= N) status = AMOD_E_NO_DATA;
        r.preamble_idx = start;
      }
      }
    } else {
      if (3 * SYM > N) status = AMOD_E_FRAME_SHORT_CE;
      else if (3 * SYM >= N) status = AMOD_E_NO_DATA;
    }

    if (status != AMOD_OK) {
      if (tid == 0) {
        r.status = status;
        if (!loop) r.preamble_idx = -1;
        w.res[f] = r;
      }
      __syncthreads();
      continue;
    }
    XSTAMP(15); // (diagnostics: detection done)
    if (w.stamps && tid == 0) w.stamps[(int64_t)f * 32 + 2] = __builtin_amdgcn_s_memrealtime();
    if (replay) {
      // detection replay: preambleIdx (and the coarse index and fine metric the result
      // reports) now equal the reference's; the demodulation is k_demod's, under its own
      // guards (a frame they list comes back here, demodulation only). The record carries
      // the normalisation of the replica's exact mean and peak, as k_detect's does.
      if (tid == 0) {
        const double mean = sm.mean, mx = sm.mx;
        DetRec d;
        d.route = ROUTE_REPLAY; d.flags = flags0 | AMOD_FLAG_REPLAY; d.start = start;
        d.M = (N - (start + 3 * SYM)) / SYM; d.T = min(d.M, w.mcap); d.coarse = r.coarse_idx;
        if (mx > 1e-6) { d.A = (float)(1.0 / mx); d.B = (float)(-mean / mx); }
        else { d.A = 1.f; d.B = (float)(-mean); }
        d.fbest = r.fine_metric; d.sc_lo = d.sc_hi = -1; d.pad = 0.f;
        w.det[f] = d;
        w.rp_list[atomicAdd(w.rp_count, 1)] = f;
      }
      __syncthreads();
      continue;
    }

    XSTAMP(11);
    // ---- channel estimate (estimateChannel, modem.js:421-440)
    const int ce0 = start + 2 * SYM, data0 = start + 3 * SYM;
    fft_exact(sig + ce0 + CP, sm, cfg.t.tw_exact);
    for (int k = tid; k < kFft; k += XT) {
      double hr = 0.0, hi = 0.0;
      if (k >= cfg.sub_start && k <= cfg.sub_end) {
        const double xr_ = (double)cfg.t.known[k - cfg.sub_start], xi_ = 0.0;
        const double d = xr_ * xr_ + xi_ * xi_;
        if (d > 1e-10) {
          hr = (sm.re[k] * xr_ + sm.im[k] * xi_) / d;
          hi = (sm.im[k] * xr_ - sm.re[k] * xi_) / d;
        }
        if (D) { D->h_re[k - cfg.sub_start] = hr; D->h_im[k - cfg.sub_start] = hi; }
      }
      sm.hr[k] = hr; sm.hi[k] = hi;
    }
    __syncthreads();

    // ---- demodulateOFDM (modem.js:365-418)
    const int M = max(0, N - data0) / SYM;
    const int nbits = M * cfg.ndata * cfg.bps;
    const int nwords = (nbits + 31) >> 5;
    for (int i = tid; i < nwords + 8; i += XT) bits[i] = 0u;
    wg_global_sync();
    const int npts = cfg.mod == AMOD_BPSK ? 2 : (cfg.mod == AMOD_QPSK ? 4 : 16);
    // opt-in soft combining (AMOD_OPT_SOFT_COMBINE, not reference behaviour): per-bit soft
    // values, < 0 for bit 1 (BPSK: cr; QPSK MSB: ci, LSB: max-log min(|cr|, |ci|) signed
    // by whether the signs differ, the Gray map of initConstellation)
    float *const sv = (soft_combine_applies(w.options, cfg.rep, cfg.mod) && w.soft &&
                       (int64_t)nbits <= w.soft_stride)
                          ? w.soft + (int64_t)blockIdx.x * w.soft_stride
                          : nullptr;
    for (int s = 0; s < M; ++s) {
      __syncthreads();
      fft_exact(sig + data0 + s * SYM + CP, sm, cfg.t.tw_exact);
      for (int k = tid; k < kFft; k += XT) {
        double er = 0.0, ei = 0.0;
        if (k >= cfg.sub_start && k <= cfg.sub_end) {
          const double hr = sm.hr[k], hi = sm.hi[k];
          const double hmag = hr * hr + hi * hi;
          if (hmag > 1e-10) {
            er = (sm.re[k] * hr + sm.im[k] * hi) / hmag;
            ei = (sm.im[k] * hr - sm.re[k] * hi) / hmag;
          } else {
            er = sm.re[k]; ei = sm.im[k];
          }
          if (D && s == 0) {
            const int b = k - cfg.sub_start;
            D->x_re[b] = sm.re[k]; D->x_im[b] = sm.im[k]; D->eq_re[b] = er; D->eq_im[b] = ei;
          }
        }
        sm.er[k] = er; sm.ei[k] = ei;
      }
      __syncthreads();
      if (tid == 0) {
        double ps = 0.0;
        int pc = 0;
        for (int i = 0; i < cfg.npilots; ++i) {
          const int p = cfg.pilots[i];
          if (p >= cfg.sub_start && p <= cfg.sub_end && fabs(sm.er[p]) > 1e-6) { ps += sm.ei[p] / sm.er[p]; pc++; }
        }
        sm.phase = pc > 0 ? ps / (double)pc : 0.0;
        if (D && s < AMOD_DBG_SYMS) D->phase[s] = sm.phase;
      }
      __syncthreads();
      const double ph = sm.phase;
      for (int b = tid; b < cfg.nband; b += XT) {
        const int di = cfg.t.band_di[b];
        if (di < 0) continue;
        const int k = cfg.sub_start + b;
        const double cr = sm.er[k] + sm.ei[k] * ph;
        const double ci = sm.ei[k] - sm.er[k] * ph;
        double md = __builtin_inf();
        int mi = 0;
        for (int i = 0; i < npts; ++i) {
          const double dr = cr - cfg.t.points[i].x, dd = ci - cfg.t.points[i].y;
          const double dist = dr * dr + dd * dd;
          if (dist < md) { md = dist; mi = i; }
        }
        const int pos = (s * cfg.ndata + di) * cfg.bps;
        if (sv) {
          // weighted by |H|^2: the equaliser's division amplifies noise where the channel
          // estimate is weak, so each bit counts in proportion to its channel power (MRC)
          const double wgt = sm.hr[k] * sm.hr[k] + sm.hi[k] * sm.hi[k];
          if (cfg.mod == AMOD_BPSK) {
            sv[pos] = (float)(cr * wgt);
          } else {
            const double m = fmin(fabs(cr), fabs(ci)) * wgt;
            sv[pos] = (float)(ci * wgt);
            sv[pos + 1] = (float)(((cr < 0.0) != (ci < 0.0)) ? -m : m);
          }
        }
        const uint32_t val = (uint32_t)mi << (32 - cfg.bps - (pos & 31));
        if (val) atomicOr(&bits[pos >> 5], val);
      }
    }
    wg_global_sync();
    XSTAMP(12);
    if (D && tid == 0) D->nsym = M;
    r.nbits = nbits;
    const uint32_t *v = bits;
    int nv = nbits;
    if (cfg.rep > 1) {
      uint32_t *voted = bits + ((nwords + 3) & ~3);
      nv = sv ? soft_vote(sv, nbits, cfg.rep, voted) : block_vote(bits, nbits, cfg.rep, voted);
      wg_global_sync();
      v = voted;
    }
    if (loop) {  // analyzeLoopback parses nothing: the raw decoded bytes go back to the caller
      const int nbytes = nv >> 3, nw = (nbytes + 3) >> 2, cap_w = (int)(w.stride >> 2);
      uint32_t *dst = reinterpret_cast<uint32_t *>(w.payload + (int64_t)f * w.stride);
      for (int i = tid; i < nw && i < cap_w; i += XT) dst[i] = __builtin_bswap32(v[i]);
      if (tid == 0) {
        r.status = AMOD_OK; r.nbytes = nbytes; r.payload_valid = min(nbytes, 4 * cap_w); r.preamble_idx = start;
        w.res[f] = r;
      }
      __syncthreads();
      continue;
    }
    finish_frame(v, nv, cfg, r, w.res + f, w.payload + (int64_t)f * w.stride, w.stride, sm.ru, nullptr, nv >> 3);
    __syncthreads();
  }
}

// list A's instance, capped at 128 VGPRs: k_demod's waves hold 128 each, so with one of
// its workgroups per CU yielded an exact wave fits on every SIMD beside three of them
// (at 168 it waited for k_demod's waves to retire); list B's runs alone after k_demod
// (no cap: its launch skips the scratch setup even when the list is empty)
template <int WPE> __global__ void k_decode_exact(const DevCfg cfg, const DevWork w);
template <> __global__ __launch_bounds__(XT) __attribute__((amdgpu_waves_per_eu(4))) void k_decode_exact<4>(const DevCfg cfg,
                                                                                                            const DevWork w) {
  exact_body(cfg, w);
}
template <> __global__ __launch_bounds__(XT) __attribute__((amdgpu_waves_per_eu(2))) void k_decode_exact<2>(const DevCfg cfg,
                                                                                                            const DevWork w) {
  exact_body(cfg, w);
}

} // namespace
} // namespace amod

extern "C" hipError_t amod_launch_exact(const amod::DevCfg &cfg, const amod::DevWork &w, int nslots, hipStream_t s,
                                        bool beside_demod) {
  if (nslots <= 0) return hipSuccess;
  if (beside_demod)
    hipLaunchKernelGGL(amod::k_decode_exact<4>, dim3(nslots), dim3(amod::XT), 0, s, cfg, w);
  else
    hipLaunchKernelGGL(amod::k_decode_exact<2>, dim3(nslots), dim3(amod::XT), 0, s, cfg, w);
  return hipGetLastError();
}
