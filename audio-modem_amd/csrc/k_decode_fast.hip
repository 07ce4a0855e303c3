// k_decode_fast.hip — LDS-resident fast path of the OFDM receive chain (gfx950).
//
// One 1024-thread workgroup (16 waves) per frame; the raw float32 frame is read
// from HBM once (float4, coalesced) into LDS and every stage works from there:
//
//   stage 0  load + stats        preprocessSignal (modem.js:213-232): fp64 sum, min, max
//   stage 1  Schmidl-Cox scan    detectPreamble (286-319): 32-block window sums + slide
//   stage 2  fine timing         inline xcorr (567-588): 4 positions x 4 tap-splits per lane
//   stage 3  FFT jobs            estimateChannel (421-440) + demodulateOFDM (365-418):
//                                two real symbols packed into one 512-pt complex FFT per
//                                wave, radix-8 x 3 with two swizzled LDS exchanges done
//                                in place in the symbols' own sample slots
//   stage 4  finish              majorityVote / bitsToBytes / parse / CRC-32 (shared)
//
// Arithmetic is fp32. Every discrete decision (detection threshold, gates, argmax,
// constellation decision, pilot/channel thresholds) carries a guard band sized
// from an error bound; a frame with any decision inside its band is appended to
// the exact list and re-decoded by k_decode_exact (IEEE double, reference order).
#include "amodem_internal.h"

namespace amod {
namespace {

constexpr int WG = 1024;
constexpr int NWAVE = WG / 64;
constexpr int SC_BLK = 32;                 // Schmidl-Cox block / segment length
constexpr int UNION_BYTES = 13312;         // stage-shared scratch
constexpr int CAP = 37120;                 // max samples per LDS-resident frame
constexpr int MAX_BITS_WORDS = 1640;       // 64 symbols x 820 bits
constexpr int FINE_MAX = 2048;             // max fine-search positions (else exact)

struct alignas(16) Smem {
  float x[CAP + 16];                       // raw samples: x[ph + i] is frame sample i
  union alignas(16) U {
    struct { float bz[1184]; float be[1184]; } sc;             // stage 1
    struct { float tmpl[768]; float m[FINE_MAX]; } fine;        // stage 2
    struct {                                                      // stage 3
      float2 tw1[8 * 64];
      float2 tw2[8 * 8];
      float2 g[kMaxBand];                  // conj(H)/|H|^2 (or 1 for passthrough)
      uint32_t bits[MAX_BITS_WORDS];
    } fq;
    unsigned char raw[UNION_BYTES];
  } u;
  float rf[4 * NWAVE];
  int ri[4 * NWAVE];
  double rd[2 * NWAVE];
  uint32_t ru[16];
  // per-frame scalars (written by one thread, read after a barrier)
  int n, ph, status, flags, coarse, clo, chi, start, nsym, data0;
  float A, B, cbest, fbest, gmax, zce;
  double mean, mx;
};
static_assert(sizeof(Smem) <= 163840 - 256, "LDS budget");

__device__ __forceinline__ float2 operator+(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 operator-(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}

// 4-point DFT, W4 = -i
__device__ __forceinline__ void dft4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
  const float2 s02 = a0 + a2, d02 = a0 - a2, s13 = a1 + a3, d13 = a1 - a3;
  a0 = s02 + s13;
  a2 = s02 - s13;
  a1 = make_float2(d02.x + d13.y, d02.y - d13.x);
  a3 = make_float2(d02.x - d13.y, d02.y + d13.x);
}
// 8-point DFT in natural order: v[q] <- sum_m v[m] W8^{mq}
__device__ __forceinline__ void dft8(float2 (&v)[8]) {
  const float r = 0.70710678118654752f;
  float2 a0 = v[0] + v[4], a1 = v[1] + v[5], a2 = v[2] + v[6], a3 = v[3] + v[7];
  float2 b0 = v[0] - v[4], b1 = v[1] - v[5], b2 = v[2] - v[6], b3 = v[3] - v[7];
  b1 = make_float2((b1.x + b1.y) * r, (b1.y - b1.x) * r);
  b2 = make_float2(b2.y, -b2.x);
  b3 = make_float2((b3.y - b3.x) * r, -(b3.x + b3.y) * r);
  dft4(a0, a1, a2, a3);
  dft4(b0, b1, b2, b3);
  v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
  v[1] = b0; v[3] = b1; v[5] = b2; v[7] = b3;
}

// exchange-buffer addressing: 8 rows of 64 float2, rows 0-3 in region a, 4-7 in b
__device__ __forceinline__ float2 *xrow(float2 *ra, float2 *rb, int row) {
  return (row < 4 ? ra : rb) + (row & 3) * 64;
}
__device__ __forceinline__ int swz2(int q, int l1, int p1) { // exchange-2 column swizzle
  return 8 * ((l1 ^ q) & 7) + ((p1 ^ ((q & 3) + 4 * (l1 >> 2))) & 7);
}
__device__ __forceinline__ int spec_idx(int n) { return n ^ (((n >> 5) & 1) << 2); }

// One wave: 512-pt complex FFT of z (lane l holds z[l + 64 m] in v[m]); result
// X[n] left in the exchange buffer at spec(n) = row n>>6, col spec_idx(n)&63.
__device__ void fft512_wave(float2 (&v)[8], float2 *ra, float2 *rb, const Smem &sm) {
  const int l = wave_lane();
  dft8(v);
#pragma unroll
  for (int q = 1; q < 8; ++q) v[q] = cmul(v[q], sm.u.fq.tw1[q * 64 + l]);
  // exchange 1: row q, col l ^ (q<<3)
#pragma unroll
  for (int q = 0; q < 8; ++q) xrow(ra, rb, q)[l ^ (q << 3)] = v[q];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int l1 = l & 7, q2 = l >> 3; // pass-2 lane = (l1, q)
#pragma unroll
  for (int l2 = 0; l2 < 8; ++l2) v[l2] = xrow(ra, rb, q2)[l1 + 8 * (l2 ^ q2)];
  dft8(v);
#pragma unroll
  for (int p1 = 1; p1 < 8; ++p1) v[p1] = cmul(v[p1], sm.u.fq.tw2[p1 * 8 + l1]);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // exchange 2: lane (l1, q) writes U[p1] at row q, col swz2(q, l1, p1)
#pragma unroll
  for (int p1 = 0; p1 < 8; ++p1) xrow(ra, rb, q2)[swz2(q2, l1, p1)] = v[p1];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int p1 = l & 7, q3 = l >> 3; // pass-3 lane = (p1, q)
#pragma unroll
  for (int a = 0; a < 8; ++a) v[a] = xrow(ra, rb, q3)[swz2(q3, a, p1)];
  dft8(v); // v[p2] = X[q3 + 8 p1 + 64 p2]
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
  for (int p2 = 0; p2 < 8; ++p2) {
    const int n = q3 + 8 * p1 + 64 * p2;
    const int s = spec_idx(n);
    xrow(ra, rb, s >> 6)[s & 63] = v[p2];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
__device__ __forceinline__ float2 spec_read(const float2 *ra, const float2 *rb, int n) {
  const int s = spec_idx(n & 511);
  return (s < 256 ? ra : rb)[s & 255];
}

// ---------------------------------------------------------------------------
// Constellation decision (modem.js:140-150) and its distance to the nearest
// decision boundary. Ties resolve to the lowest index like the reference loop.
__device__ __forceinline__ int decide(int mod, float cr, float ci, float &margin) {
  if (mod == AMOD_BPSK) { margin = fabsf(cr); return cr < 0.f ? 1 : 0; }
  if (mod == AMOD_QPSK) {
    margin = fminf(fabsf(cr), fabsf(ci));
    const int re_neg = cr < 0.f, im_neg = ci < 0.f;
    return im_neg ? (re_neg ? 2 : 3) : (re_neg ? 1 : 0);
  }
  const float t = 0.63245553203367587f; // 2/sqrt(10): midpoint of the -3/-1 and 1/3 levels
  // col order of the Gray-coded levels: col0 -3, col1 -1, col2 +3, col3 +1
  const int col = cr < -t ? 0 : (cr < 0.f ? 1 : (cr < t ? 3 : 2));
  const int row = ci < -t ? 0 : (ci < 0.f ? 1 : (ci < t ? 3 : 2));
  const float mr = fminf(fabsf(cr), fabsf(fabsf(cr) - t));
  const float mi = fminf(fabsf(ci), fabsf(fabsf(ci) - t));
  margin = fminf(mr, mi);
  return 4 * row + col;
}

__device__ __forceinline__ void block_reduce_begin() { __syncthreads(); }

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_decode_fast(const DevCfg cfg, const DevWork w) {
  __shared__ Smem sm;
  const int f = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t off = w.off[f];
  const int N = w.len[f];
  const int SYM = cfg.sym, CP = cfg.cp;
  const bool dbg = w.dbg != nullptr;
  amod_debug *D = dbg ? w.dbg + f : nullptr;

  // ------------------------------------------------ routing to the exact path
  {
    int route = 0;
    if (w.options & AMOD_OPT_FORCE_EXACT) route = AMOD_FLAG_FORCED;
    else if (N > CAP - 8) route = AMOD_FLAG_BIG;
    if (route) {
      if (tid == 0) {
        const int i = atomicAdd(w.fb_count, 1);
        w.fb_list[i] = f;
        w.fb_flags[i] = route;
      }
      return;
    }
  }

  // ------------------------------------------------ stage 0: load + stats
  const int64_t a0 = off & ~int64_t(3);
  const int ph = (int)(off - a0);
  const int nvec = (ph + N + 3) >> 2;
  double s = 0.0;
  float mn = INFINITY, mxv = -INFINITY;
  int nonfinite = 0;
  const float *src = w.samples + a0;
  for (int v = tid; v < nvec; v += WG) {
    const int i0 = 4 * v - ph; // frame index of component 0
    float4 q;
    if (i0 >= 0 && i0 + 4 <= N) {
      q = *reinterpret_cast<const float4 *>(src + 4 * v);
    } else {
      q.x = (i0 + 0 >= 0 && i0 + 0 < N) ? src[4 * v + 0] : 0.f;
      q.y = (i0 + 1 >= 0 && i0 + 1 < N) ? src[4 * v + 1] : 0.f;
      q.z = (i0 + 2 >= 0 && i0 + 2 < N) ? src[4 * v + 2] : 0.f;
      q.w = (i0 + 3 >= 0 && i0 + 3 < N) ? src[4 * v + 3] : 0.f;
    }
    *reinterpret_cast<float4 *>(&sm.x[4 * v]) = q;
    const float c[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j;
      if (i >= 0 && i < N) {
        s += (double)c[j];
        mn = fminf(mn, c[j]);
        mxv = fmaxf(mxv, c[j]);
        nonfinite |= !isfinite(c[j]);
      }
    }
  }
  s = wave_sum(s);
  mn = wave_min(mn);
  mxv = wave_max(mxv);
  nonfinite = wave_or(nonfinite);
  if (lane == 0) { sm.rd[wave] = s; sm.rf[wave] = mn; sm.rf[NWAVE + wave] = mxv; sm.ri[wave] = nonfinite; }
  __syncthreads();
  if (tid == 0) {
    double S = 0.0;
    float MN = INFINITY, MX = -INFINITY;
    int NF = 0;
    for (int i = 0; i < NWAVE; ++i) {
      S += sm.rd[i]; MN = fminf(MN, sm.rf[i]); MX = fmaxf(MX, sm.rf[NWAVE + i]); NF |= sm.ri[i];
    }
    int flags = NF ? AMOD_FLAG_NONFINITE : 0;
    float A = 1.f, B = 0.f;
    double mean = 0.0, mx = 0.0;
    if (cfg.mode == AMOD_MODE_RECEIVED && N > 0) {
      mean = S / (double)N;
      // max |f32(x - mean)| is reached at the extremes: rounding to f32 is monotone
      mx = fmax(fabs((double)(float)((double)MX - mean)), fabs((double)(float)((double)MN - mean)));
      if (fabs(mx - 1e-6) <= 1e-6 * 1e-5) flags |= AMOD_FLAG_THRESH;
      if (mx > 1e-6) { A = (float)(1.0 / mx); B = (float)(-mean / mx); }
      else { A = 1.f; B = (float)(-mean); }
    }
    sm.n = N; sm.ph = ph; sm.flags = flags; sm.status = AMOD_OK;
    sm.A = A; sm.B = B; sm.mean = mean; sm.mx = mx;
    sm.coarse = -1; sm.clo = -1; sm.chi = -1; sm.start = 0;
    if (dbg) { D->mean = mean; D->mx = mx; }
  }
  __syncthreads();
  if (sm.flags & (AMOD_FLAG_NONFINITE | AMOD_FLAG_THRESH)) {
    if (tid == 0) {
      const int i = atomicAdd(w.fb_count, 1);
      w.fb_list[i] = f;
      w.fb_flags[i] = sm.flags;
    }
    return;
  }
  const float A = sm.A, B = sm.B;
  const float *X = sm.x + ph; // frame sample i at X[i]
  auto Y = [&](int i) -> float { return fmaf(X[i], A, B); };

  amod_result r;
  init_result(r);
  int start = 0;
  const float eps_c = 2e-3f * cfg.guard;     // Schmidl-Cox metric guard (absolute)
  const float eps_g = 1e-3f * cfg.guard;     // energy-gate guard (relative)
  const float eps_f = 1e-3f * cfg.guard;     // fine metric guard (absolute)

  if (cfg.mode == AMOD_MODE_RECEIVED) {
    // ---------------------------------------------- stage 1: Schmidl-Cox scan
    const int E = N - 512;
    if (E < 0) {
      if (tid == 0) sm.status = AMOD_E_PREAMBLE;
      __syncthreads();
    } else {
      const int NB = (N + SC_BLK - 1) / SC_BLK;
      for (int b = tid; b < NB; b += WG) {
        float zz = 0.f, ee = 0.f;
        const int i0 = b * SC_BLK;
#pragma unroll 8
        for (int j = 0; j < SC_BLK; ++j) {
          const int i = i0 + j;
          if (i < N) {
            const float yi = Y(i);
            ee = fmaf(yi, yi, ee);
            if (i < N - 256) zz = fmaf(yi, Y(i + 256), zz);
          }
        }
        sm.u.sc.bz[b] = zz;
        sm.u.sc.be[b] = ee;
      }
      __syncthreads();
      const float gate_lo = 0.01f * (1.f - eps_g), gate_hi = 0.01f * (1.f + eps_g);
      const int nseg = (E + SC_BLK) / SC_BLK;
      // pass 1: best metric (loose gate) and first index
      float best = -1.f;
      int bidx = 0x7fffffff;
      for (int g = tid; g < nseg; g += WG) {
        float p = 0.f, ra = 0.f, rb = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) { p += sm.u.sc.bz[g + k]; ra += sm.u.sc.be[g + k]; rb += sm.u.sc.be[g + 8 + k]; }
        const int d0 = g * SC_BLK;
        const int dend = min(d0 + SC_BLK - 1, E);
        for (int d = d0; d <= dend; ++d) {
          if (ra > gate_lo && rb > gate_lo) {
            const float m = (p * p) / (ra * rb);
            if (m > best) { best = m; bidx = d; }
          }
          if (d < dend) {
            const float a = Y(d), mid = Y(d + 256), bb = Y(d + 512);
            p = fmaf(mid, bb - a, p);
            ra = fmaf(-a, a, fmaf(mid, mid, ra));
            rb = fmaf(-mid, mid, fmaf(bb, bb, rb));
          }
        }
      }
      // block argmax (max value, then lowest index)
      {
        float bw = wave_max(best);
        int iw = wave_min(best == bw ? bidx : 0x7fffffff);
        if (lane == 0) { sm.rf[wave] = bw; sm.ri[wave] = iw; }
        __syncthreads();
        if (tid == 0) {
          float B2 = -1.f; int I2 = 0x7fffffff;
          for (int i = 0; i < NWAVE; ++i)
            if (sm.rf[i] > B2 || (sm.rf[i] == B2 && sm.ri[i] < I2)) { B2 = sm.rf[i]; I2 = sm.ri[i]; }
          sm.cbest = B2; sm.coarse = I2;
        }
        __syncthreads();
      }
      const float CB = sm.cbest;
      // pass 2: candidate range {d : metric >= CB - eps_c}, and gate uncertainty there
      int lo = 0x7fffffff, hi = -1, unc = 0;
      if (CB > 0.5f - eps_c) {
        for (int g = tid; g < nseg; g += WG) {
          float p = 0.f, ra = 0.f, rb = 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) { p += sm.u.sc.bz[g + k]; ra += sm.u.sc.be[g + k]; rb += sm.u.sc.be[g + 8 + k]; }
          const int d0 = g * SC_BLK;
          const int dend = min(d0 + SC_BLK - 1, E);
          for (int d = d0; d <= dend; ++d) {
            if (ra > gate_lo && rb > gate_lo) {
              const float m = (p * p) / (ra * rb);
              if (m >= CB - eps_c) {
                lo = min(lo, d); hi = max(hi, d);
                unc |= (ra <= gate_hi || rb <= gate_hi);
              }
            }
            if (d < dend) {
              const float a = Y(d), mid = Y(d + 256), bb = Y(d + 512);
              p = fmaf(mid, bb - a, p);
              ra = fmaf(-a, a, fmaf(mid, mid, ra));
              rb = fmaf(-mid, mid, fmaf(bb, bb, rb));
            }
          }
        }
      }
      lo = wave_min(lo); hi = wave_max(hi); unc = wave_or(unc);
      if (lane == 0) { sm.ri[wave] = lo; sm.ri[NWAVE + wave] = hi; sm.ri[2 * NWAVE + wave] = unc; }
      __syncthreads();
      if (tid == 0) {
        int LO = 0x7fffffff, HI = -1, U = 0;
        for (int i = 0; i < NWAVE; ++i) { LO = min(LO, sm.ri[i]); HI = max(HI, sm.ri[NWAVE + i]); U |= sm.ri[2 * NWAVE + i]; }
        int flags = sm.flags;
        if (CB < 0.5f - eps_c) sm.status = AMOD_E_PREAMBLE;          // confidently not detected
        else if (CB <= 0.5f + eps_c || U) flags |= AMOD_FLAG_COARSE;  // threshold or gate ambiguous
        else if (HI - LO > 2 * 3 * CP) flags |= AMOD_FLAG_COARSE;     // no common fine window
        sm.flags = flags; sm.clo = LO; sm.chi = HI;
        if (dbg) { D->coarse_metric = CB; D->coarse_lo = LO; D->coarse_hi = HI; }
      }
      __syncthreads();
    }
    if (sm.flags) goto to_exact;
    if (sm.status != AMOD_OK) goto finish_error;

    // ---------------------------------------------- stage 2: fine timing
    {
      const int R = 3 * CP;
      const int c_lo = sm.clo, c_hi = sm.chi;
      const int w0 = max(0, c_lo - R), w1 = min(N - SYM, c_hi + R);
      const int P = w1 - w0 + 1;
      if (P > FINE_MAX) {
        if (tid == 0) sm.flags |= AMOD_FLAG_FINE;
        __syncthreads();
        goto to_exact;
      }
      if (P <= 0) {
        if (tid == 0) sm.status = AMOD_E_LOW_CORR;
        __syncthreads();
        goto finish_error;
      }
      for (int i = tid; i < SYM; i += WG) sm.u.fine.tmpl[i] = cfg.t.pre1[i];
      __syncthreads();
      const float te = cfg.te_f;
      const int nquad = (P + 3) >> 2;
      const int split = SYM / 4; // 4 tap ranges per quad of positions
      for (int task = tid; task < nquad * 4; task += WG) {
        const int qd = task >> 2, sp = task & 3;
        const int d = w0 + 4 * qd;
        const int i0 = sp * split, i1 = (sp == 3) ? SYM : i0 + split;
        float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, e0 = 0.f;
        // sliding window of 4 samples y[d+i .. d+i+3]
        float y0 = (d + i0 + 0 < N) ? Y(d + i0 + 0) : 0.f;
        float y1 = (d + i0 + 1 < N) ? Y(d + i0 + 1) : 0.f;
        float y2 = (d + i0 + 2 < N) ? Y(d + i0 + 2) : 0.f;
        for (int i = i0; i < i1; ++i) {
          const float y3 = (d + i + 3 < N) ? Y(d + i + 3) : 0.f;
          const float t = sm.u.fine.tmpl[i];
          c0 = fmaf(y0, t, c0); c1 = fmaf(y1, t, c1); c2 = fmaf(y2, t, c2); c3 = fmaf(y3, t, c3);
          e0 = fmaf(y0, y0, e0);
          y0 = y1; y1 = y2; y2 = y3;
        }
        // combine the 4 tap ranges (lanes 4qd .. 4qd+3 are adjacent)
#pragma unroll
        for (int o = 1; o < 4; o <<= 1) {
          c0 += __shfl_xor(c0, o, 64); c1 += __shfl_xor(c1, o, 64);
          c2 += __shfl_xor(c2, o, 64); c3 += __shfl_xor(c3, o, 64);
          e0 += __shfl_xor(e0, o, 64);
        }
        if (sp == 0) {
          const float cs[4] = {c0, c1, c2, c3};
          float en = e0;
          for (int j = 0; j < 4; ++j) {
            const int dd = d + j;
            if (dd > w1) break;
            if (j > 0) { const float yo = Y(dd - 1), yn = Y(dd - 1 + SYM); en = fmaf(yn, yn, fmaf(-yo, yo, en)); }
            const float den = sqrtf(fmaxf(en, 0.f) * te);
            float m;
            if (den > 0.001f * (1.f + eps_g)) m = cs[j] / den;
            else if (den > 0.001f * (1.f - eps_g)) m = cs[j] / den + 4.f; // uncertain gate: tagged
            else m = -8.f;                                                 // gated out
            sm.u.fine.m[dd - w0] = m;
          }
        }
      }
      __syncthreads();
      // argmax (first index), second best, uncertain-gate candidates
      float b1 = -8.f; int i1x = 0x7fffffff;
      for (int k = tid; k < P; k += WG) {
        float m = sm.u.fine.m[k];
        if (m > 2.f) m -= 4.f;
        if (m > b1) { b1 = m; i1x = k; }
      }
      {
        const float bw = wave_max(b1);
        const int iw = wave_min(b1 == bw ? i1x : 0x7fffffff);
        if (lane == 0) { sm.rf[wave] = bw; sm.ri[wave] = iw; }
        __syncthreads();
        if (tid == 0) {
          float BB = -8.f; int II = 0x7fffffff;
          for (int i = 0; i < NWAVE; ++i)
            if (sm.rf[i] > BB || (sm.rf[i] == BB && sm.ri[i] < II)) { BB = sm.rf[i]; II = sm.ri[i]; }
          sm.fbest = BB; sm.start = II;
        }
        __syncthreads();
      }
      const float FB = sm.fbest;
      const int kst = sm.start;
      float b2 = -8.f; int unc = 0;
      for (int k = tid; k < P; k += WG) {
        float m = sm.u.fine.m[k];
        const bool tagged = m > 2.f;
        if (tagged) m -= 4.f;
        if (k != kst) b2 = fmaxf(b2, m);
        if (tagged && m >= FB - eps_f) unc = 1;
      }
      b2 = wave_max(b2); unc = wave_or(unc);
      if (lane == 0) { sm.rf[wave] = b2; sm.ri[wave] = unc; }
      __syncthreads();
      if (tid == 0) {
        float B2 = -8.f; int U = 0;
        for (int i = 0; i < NWAVE; ++i) { B2 = fmaxf(B2, sm.rf[i]); U |= sm.ri[i]; }
        const int dstar = w0 + kst;
        int flags = sm.flags;
        if (FB <= -7.f) {
          if (U) flags |= AMOD_FLAG_FINE; else sm.status = AMOD_E_LOW_CORR; // nothing passed the gate
        } else if (FB < 0.1f - eps_f && !U) {
          sm.status = AMOD_E_LOW_CORR;
        } else if (FB <= 0.1f + eps_f || U || FB - B2 <= eps_f || dstar < c_hi - R || dstar > c_lo + R) {
          flags |= AMOD_FLAG_FINE;
        }
        sm.flags = flags;
        sm.start = dstar;
        if (dbg) { D->fine_metric = FB; D->fine_idx = dstar; }
      }
      __syncthreads();
      if (sm.flags) goto to_exact;
      if (sm.status != AMOD_OK) goto finish_error;
      start = sm.start;
      r.fine_metric = sm.fbest;
      r.coarse_idx = sm.coarse;
      r.preamble_idx = start;
    }
    // CE / data checks (modem.js:591-600)
    if (start + 3 * SYM > N) { if (tid == 0) sm.status = AMOD_E_SHORT_CE; __syncthreads(); goto finish_error; }
    if (start + 3 * SYM >= N) { if (tid == 0) sm.status = AMOD_E_NO_DATA; __syncthreads(); goto finish_error; }
  } else {
    // decodeChunkFrame checks (modem.js:774-786)
    if (3 * SYM > N) { if (tid == 0) sm.status = AMOD_E_FRAME_SHORT_CE; __syncthreads(); goto finish_error; }
    if (3 * SYM >= N) { if (tid == 0) sm.status = AMOD_E_NO_DATA; __syncthreads(); goto finish_error; }
  }

  // ------------------------------------------------ stage 3: FFT jobs
  {
    const int ce0 = start + 2 * SYM, data0 = start + 3 * SYM;
    const int M = (N - data0) / SYM; // data symbols decoded (whole symbols to the end)
    const int nbits = M * cfg.ndata * cfg.bps;
    const int nwords = (nbits + 31) >> 5;
    // tables + clear bit array
    for (int i = tid; i < 8 * 64; i += WG) sm.u.fq.tw1[i] = cfg.t.tw1[i];
    for (int i = tid; i < 64; i += WG) sm.u.fq.tw2[i] = cfg.t.tw2[i];
    for (int i = tid; i < nwords; i += WG) sm.u.fq.bits[i] = 0u;
    if (tid == 0) { sm.nsym = M; sm.data0 = data0; sm.gmax = 0.f; sm.zce = 0.f; }
    if (nbits > MAX_BITS_WORDS * 32) { if (tid == 0) sm.flags |= AMOD_FLAG_BIG; }
    __syncthreads();
    if (sm.flags) goto to_exact;
    const bool odd = (M & 1) != 0;
    const int njobs = 1 + (M - (odd ? 1 : 0)) / 2;
    const int nband = cfg.nband;
    float gmax_local = 0.f;
    int wflags = 0;

    for (int round = 0; round * NWAVE < njobs; ++round) {
      const int job = round * NWAVE + wave;
      const bool active = job < njobs;
      // symbols of this job: job 0 = (CE, last odd symbol or none), job j = (2j-2, 2j-1)
      int s1 = -1, s2 = -1; // data-symbol indices; s1 = -2 marks the CE symbol
      if (active) {
        if (job == 0) { s1 = -2; s2 = odd ? M - 1 : -1; }
        else { s1 = 2 * job - 2; s2 = 2 * job - 1; }
      }
      const int pos1 = s1 == -2 ? ce0 : data0 + s1 * SYM;
      const int pos2 = s2 >= 0 ? data0 + s2 * SYM : start + SYM; // pre2 slot when absent
      // exchange regions: 2 KB, 8-byte aligned, inside each symbol's sample slot
      float2 *ra = reinterpret_cast<float2 *>(
          reinterpret_cast<uintptr_t>(&sm.x[ph + pos1] + 1) & ~uintptr_t(7));
      float2 *rb = reinterpret_cast<float2 *>(
          reinterpret_cast<uintptr_t>(&sm.x[ph + pos2] + 1) & ~uintptr_t(7));
      float2 v[8];
      int const1 = 0, const2 = 0;
      if (active) {
        float mn1 = INFINITY, mx1 = -INFINITY, mn2 = INFINITY, mx2 = -INFINITY;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const int i = CP + lane + 64 * m;
          const float r1 = X[pos1 + i];
          const float r2 = s2 >= 0 ? X[pos2 + i] : 0.f;
          mn1 = fminf(mn1, r1); mx1 = fmaxf(mx1, r1); mn2 = fminf(mn2, r2); mx2 = fmaxf(mx2, r2);
          v[m] = make_float2(fmaf(r1, A, B), s2 >= 0 ? fmaf(r2, A, B) : 0.f);
        }
        const1 = wave_min(mn1) == wave_max(mx1);
        const2 = wave_min(mn2) == wave_max(mx2);
        fft512_wave(v, ra, rb, sm);
        if (job == 0) {
          // channel estimate from the CE symbol: H = Y * known (X = +-1, modem.js:431-438)
          float zmax = 0.f;
          for (int b = lane; b < nband; b += 64) {
            const int k = cfg.sub_start + b;
            const float2 zk = spec_read(ra, rb, k), zn = spec_read(ra, rb, kFft - k);
            zmax = fmaxf(zmax, fmaxf(fabsf(zk.x) + fabsf(zk.y), fabsf(zn.x) + fabsf(zn.y)));
          }
          zmax = wave_max(zmax);
          for (int b = lane; b < nband; b += 64) {
            const int k = cfg.sub_start + b;
            float2 h = make_float2(0.f, 0.f);
            if (!const1) {
              const float2 zk = spec_read(ra, rb, k), zn = spec_read(ra, rb, kFft - k);
              const float2 y = make_float2(0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y));
              const float kn = cfg.t.known[b];
              h = make_float2(y.x * kn, y.y * kn);
            }
            const float m2 = h.x * h.x + h.y * h.y;
            float2 g;
            if (m2 > 1e-10f) g = make_float2(h.x / m2, -h.y / m2);
            else g = make_float2(1.f, 0.f);
            // |H|^2 close to 1e-10 (or tiny but non-zero) decides passthrough differently
            if (!const1 && m2 < 1e-6f) wflags |= AMOD_FLAG_CHANNEL;
            sm.u.fq.g[b] = g;
            gmax_local = fmaxf(gmax_local, fabsf(g.x) + fabsf(g.y));
            if (dbg) { D->h_re[b] = h.x; D->h_im[b] = h.y; }
          }
          if (lane == 0) sm.zce = zmax;
        }
      }
      if (round == 0) {
        // publish G, |G|max and the CE spectrum scale to every wave
        gmax_local = wave_max(gmax_local);
        if (wave == 0 && lane == 0) sm.gmax = gmax_local;
        __syncthreads();
      }
      if (!active) continue;
      const float gmax = sm.gmax, zce = sm.zce;
      // ---- per data symbol of this job: equalise, pilot phase, demap
      for (int which = 0; which < 2; ++which) {
        const int sidx = which == 0 ? s1 : s2;
        if (sidx < 0) continue; // CE or absent
        const bool cst = which == 0 ? const1 : const2;
        uint32_t *bits = sm.u.fq.bits;
        const int sbase = sidx * cfg.ndata * cfg.bps;
        if (cst) {
          // constant window: every bin is exactly 0 in the reference -> origin decision
          for (int b = lane; b < nband; b += 64) {
            const int di = cfg.t.band_di[b];
            if (di < 0) continue;
            const int pos = sbase + di * cfg.bps;
            const uint32_t val = (uint32_t)cfg.origin_idx << (32 - cfg.bps - (pos & 31));
            if (val) atomicOr(&bits[pos >> 5], val);
          }
          if (dbg && sidx < AMOD_DBG_SYMS) if (lane == 0) D->phase[sidx] = 0.0;
          if (dbg && sidx == 0)
            for (int b = lane; b < nband; b += 64) { D->x_re[b] = 0; D->x_im[b] = 0; D->eq_re[b] = 0; D->eq_im[b] = 0; }
          continue;
        }
        float2 eq[4];
        float zmax = 0.f, emax = 0.f;
        float psum = 0.f, perr = 0.f;
        int pcnt = 0, pflag = 0;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = lane + 64 * rr;
          eq[rr] = make_float2(0.f, 0.f);
          if (b < nband) {
            const int k = cfg.sub_start + b;
            const float2 zk = spec_read(ra, rb, k), zn = spec_read(ra, rb, kFft - k);
            zmax = fmaxf(zmax, fmaxf(fabsf(zk.x) + fabsf(zk.y), fabsf(zn.x) + fabsf(zn.y)));
            const float2 xs = which == 0 ? make_float2(0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y))
                                         : make_float2(0.5f * (zk.y + zn.y), 0.5f * (zn.x - zk.x));
            const float2 g = sm.u.fq.g[b];
            eq[rr] = cmul(xs, g);
            emax = fmaxf(emax, fabsf(eq[rr].x) + fabsf(eq[rr].y));
            if (dbg && sidx == 0) { D->x_re[b] = xs.x; D->x_im[b] = xs.y; D->eq_re[b] = eq[rr].x; D->eq_im[b] = eq[rr].y; }
          }
        }
        zmax = wave_max(zmax);
        emax = wave_max(emax);
        // error bound of eq (fp32 FFT + channel estimate), see DESIGN.md §guards
        const float delta = 2e-6f * cfg.guard * (zmax + emax * zce) * gmax + 1e-12f;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = lane + 64 * rr;
          if (b < nband && cfg.t.band_di[b] < 0) {
            const float er = eq[rr].x, ei = eq[rr].y;
            const float aer = fabsf(er);
            if (aer > 1e-6f) {
              psum += ei / er;
              pcnt += 1;
              perr += delta * (1.f / aer + fabsf(ei) / (aer * aer));
            }
            if (fabsf(aer - 1e-6f) <= 2.f * delta + 1e-7f) pflag = 1;
          }
        }
        psum = wave_sum(psum); perr = wave_sum(perr); pcnt = wave_sum(pcnt); pflag = wave_or(pflag);
        const float phase = pcnt > 0 ? psum / (float)pcnt : 0.f;
        const float dphase = pcnt > 0 ? perr / (float)pcnt : 0.f;
        if (pflag) wflags |= AMOD_FLAG_PHASE;
        if (dbg && sidx < AMOD_DBG_SYMS && lane == 0) D->phase[sidx] = phase;
        const float tau = 4.f * (delta * (1.f + fabsf(phase)) + emax * dphase) + 1e-9f;
        int dflag = 0;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = lane + 64 * rr;
          if (b >= nband) continue;
          const int di = cfg.t.band_di[b];
          if (di < 0) continue;
          const float cr = fmaf(eq[rr].y, phase, eq[rr].x);
          const float ci = fmaf(-eq[rr].x, phase, eq[rr].y);
          float margin;
          const int idx = decide(cfg.mod, cr, ci, margin);
          dflag |= margin <= tau;
          const int pos = sbase + di * cfg.bps;
          const uint32_t val = (uint32_t)idx << (32 - cfg.bps - (pos & 31));
          if (val) atomicOr(&bits[pos >> 5], val);
        }
        if (wave_or(dflag)) wflags |= AMOD_FLAG_DEMAP;
      }
    }
    wflags = wave_or(wflags);
    if (lane == 0 && wflags) atomicOr(&sm.flags, wflags);
    __syncthreads();
    if (sm.flags) goto to_exact;
    // ------------------------------------------------ stage 4: finish
    {
      r.nbits = nbits;
      if (dbg && tid == 0) D->nsym = M;
      const uint32_t *v = sm.u.fq.bits;
      int nv = nbits;
      if (cfg.rep > 1) {
        uint32_t *voted = reinterpret_cast<uint32_t *>(sm.x); // samples are dead now
        nv = block_vote(sm.u.fq.bits, nbits, cfg.rep, voted);
        __syncthreads();
        v = voted;
      }
      r.flags = 0;
      finish_frame(v, nv, cfg, r, w.res + f, w.payload + (int64_t)f * w.stride, w.stride, sm.ru, nullptr);
      return;
    }
  }

finish_error:
  if (tid == 0) {
    r.status = sm.status;
    if (cfg.mode == AMOD_MODE_RECEIVED) {
      r.coarse_idx = sm.status == AMOD_E_PREAMBLE ? -1 : sm.coarse;
      r.fine_metric = sm.status == AMOD_E_PREAMBLE ? 0.f : sm.fbest;
    }
    r.preamble_idx = -1;
    w.res[f] = r;
  }
  return;

to_exact:
  if (tid == 0) {
    const int i = atomicAdd(w.fb_count, 1);
    w.fb_list[i] = f;
    w.fb_flags[i] = sm.flags;
  }
}

} // namespace
} // namespace amod

extern "C" hipError_t amod_launch_fast(const amod::DevCfg &cfg, const amod::DevWork &w, hipStream_t s) {
  if (w.nframes <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_decode_fast, dim3(w.nframes), dim3(amod::WG), 0, s, cfg, w);
  return hipGetLastError();
}
extern "C" int amod_fast_capacity(void) { return amod::CAP - 8; }
