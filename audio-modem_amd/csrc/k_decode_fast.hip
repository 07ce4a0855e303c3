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

constexpr int WG = 1024;                   // 16 waves (128 VGPRs each)
constexpr int NWAVE = WG / 64;
constexpr int SC_BLK = 32;                 // Schmidl-Cox block / segment length
constexpr int UNION_BYTES = 14848;         // stage-shared scratch
constexpr int CAP = 36736;                 // max samples per LDS-resident frame
constexpr int PFV = (CAP + 8 + 4 * WG - 1) / (4 * WG); // float4 vectors per lane per frame
constexpr int PF = PFV;                    // all issued before the first use: full memory-level parallelism
constexpr int MAX_BITS_WORDS = 1640;       // 64 symbols x 820 bits
constexpr int FINE_MAX = 1008;             // max fine-search positions (else exact)
constexpr int SC_NB = (CAP + 31) / 32 + 8; // Schmidl-Cox blocks (k-space), with slack
constexpr int SC_MAXCAND = 256;            // blocks slid position by position (else exact)

struct alignas(16) Smem {
  float x[CAP + 16];                       // raw samples: x[ph + i] is frame sample i
  union alignas(16) U {
    struct { float bz[SC_NB]; float be[SC_NB]; float ba[SC_NB]; int16_t cand[SC_MAXCAND]; } sc; // stage 1
    struct { float tmpl[768]; float m[FINE_MAX]; float yw[FINE_MAX + 776]; } fine; // stage 2
    struct {                                                      // stage 3
      float2 tw1[8 * 64];
      float2 tw2[8 * 8];
      float2 g[kMaxBand];                  // conj(H)/|H|^2 (or 1 for passthrough)
      uint32_t bits[MAX_BITS_WORDS];
      float known[kMaxBand];               // CE symbol signs, band order
      int16_t band_di[kMaxBand];           // data-subcarrier index, -1 for pilots
    } fq;
    unsigned char raw[UNION_BYTES];
  } u;
  float rf[4 * NWAVE];
  int ri[4 * NWAVE];
  double rd[2 * NWAVE];
  uint32_t ru[16];
  // per-frame scalars (written by one thread, read after a barrier)
  int n, ph, status, flags, coarse, clo, chi, start, nsym, data0, ncand;
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

// Exchange buffer of one FFT job: 8 rows of 64 float2; rows 0-3 live at float2
// index a of the LDS sample array, rows 4-7 at index b (each inside one symbol's
// sample slot). Plain 32-bit LDS indices keep every access a ds_read/ds_write.
struct XB {
  int a, b;
};
__device__ __forceinline__ int xrow(const XB &x, int row) { return (row < 4 ? x.a : x.b) + (row & 3) * 64; }
__device__ __forceinline__ int swz2(int q, int l1, int p1) { // exchange-2 column swizzle
  return 8 * ((l1 ^ q) & 7) + ((p1 ^ ((q & 3) + 4 * (l1 >> 2))) & 7);
}
__device__ __forceinline__ int spec_idx(int n) { return n ^ (((n >> 5) & 1) << 2); }

// One wave: 512-pt complex FFT of z (lane l holds z[l + 64 m] in v[m]); result
// X[n] left in the exchange buffer at row spec_idx(n)>>6, col spec_idx(n)&63.
__device__ void fft512_wave(float2 (&v)[8], const XB xb, Smem &sm) {
  float2 *const X2 = reinterpret_cast<float2 *>(sm.x);
  int l = wave_lane();
  // keep the lane-derived swizzle indices inside the job loop: hoisted out of it
  // they occupy ~40 VGPRs for the whole stage and force spills
  asm volatile("" : "+v"(l));
  dft8(v);
#pragma unroll
  for (int q = 1; q < 8; ++q) v[q] = cmul(v[q], sm.u.fq.tw1[q * 64 + l]);
  // exchange 1: row q, col l ^ (q<<3)
#pragma unroll
  for (int q = 0; q < 8; ++q) X2[xrow(xb, q) + (l ^ (q << 3))] = v[q];
  __builtin_amdgcn_wave_barrier();
  const int l1 = l & 7, q2 = l >> 3; // pass-2 lane = (l1, q)
  const int r2 = xrow(xb, q2);
#pragma unroll
  for (int l2 = 0; l2 < 8; ++l2) v[l2] = X2[r2 + l1 + 8 * (l2 ^ q2)];
  dft8(v);
#pragma unroll
  for (int p1 = 1; p1 < 8; ++p1) v[p1] = cmul(v[p1], sm.u.fq.tw2[p1 * 8 + l1]);
  __builtin_amdgcn_wave_barrier();
  // exchange 2: lane (l1, q) writes U[p1] at row q, col swz2(q, l1, p1)
#pragma unroll
  for (int p1 = 0; p1 < 8; ++p1) X2[r2 + swz2(q2, l1, p1)] = v[p1];
  __builtin_amdgcn_wave_barrier();
  const int p1 = l & 7; // pass-3 lane = (p1, q), same row as pass 2
#pragma unroll
  for (int a = 0; a < 8; ++a) v[a] = X2[r2 + swz2(q2, a, p1)];
  dft8(v); // v[p2] = X[q2 + 8 p1 + 64 p2]
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int p2 = 0; p2 < 8; ++p2) {
    const int s = spec_idx(q2 + 8 * p1 + 64 * p2);
    X2[xrow(xb, s >> 6) + (s & 63)] = v[p2];
  }
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ float2 spec_read(const Smem &sm, const XB &xb, int n) {
  const int s = spec_idx(n & 511);
  return reinterpret_cast<const float2 *>(sm.x)[(s < 256 ? xb.a : xb.b) + (s & 255)];
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
// Frame prefetch: the next frame's samples travel HBM -> VGPRs (PF float4 per
// lane) while the current frame's FFT/demap/CRC stages run from LDS, so the
// HBM stream overlaps compute. Routing decisions that need no samples (forced
// exact, frame longer than LDS) are taken here.
__device__ __forceinline__ int frame_route(const DevWork &w, int N) {
  if (w.options & AMOD_OPT_FORCE_EXACT) return AMOD_FLAG_FORCED;
  if (N > CAP - 8) return AMOD_FLAG_BIG;
  return 0;
}

// float4 vector v of a frame (aligned base a0 = off & ~3), zero outside [0, N)
__device__ __forceinline__ float4 load_vec(const float *src, int v, int ph, int N) {
  const int i0 = 4 * v - ph; // frame index of component 0
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 >= 0 && i0 + 4 <= N) {
    t = *reinterpret_cast<const float4 *>(src + 4 * v);
  } else {
    if (i0 + 0 >= 0 && i0 + 0 < N) t.x = src[4 * v + 0];
    if (i0 + 1 >= 0 && i0 + 1 < N) t.y = src[4 * v + 1];
    if (i0 + 2 >= 0 && i0 + 2 < N) t.z = src[4 * v + 2];
    if (i0 + 3 >= 0 && i0 + 3 < N) t.w = src[4 * v + 3];
  }
  return t;
}

__device__ __forceinline__ void pf_issue(const DevWork &w, int g, float4 (&q)[PF]) {
  if (g >= w.nframes) return;
  const int64_t off = w.off[g];
  const int N = w.len[g];
  if (frame_route(w, N)) return;
  const int ph = (int)(off & 3);
  const int nvec = (ph + N + 3) >> 2;
  const float *src = w.samples + (off - ph);
  const int tid = ltid();
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int v = tid + WG * j;
    q[j] = v < nvec ? load_vec(src, v, ph, N) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// stage 0: registers -> LDS, preprocessSignal statistics (modem.js:213-232):
// fp64 sum, min, max; sets the per-frame scalars in LDS. Whole workgroup.
__device__ __forceinline__ void stage_in(const DevCfg &cfg, const DevWork &w, int f, const float4 (&q)[PF], Smem &sm) {
  const int tid = ltid(), lane = tid & 63, wave = tid >> 6;
  const int64_t off = w.off[f];
  const int N = w.len[f];
  const int route = frame_route(w, N);
  const int ph = (int)(off & 3);
  const int nvec = (ph + N + 3) >> 2;
  double s = 0.0;
  float mn = INFINITY, mxv = -INFINITY;
  int nonfinite = 0;
  if (!route) {
    const float *src = w.samples + (off - ph);
#pragma unroll
    for (int j = 0; j < PFV; ++j) {
      const int v = tid + WG * j;
      if (v < nvec) {
        const float4 t = j < PF ? q[j] : load_vec(src, v, ph, N);
        *reinterpret_cast<float4 *>(&sm.x[4 * v]) = t;
        const int i0 = 4 * v - ph;
        const float c[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = i0 + k;
          if (i >= 0 && i < N) {
            s += (double)c[k];
            mn = fminf(mn, c[k]);
            mxv = fmaxf(mxv, c[k]);
            nonfinite |= !isfinite(c[k]);
          }
        }
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
    if (route) flags = route;
    sm.n = N; sm.ph = ph; sm.flags = flags; sm.status = AMOD_OK;
    sm.A = A; sm.B = B; sm.mean = mean; sm.mx = mx;
    sm.coarse = -1; sm.clo = -1; sm.chi = -1; sm.start = 0; sm.fbest = 0.f;
    if (w.dbg && !route) { w.dbg[f].mean = mean; w.dbg[f].mx = mx; }
  }
  __syncthreads();
}

// Stages 1-4 of one frame already staged in LDS by stage_in. `issue_prefetch`
// is called once the stage no longer issues vector-memory loads it waits on
// (after the FFT tables are staged), so the next frame streams in behind it.
// diagnostics only (AMOD_STAMPS): wave 0's shader-clock timeline of a frame
#define STAMP(k)                                                                        \
  do {                                                                                  \
    if (w.stamps && tid == 0) w.stamps[(int64_t)f * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

template <typename Issue>
__device__ __forceinline__ void process_frame(const DevCfg &cfg, const DevWork &w, const int f, Smem &sm,
                                              Issue &&issue_prefetch) {
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid)); // per-frame lane id: nothing lane-derived is hoisted out of the frame loop
  const int lane = tid & 63, wave = tid >> 6;
  const int N = sm.n, ph = sm.ph;
  const int SYM = cfg.sym, CP = cfg.cp;
  const bool dbg = w.dbg != nullptr;
  amod_debug *D = dbg ? w.dbg + f : nullptr;
  if (sm.flags) { // forced / too long / NaN-Inf / peak at threshold
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

  STAMP(1);
  if (cfg.stop_after == 0) return;
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
      // Blocks of 32 in LDS-index space k = ph + i (so every block starts 16-byte aligned);
      // window sums at block starts come from 8 block sums, and per-block bounds
      // |p| <= |p_c| + A_c + A_{c+8}, ra >= ra_c - E_c, rb >= rb_c - E_{c+8} cap the metric
      // of every position in the block. Only blocks whose cap can reach the best
      // block-start metric are slid through position by position.
      const int NB = (ph + N + SC_BLK - 1) / SC_BLK;
      const int klo = ph, khi_e = ph + N, khi_z = ph + N - 256; // valid k ranges for e and z
      for (int t = tid; t < NB * 4; t += WG) {
        const int k0 = 8 * t;
        float4 a0 = *reinterpret_cast<const float4 *>(&sm.x[k0]);
        float4 a1 = *reinterpret_cast<const float4 *>(&sm.x[k0 + 4]);
        float4 b0 = *reinterpret_cast<const float4 *>(&sm.x[k0 + 256]);
        float4 b1 = *reinterpret_cast<const float4 *>(&sm.x[k0 + 260]);
        const float ua[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float ub[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        float zz = 0.f, ee = 0.f, za = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = k0 + j;
          const float ya = (k >= klo && k < khi_e) ? fmaf(ua[j], A, B) : 0.f;
          const float yb = (k + 256 < khi_e) ? fmaf(ub[j], A, B) : 0.f;
          const float z = (k >= klo && k < khi_z) ? ya * yb : 0.f;
          ee = fmaf(ya, ya, ee);
          zz += z;
          za += fabsf(z);
        }
#pragma unroll
        for (int o = 1; o < 4; o <<= 1) {
          zz += __shfl_xor(zz, o, 64); ee += __shfl_xor(ee, o, 64); za += __shfl_xor(za, o, 64);
        }
        if ((t & 3) == 0) { sm.u.sc.bz[t >> 2] = zz; sm.u.sc.be[t >> 2] = ee; sm.u.sc.ba[t >> 2] = za; }
      }
      if (cfg.stop_after == 10) return;
      if (tid == 0) sm.ncand = 0;
      __syncthreads();
      STAMP(2);
      const float gate_lo = 0.01f * (1.f - eps_g), gate_hi = 0.01f * (1.f + eps_g);
      const int ncb = (E + ph) / SC_BLK + 1; // blocks holding at least one position d in [0, E]
      // (a) exact window sums at block starts -> lower bound L on the best metric
      float lmax = -1.f;
      for (int c = tid; c < ncb; c += WG) {
        float p = 0.f, ra = 0.f, rb = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) { p += sm.u.sc.bz[c + q]; ra += sm.u.sc.be[c + q]; rb += sm.u.sc.be[c + 8 + q]; }
        if (SC_BLK * c - ph >= 0 && ra > gate_lo && rb > gate_lo) lmax = fmaxf(lmax, (p * p) / (ra * rb));
      }
      lmax = wave_max(lmax);
      if (lane == 0) sm.rf[wave] = lmax;
      __syncthreads();
      float Lb = -1.f;
      for (int i = 0; i < NWAVE; ++i) Lb = fmaxf(Lb, sm.rf[i]);
      // (b) blocks whose cap reaches Lb - eps_c become candidates
      for (int c = tid; c < ncb; c += WG) {
        float p = 0.f, ra = 0.f, rb = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) { p += sm.u.sc.bz[c + q]; ra += sm.u.sc.be[c + q]; rb += sm.u.sc.be[c + 8 + q]; }
        const float e0 = sm.u.sc.be[c], e8 = sm.u.sc.be[c + 8], e16 = c + 16 < NB ? sm.u.sc.be[c + 16] : 0.f;
        const float ra_hi = ra + e8, rb_hi = rb + e16, ra_lo = ra - e0, rb_lo = rb - e8;
        if (!(ra_hi > gate_lo && rb_hi > gate_lo)) continue; // every position gated out
        bool cand = true;
        if (ra_lo > 0.f && rb_lo > 0.f) {
          const float pm = fabsf(p) + sm.u.sc.ba[c] + sm.u.sc.ba[c + 8];
          cand = (pm * pm) * 1.0001f >= (Lb - eps_c) * (ra_lo * rb_lo);
        }
        if (cand) {
          const int slot = atomicAdd(&sm.ncand, 1);
          if (slot < SC_MAXCAND) sm.u.sc.cand[slot] = (int16_t)c;
        }
      }
      __syncthreads();
      STAMP(3);
      if (cfg.stop_after == 11) return;
      const int ncand = sm.ncand;
      if (ncand > SC_MAXCAND) { // too many blocks near the best: leave it to the exact path
        if (tid == 0) sm.flags |= AMOD_FLAG_COARSE;
        __syncthreads();
        goto to_exact;
      }
      // (c) every position of a candidate block: one 32-lane group per block; the
      // window sums at position d0 + j are the block-start sums plus an exclusive
      // prefix (across the group) of the per-position slide increments
      auto cand_eval = [&](int cidx, float &m, int &d, float &ra, float &rb) -> bool {
        const int j = lane & 31;
        const int c = sm.u.sc.cand[cidx];
        float p = 0.f;
        ra = 0.f; rb = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) { p += sm.u.sc.bz[c + q]; ra += sm.u.sc.be[c + q]; rb += sm.u.sc.be[c + 8 + q]; }
        d = SC_BLK * c - ph + j;
        const float y0 = (d >= 0 && d < N) ? Y(d) : 0.f;
        const float y1 = (d + 256 < N) ? Y(d + 256) : 0.f;
        const float y2 = (d + 512 < N) ? Y(d + 512) : 0.f;
        const float z0 = (d >= 0 && d < N - 256) ? y0 * y1 : 0.f;
        const float z1 = (d + 256 < N - 256) ? y1 * y2 : 0.f;
        const float vp = z1 - z0, va = fmaf(y1, y1, -y0 * y0), vb = fmaf(y2, y2, -y1 * y1);
        float sp = vp, sa = va, sb = vb; // inclusive scans over the 32-lane group
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const float tp = __shfl_up(sp, o, 32), ta = __shfl_up(sa, o, 32), tb = __shfl_up(sb, o, 32);
          if (j >= o) { sp += tp; sa += ta; sb += tb; }
        }
        p += sp - vp; ra += sa - va; rb += sb - vb;
        const bool ok = d >= 0 && d <= E && ra > gate_lo && rb > gate_lo;
        m = ok ? (p * p) / (ra * rb) : -1.f;
        return ok;
      };
      float best = -1.f;
      int bidx = 0x7fffffff;
      for (int g = 2 * wave + (lane >> 5); g - (lane >> 5) < ncand; g += 2 * NWAVE) {
        if (g < ncand) {
          float m, ra, rb;
          int d;
          if (cand_eval(g, m, d, ra, rb) && (m > best || (m == best && d < bidx))) { best = m; bidx = d; }
        } // a group's 32 lanes share g, so the width-32 shuffles stay inside active lanes
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
      STAMP(4);
      if (cfg.stop_after == 12) return;
      const float CB = sm.cbest;
      // candidate range {d : metric >= CB - eps_c}, and gate uncertainty there
      int lo = 0x7fffffff, hi = -1, unc = 0;
      if (CB > 0.5f - eps_c) {
        for (int g = 2 * wave + (lane >> 5); g - (lane >> 5) < ncand; g += 2 * NWAVE) {
          if (g < ncand) {
            float m, ra, rb;
            int d;
            if (cand_eval(g, m, d, ra, rb) && m >= CB - eps_c) {
              lo = min(lo, d); hi = max(hi, d);
              unc |= (ra <= gate_hi || rb <= gate_hi);
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
    STAMP(5);
    if (cfg.stop_after == 1) return;

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
      // template + the normalised search window, staged once in LDS
      for (int i = tid; i < SYM; i += WG) sm.u.fine.tmpl[i] = cfg.t.pre1[i];
      const int span = P + SYM + 8;
      for (int j = tid; j < span; j += WG) sm.u.fine.yw[j] = (w0 + j < N) ? Y(w0 + j) : 0.f;
      __syncthreads();
      const float te = cfg.te_f;
      const int nquad = (P + 3) >> 2;
      const int L8 = (SYM / 8) | 1; // odd split length spreads the 8 splits over LDS banks
      const float *yw = sm.u.fine.yw;
      const float *tm = sm.u.fine.tmpl;
      // lane = (quad of 4 positions, one of 8 tap ranges); 4 correlations + 1 energy per tap
      for (int task = tid; task < nquad * 8; task += WG) {
        const int qd = task >> 3, sp = task & 7;
        const int j0 = 4 * qd; // window offset of the quad's first position
        const int i0 = sp * L8, i1 = (sp == 7) ? SYM : i0 + L8;
        float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, e0 = 0.f;
        float y0 = yw[j0 + i0], y1 = yw[j0 + i0 + 1], y2 = yw[j0 + i0 + 2];
#pragma unroll 4
        for (int i = i0; i < i1; ++i) {
          const float y3 = yw[j0 + i + 3];
          const float t = tm[i];
          c0 = fmaf(y0, t, c0); c1 = fmaf(y1, t, c1); c2 = fmaf(y2, t, c2); c3 = fmaf(y3, t, c3);
          e0 = fmaf(y0, y0, e0);
          y0 = y1; y1 = y2; y2 = y3;
        }
        // combine the 8 tap ranges (lanes 8qd .. 8qd+7 are adjacent)
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
          c0 += __shfl_xor(c0, o, 64); c1 += __shfl_xor(c1, o, 64);
          c2 += __shfl_xor(c2, o, 64); c3 += __shfl_xor(c3, o, 64);
          e0 += __shfl_xor(e0, o, 64);
        }
        if (sp < 4 && j0 + sp < P) {
          // lane sp finishes position j0 + sp: slide the energy forward sp samples
          const float cj = sp == 0 ? c0 : (sp == 1 ? c1 : (sp == 2 ? c2 : c3));
          float en = e0;
          for (int j = 0; j < sp; ++j) {
            const float yo = yw[j0 + j], yn = yw[j0 + j + SYM];
            en = fmaf(yn, yn, fmaf(-yo, yo, en));
          }
          const float den = sqrtf(fmaxf(en, 0.f) * te);
          float m;
          if (den > 0.001f * (1.f + eps_g)) m = cj / den;
          else if (den > 0.001f * (1.f - eps_g)) m = cj / den + 4.f; // uncertain gate: tagged
          else m = -8.f;                                              // gated out
          sm.u.fine.m[j0 + sp] = m;
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
    }
    STAMP(6);
    if (cfg.stop_after == 2) return;
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
    for (int i = tid; i < cfg.nband; i += WG) { sm.u.fq.known[i] = cfg.t.known[i]; sm.u.fq.band_di[i] = cfg.t.band_di[i]; }
    for (int i = tid; i < nwords; i += WG) sm.u.fq.bits[i] = 0u;
    if (tid == 0) { sm.nsym = M; sm.data0 = data0; sm.gmax = 0.f; sm.zce = 0.f; }
    if (nbits > MAX_BITS_WORDS * 32) { if (tid == 0) sm.flags |= AMOD_FLAG_BIG; }
    __syncthreads();
    STAMP(7);
    issue_prefetch(); // no vector-memory loads are waited on from here to the CRC
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
      const XB xb{(ph + pos1 + 1) >> 1, (ph + pos2 + 1) >> 1}; // float2 index, first whole slot pair
      float2 v[8];
      int const1 = 0, const2 = 0;
      if (active) {
        // a window is constant iff every raw sample equals its first one (NaN frames never get here)
        const float f1 = X[pos1 + CP], f2 = s2 >= 0 ? X[pos2 + CP] : 0.f;
        int ne1 = 0, ne2 = 0;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const int i = CP + lane + 64 * m;
          const float r1 = X[pos1 + i];
          const float r2 = s2 >= 0 ? X[pos2 + i] : 0.f;
          ne1 |= r1 != f1;
          ne2 |= r2 != f2;
          v[m] = make_float2(fmaf(r1, A, B), s2 >= 0 ? fmaf(r2, A, B) : 0.f);
        }
        const1 = __ballot(ne1) == 0;
        const2 = __ballot(ne2) == 0;
        fft512_wave(v, xb, sm);
        if (round == 0) STAMP(8);
        if (job == 0) {
          // channel estimate from the CE symbol: H = Y * known (X = +-1, modem.js:431-438)
          float zmax = 0.f;
          for (int b = lane; b < nband; b += 64) {
            const int k = cfg.sub_start + b;
            const float2 zk = spec_read(sm, xb, k), zn = spec_read(sm, xb, kFft - k);
            zmax = fmaxf(zmax, fmaxf(fabsf(zk.x) + fabsf(zk.y), fabsf(zn.x) + fabsf(zn.y)));
          }
          zmax = wave_max(zmax);
          for (int b = lane; b < nband; b += 64) {
            const int k = cfg.sub_start + b;
            float2 h = make_float2(0.f, 0.f);
            if (!const1) {
              const float2 zk = spec_read(sm, xb, k), zn = spec_read(sm, xb, kFft - k);
              const float2 y = make_float2(0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y));
              const float kn = sm.u.fq.known[b];
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
        STAMP(9);
      }
      if (!active) continue;
      const float gmax = sm.gmax, zce = sm.zce;
      // ---- both data symbols of this job in one pass: equalise, pilot phase, demap
      {
        int ln = lane;
        asm volatile("" : "+v"(ln)); // per-round lane (keeps debug/bit addresses out of registers)
        const bool live1 = s1 >= 0 && !const1, live2 = s2 >= 0 && !const2;
        uint32_t *bits = sm.u.fq.bits;
        const int per_sym = cfg.ndata * cfg.bps;
        float2 e1[4], e2[4];
        float zm = 0.f, em1 = 0.f, em2 = 0.f;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = ln + 64 * rr;
          e1[rr] = e2[rr] = make_float2(0.f, 0.f);
          if (b < nband) {
            const int k = cfg.sub_start + b;
            const float2 zk = spec_read(sm, xb, k), zn = spec_read(sm, xb, kFft - k);
            zm = fmaxf(zm, fmaxf(fabsf(zk.x) + fabsf(zk.y), fabsf(zn.x) + fabsf(zn.y)));
            // Z = x1 + i x2:  X1 = (Z[k] + conj Z[-k]) / 2,  X2 = (Z[k] - conj Z[-k]) / 2i
            const float2 x1 = make_float2(0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y));
            const float2 x2 = make_float2(0.5f * (zk.y + zn.y), 0.5f * (zn.x - zk.x));
            const float2 g = sm.u.fq.g[b];
            e1[rr] = cmul(x1, g);
            e2[rr] = cmul(x2, g);
            em1 = fmaxf(em1, fabsf(e1[rr].x) + fabsf(e1[rr].y));
            em2 = fmaxf(em2, fabsf(e2[rr].x) + fabsf(e2[rr].y));
            if (dbg && (s1 == 0 || s2 == 0)) {
              const bool one = s1 == 0;
              const float2 xx = one ? x1 : x2, ee = one ? e1[rr] : e2[rr];
              const bool c = one ? const1 : const2;
              D->x_re[b] = c ? 0.f : xx.x; D->x_im[b] = c ? 0.f : xx.y;
              D->eq_re[b] = c ? 0.f : ee.x; D->eq_im[b] = c ? 0.f : ee.y;
            }
          }
        }
        // error bound of eq per symbol (fp32 FFT + channel estimate), DESIGN.md "guards"
        const float gsc = 2e-6f * cfg.guard * gmax;
        float d1 = gsc * (zm + em1 * zce), d2 = gsc * (zm + em2 * zce);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { d1 = fmaxf(d1, __shfl_xor(d1, o, 64)); d2 = fmaxf(d2, __shfl_xor(d2, o, 64)); }
        d1 += 1e-12f; d2 += 1e-12f;
        // pilot phase: mean of eqIm/eqRe over pilots with |eqRe| > 1e-6 (modem.js:398-405)
        float ps1 = 0.f, pe1 = 0.f, ps2 = 0.f, pe2 = 0.f;
        int pc1 = 0, pc2 = 0, pflag = 0;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = ln + 64 * rr;
          const bool pil = b < nband && sm.u.fq.band_di[b] < 0;
          const float a1 = fabsf(e1[rr].x), a2 = fabsf(e2[rr].x);
          const bool ok1 = pil && a1 > 1e-6f, ok2 = pil && a2 > 1e-6f;
          if (ok1) { ps1 += e1[rr].y / e1[rr].x; pe1 += 1.f / a1 + fabsf(e1[rr].y) / (a1 * a1); }
          if (ok2) { ps2 += e2[rr].y / e2[rr].x; pe2 += 1.f / a2 + fabsf(e2[rr].y) / (a2 * a2); }
          pc1 += __popcll(__ballot(ok1));
          pc2 += __popcll(__ballot(ok2));
          pflag |= pil && ((live1 && fabsf(a1 - 1e-6f) <= 2.f * d1 + 1e-7f) || (live2 && fabsf(a2 - 1e-6f) <= 2.f * d2 + 1e-7f));
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          ps1 += __shfl_xor(ps1, o, 64); pe1 += __shfl_xor(pe1, o, 64);
          ps2 += __shfl_xor(ps2, o, 64); pe2 += __shfl_xor(pe2, o, 64);
        }
        if (__ballot(pflag)) wflags |= AMOD_FLAG_PHASE;
        const float ph1 = pc1 > 0 ? ps1 / (float)pc1 : 0.f, ph2 = pc2 > 0 ? ps2 / (float)pc2 : 0.f;
        const float dp1 = pc1 > 0 ? d1 * pe1 / (float)pc1 : 0.f, dp2 = pc2 > 0 ? d2 * pe2 / (float)pc2 : 0.f;
        const float tau1 = 4.f * (d1 * (1.f + fabsf(ph1)) + em1 * dp1) + 1e-9f;
        const float tau2 = 4.f * (d2 * (1.f + fabsf(ph2)) + em2 * dp2) + 1e-9f;
        if (dbg && ln == 0) {
          if (s1 >= 0 && s1 < AMOD_DBG_SYMS) D->phase[s1] = const1 ? 0.f : ph1;
          if (s2 >= 0 && s2 < AMOD_DBG_SYMS) D->phase[s2] = const2 ? 0.f : ph2;
        }
        // a constant FFT window has an all-zero spectrum in the reference: every data
        // subcarrier takes the origin decision (ties resolve to the first point)
        int dflag = 0;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = ln + 64 * rr;
          if (b >= nband) continue;
          const int di = sm.u.fq.band_di[b];
          if (di < 0) continue;
#pragma unroll
          for (int which = 0; which < 2; ++which) {
            const int sidx = which == 0 ? s1 : s2;
            if (sidx < 0) continue;
            const bool live = which == 0 ? live1 : live2;
            int idx = cfg.origin_idx;
            if (live) {
              const float2 e = which == 0 ? e1[rr] : e2[rr];
              const float ph = which == 0 ? ph1 : ph2;
              const float cr = fmaf(e.y, ph, e.x);
              const float ci = fmaf(-e.x, ph, e.y);
              float margin;
              idx = decide(cfg.mod, cr, ci, margin);
              dflag |= margin <= (which == 0 ? tau1 : tau2);
            }
            const int pos = sidx * per_sym + di * cfg.bps;
            const uint32_t val = (uint32_t)idx << (32 - cfg.bps - (pos & 31));
            if (val) atomicOr(&bits[pos >> 5], val);
          }
        }
        if (__ballot(dflag)) wflags |= AMOD_FLAG_DEMAP;
      }
      STAMP(10 + round);
    }
    wflags = wave_or(wflags);
    if (lane == 0 && wflags) atomicOr(&sm.flags, wflags);
    __syncthreads();
    STAMP(14);
    if (sm.flags) goto to_exact;
    // ------------------------------------------------ stage 4: finish
    if (cfg.stop_after == 3) return;
    {
      if (dbg && tid == 0) D->nsym = M;
      const uint32_t *v = sm.u.fq.bits;
      int nv = nbits;
      if (cfg.rep > 1) {
        uint32_t *voted = reinterpret_cast<uint32_t *>(sm.x); // samples are dead now
        nv = block_vote(sm.u.fq.bits, nbits, cfg.rep, voted);
        __syncthreads();
        v = voted;
      }
      amod_result r;
      init_result(r);
      r.nbits = nbits;
      if (cfg.mode == AMOD_MODE_RECEIVED) { r.fine_metric = sm.fbest; r.coarse_idx = sm.coarse; r.preamble_idx = start; }
      finish_frame(v, nv, cfg, r, w.res + f, w.payload + (int64_t)f * w.stride, w.stride, sm.ru, nullptr);
      STAMP(15);
      return;
    }
  }

finish_error:
  if (tid == 0) {
    amod_result r;
    init_result(r);
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

// One workgroup per frame (LDS admits one per CU; the dispatcher refills a CU as
// soon as its frame is done, so other CUs' compute overlaps this CU's load).
// Every float4 of the frame is requested before the first is consumed.
__global__ __launch_bounds__(WG) void k_decode_fast(const DevCfg cfg, const DevWork w) {
  __shared__ Smem sm;
  const int f = blockIdx.x;
  {
    const int tid = threadIdx.x;
    STAMP(0);
    float4 q[PF];
    pf_issue(w, f, q);
    stage_in(cfg, w, f, q, sm);
  }
  process_frame(cfg, w, f, sm, []() {});
}

} // namespace
} // namespace amod

extern "C" hipError_t amod_launch_fast(const amod::DevCfg &cfg, const amod::DevWork &w, hipStream_t s) {
  if (w.nframes <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_decode_fast, dim3(w.nframes), dim3(amod::WG), 0, s, cfg, w);
  return hipGetLastError();
}
extern "C" int amod_fast_capacity(void) { return amod::CAP - 8; }
