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
#ifndef AMOD_SC_CQ
#define AMOD_SC_CQ 8
#endif

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
// a[k] for a wave-uniform k < 4 (a select chain: no private-array indexing)
__device__ __forceinline__ double sel4(const double (&a)[4], int k) {
  return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}
// DPP move of a double: lanes whose source is out of the row (row_shr) or whose row is
// masked off read 0
template <int CTRL, int ROWS> __device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROWS, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// inclusive wave scan of doubles (row_shr 1/2/4/8, then row_bcast 15 / 31): exact when
// every sum of a run of lanes is representable (the caller's certificate)
__device__ __forceinline__ double wave_scan_f64(double v) {
  v += dpp_f64<0x111, 0xf>(v);
  v += dpp_f64<0x112, 0xf>(v);
  v += dpp_f64<0x114, 0xf>(v);
  v += dpp_f64<0x118, 0xf>(v);
  v += dpp_f64<0x142, 0xa>(v);
  v += dpp_f64<0x143, 0xc>(v);
  return v;
}
// the wave's minimum (DPP: a lane without a source keeps its own value; lane 63 ends
// with the minimum of all 64)
template <int CTRL, int ROWS> __device__ __forceinline__ int dpp_min_step(int v) {
  return min(v, __builtin_amdgcn_update_dpp(v, v, CTRL, ROWS, 0xf, false));
}
__device__ __forceinline__ int wave_min_i32(int v) {
  v = dpp_min_step<0x111, 0xf>(v);
  v = dpp_min_step<0x112, 0xf>(v);
  v = dpp_min_step<0x114, 0xf>(v);
  v = dpp_min_step<0x118, 0xf>(v);
  v = dpp_min_step<0x142, 0xa>(v);
  v = dpp_min_step<0x143, 0xc>(v);
  return __builtin_amdgcn_readlane(v, 63);
}
// lane l's double (l wave-uniform)
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

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

// fft(re, 0) of 512 real samples src[0..511] on one wave (modem.js:6-13, 26-66): the same
// butterflies as fft_exact with the same operations in the same order, three stages at a
// time inside each lane's registers, the element-to-lane map changed between the groups
// by two transposes through the wave's LDS slot `buf` (512 doubles, re then im):
//   A: e = 8 l + r                         stages half 1, 2, 4   (pairs differ in r)
//   B: e = (l & 7) | r << 3 | (l >> 3) << 6  stages half 8, 16, 32
//   C: e = l | r << 6                       stages half 64, 128, 256; bin k = l + 64 r
// (e: the element index of fft_exact's arrays; the input is bit-reversed, rev9(e)).
__device__ __forceinline__ void fft_stage3(double (&re)[8], double (&im)[8], const double2 *tw, int s0, int ebase,
                                           int rshift) {
  // stages half = 2^s0, 2^(s0+1), 2^(s0+2); slot r's element index: ebase | r << rshift
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int half = 1 << (s0 + q), sb = 1 << q; // the pair differs in slot bit q
    // (no twiddle load hoisted past a stage: all 36 in flight at once spilled the kernel)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (r & sb) continue;
      const int a = r, b = r | sb;
      const int e = ebase | (r << rshift);
      const double2 w = tw[half - 1 + (e & (half - 1))];
      const double t_re = w.x * re[b] - w.y * im[b];
      const double t_im = w.x * im[b] + w.y * re[b];
      re[b] = re[a] - t_re;
      im[b] = im[a] - t_im;
      re[a] = re[a] + t_re;
      im[a] = im[a] + t_im;
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// buf[from(r)] = v[r] for the lane's slots, then v[r] = buf[to(r)]
template <typename F, typename G>
__device__ __forceinline__ void wave_permute(double (&v)[8], double *buf, F &&from, G &&to) {
#pragma unroll
  for (int r = 0; r < 8; ++r) buf[from(r)] = v[r];
  wave_lds_sync();
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = buf[to(r)];
  wave_lds_sync();
}

// the lane's eight input samples of a symbol window (layout A: element 8 lane + r, read
// from src[rev9(8 lane + r)]: for each r the lanes read 64 consecutive samples)
__device__ __forceinline__ void wave_fft_load(const float *src, float (&xv)[8], int lane) {
  asm volatile("" : "+v"(lane)); // (addresses formed here, not eight 64-bit ones held across the loop)
#pragma unroll
  for (int r = 0; r < 8; ++r) xv[r] = src[rev9(8 * lane + r)];
}

__device__ void wave_fft_exact(const float (&xv)[8], double (&re)[8], double (&im)[8], const double2 *tw, int lane,
                               double *buf) {
  // (an opaque lane per call: every lane-derived address is invariant across symbols, and
  // hoisted out of the symbol loop they held the registers that spilled the kernel)
  asm volatile("" : "+v"(lane));
#pragma unroll
  for (int r = 0; r < 8; ++r) { re[r] = or_zero(xv[r]); im[r] = 0.0; }
  fft_stage3(re, im, tw, 0, 8 * lane, 0);                        // A
  const int eb = (lane & 7) | ((lane >> 3) << 6);
  auto fa = [&](int r) { return 8 * lane + r; };
  auto fb = [&](int r) { return eb | (r << 3); };
  wave_permute(re, buf, fa, fb);
  wave_permute(im, buf, fa, fb);
  fft_stage3(re, im, tw, 3, eb, 3);                              // B
  auto fc = [&](int r) { return lane | (r << 6); };
  wave_permute(re, buf, fb, fc);
  wave_permute(im, buf, fb, fc);
  fft_stage3(re, im, tw, 6, lane, 6);                            // C
}

// Make this workgroup's global stores (plain or atomic) visible to its own later
// plain loads. Every wave of the workgroup runs on one CU and shares its L1, so the
// stores need only workgroup scope (the LLVM AMDGPU memory model for gfx942/gfx950
// without threadgroup split); the atomics (the global bit stream's ORs) are performed in
// L2, so the CU's L1 is dropped after the barrier (buffer_inv sc0: this CU's vector L1
// only), in case a line of the slot is still there from an earlier frame's reads. Agent
// scope compiled to buffer_wbl2 sc1 + buffer_inv sc1 at each call: a write-back and
// invalidate of the XCD's L2 under every k_demod and exact workgroup sharing it.
__device__ __forceinline__ void wg_global_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");
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
      // One pass, one wave per G-sample segment (lanes on consecutive samples): each
      // segment's sum, sum|x| and smallest sample ulp (the certificate of the sequential
      // chain below), and the frame's extremes; the frame's parallel sum and its certificate
      // then come from the segment table (round 6: a second pass re-read the frame for the
      // segment sums, ≈ 90 K cycles per listed C5 frame).
      constexpr int SEGCAP = SCH, kSegG = 1024;
      double *const seg_s = sm.sc, *const seg_a = sm.sc + SEGCAP, *const seg_e = sm.sc + 2 * SEGCAP;
      const int G = kSegG * max(1, (N + kSegG * SEGCAP - 1) / (kSegG * SEGCAP));
      const int nseg = (N + G - 1) / G;
      {
        int nonfin = 0;
        float xmn = INFINITY, xmx = -INFINITY;
        for (int sg = wave; sg < nseg; sg += XT / 64) {
          const int b0 = sg * G, e1 = min(N, b0 + G);
          double ss = 0.0, sa = 0.0;
          int em = 1 << 20;
          auto add = [&](float x) {
            ss += (double)x;
            sa += fabs((double)x);
            xmn = fminf(xmn, x);
            xmx = fmaxf(xmx, x);
            const uint32_t e = (__float_as_uint(x) >> 23) & 0xFFu;
            if (e == 0xFFu) nonfin = 1;
            else if (x != 0.0f) em = min(em, e == 0 ? -149 : (int)e - 150);
          };
          int i = b0 + lane;
          for (; i + 7 * 64 < e1; i += 8 * 64) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = xr[i + 64 * u];
#pragma unroll
            for (int u = 0; u < 8; ++u) add(v[u]);
          }
          for (; i < e1; i += 64) add(xr[i]);
          // (the order of the adds is free: ss is used only where certified or non-finite,
          // where every order gives the same result, and sa's rounding is within its slack)
          ss = wave_scan_f64(ss);
          sa = wave_scan_f64(sa);
          em = wave_min_i32(em);
          if (lane == 63) { seg_s[sg] = ss; seg_a[sg] = sa; seg_e[sg] = (double)em; }
        }
        for (int o = 32; o > 0; o >>= 1) {
          nonfin |= __shfl_xor(nonfin, o, 64);
          xmn = fminf(xmn, __shfl_xor(xmn, o, 64));
          xmx = fmaxf(xmx, __shfl_xor(xmx, o, 64));
        }
        if (lane == 0) { sm.ri[XT / 64 + wave] = nonfin; sm.rf[wave] = xmn; sm.ru[wave] = __float_as_uint(xmx); }
      }
      __syncthreads();
      bool exact_par = true;
      if (wave == 0) { // the frame's sums over the segment table (any order: see below)
        double S = 0.0, PA = 0.0;
        int EM = 1 << 20;
        for (int sg = lane; sg < nseg; sg += 64) { S += seg_s[sg]; PA += seg_a[sg]; EM = min(EM, (int)seg_e[sg]); }
        S = wave_scan_f64(S);
        PA = wave_scan_f64(PA);
        EM = wave_min_i32(EM);
        if (lane == 63) {
          int NF = 0;
          float MN = INFINITY, MX = -INFINITY;
          for (int i = 0; i < XT / 64; ++i) {
            NF |= sm.ri[XT / 64 + i];
            MN = fminf(MN, sm.rf[i]); MX = fmaxf(MX, __uint_as_float(sm.ru[i]));
          }
          sm.xmn = MN; sm.xmx = MX; sm.nonfin = NF;
          // non-finite samples: NaN, or +-Inf, whatever the order (finite sums stay finite);
          // (sum|x| in fp64 over N terms: relative error below N 2^-53 < 2^-40)
          exact_par = NF || EM >= (1 << 19) || PA * (1.0 + 0x1p-40) < ldexp(1.0, EM + 53);
          sm.mean = S / (double)N;
          sm.status = exact_par;
        }
      }
      __syncthreads();
      exact_par = sm.status != 0;
      __syncthreads();
      XSTAMP(13);
      if (!exact_par) {
        // Segments of G >= 1024 samples, certified one by one along the sequential order. A
        // segment whose sum|x| < 2^(em + 53) (em: its smallest sample ulp exponent) has
        // exact internal sums in any order, so its total comes out exact from one thread's
        // running sum. With S the running (sequential) sum at its start and q the smaller
        // of em and the exponent of S's lowest set bit, every partial sum S + P_j is a
        // multiple of 2^q no larger than |S| + sum|x| in magnitude; below 2^(q + 53) none
        // of them rounds and S + total is the sequential result.
        //
        // A segment failing the test (a partial sum that could round: once S has a full
        // mantissa, any segment that could carry it across a binade) is walked in pieces of
        // 256 samples, one per wave at a time: each wave forms its piece's exact prefix sums
        // Q_j (four consecutive samples per lane, a DPP wave scan); wave 0 then walks the
        // pieces: with S exact at a piece start, lane j's s_j = fl(S + Q_j) IS the sequential
        // state after sample j as long as no earlier sum rounded (by induction: state_j =
        // fl(state_{j-1} + x_j) with state_{j-1} = S + Q_{j-1} exactly). TwoSum finds the
        // first j* whose sum rounded; its s is still the sequential state (the rounding the
        // reference makes), and the piece continues from S = s_{j*} with Q_j - Q_{j*}
        // (exact: a sum within the piece). A piece costs one pass plus one per rounding
        // event where one lane adding sample by sample cost ≈ 120 cycles a sample (a C5
        // frame at 7 dB took 13 M cycles). A piece's Q are exact when the segment's
        // sum|x| < 2^(em + 53) for the piece's own em; a piece failing that is added sample
        // by sample.
        // (the segment table is pass 1's)
        constexpr int PW = 256, NW = XT / 64;
        double *const qb = reinterpret_cast<double *>(sm.chunk); // one piece per wave
        uint32_t *const qok = sm.ru;
        static_assert(sizeof(sm.chunk) >= NW * PW * sizeof(double) && NW <= 16, "piece buffers");
        // (sum|x| in fp64 over G terms: relative error below G 2^-53)
        const double slack = 1.0 + ldexp((double)G, -52);
        double S = 0.0; // (every thread holds the same)
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
          const double sa = seg_a[sg] * slack;
          if (sa < ldexp(1.0, em + 53) && (fabs(S) * slack + sa) < ldexp(1.0, q + 53)) {
            S += seg_s[sg];
            continue;
          }
          const int e1 = min(N, (sg + 1) * G);
          for (int p0 = sg * G; p0 < e1; p0 += NW * PW) {
            { // every wave: its piece's exact prefix sums
              const int i0 = p0 + wave * PW + 4 * lane;
              float xv[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) xv[k] = i0 + k < e1 ? xr[i0 + k] : 0.f;
              double l[4];
              int eb = 1 << 20;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                l[k] = (k ? l[k - 1] : 0.0) + (double)xv[k];
                const uint32_t e = (__float_as_uint(xv[k]) >> 23) & 0xFFu;
                if (xv[k] != 0.0f) eb = min(eb, e == 0 ? -149 : (int)e - 150);
              }
              const double ex = wave_scan_f64(l[3]) - l[3]; // exclusive (exact: a sub-range sum)
              eb = wave_min_i32(eb);
              double2 *const qd = reinterpret_cast<double2 *>(qb + wave * PW) + 2 * lane;
              qd[0] = make_double2(ex + l[0], ex + l[1]);
              qd[1] = make_double2(ex + l[2], ex + l[3]);
              if (lane == 0) qok[wave] = eb >= (1 << 19) || sa < ldexp(1.0, eb + 53);
            }
            __syncthreads();
            if (wave == 0) {
              for (int pi = 0; pi < NW; ++pi) {
                const int ps = p0 + pi * PW;
                if (ps >= e1) break;
                const int nv = min(PW, e1 - ps);
                if (qok[pi]) {
                  const double2 *const q2 = reinterpret_cast<const double2 *>(qb + pi * PW) + 2 * lane;
                  const double2 qa = q2[0], qc = q2[1];
                  const double qv[4] = {qa.x, qa.y, qc.x, qc.y};
                  double base = 0.0;
                  int j0 = -1;
                  while (true) {
                    double sv[4];
                    uint64_t m[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                      const double pj = qv[k] - base; // exact
                      const double s = S + pj;
                      const double bq = s - S, aq = s - bq; // TwoSum: s + (da + db) = S + pj
                      const double da = S - aq, db = pj - bq;
                      const int j = 4 * lane + k;
                      sv[k] = s;
                      m[k] = __ballot(j > j0 && j < nv && da + db != 0.0);
                    }
                    const uint64_t any = m[0] | m[1] | m[2] | m[3];
                    if (any == 0) {
                      const int jl = nv - 1;
                      S = readlane_f64(sel4(sv, jl & 3), jl >> 2);
                      break;
                    }
                    const int L0 = __builtin_ctzll(any);
                    const int k = (m[0] >> L0) & 1 ? 0 : (m[1] >> L0) & 1 ? 1 : (m[2] >> L0) & 1 ? 2 : 3;
                    S = readlane_f64(sel4(sv, k), L0);
                    base = readlane_f64(sel4(qv, k), L0);
                    j0 = 4 * L0 + k;
                    if (j0 == nv - 1) break;
                  }
                } else { // sample by sample: 64 coalesced loads, then lane by lane in order
                  for (int c = 0; c < nv; c += 64) {
                    const float v = c + lane < nv ? xr[ps + c + lane] : 0.f;
                    const int nj = min(64, nv - c);
                    for (int j = 0; j < nj; ++j) S += (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
                  }
                }
              }
              if (lane == 0) sm.phase = S; // (the state after these pieces, to every wave)
            }
            __syncthreads();
            S = sm.phase; // (its next write follows the next round's barrier)
          }
        }
        if (tid == 0) sm.mean = S / (double)N;
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
        if (tid < 3) { // P(0), Ra(0), Rb(0) (modem.js:292-298), one sum per lane
          for (int m = 0; m < half; ++m) {
            const double a = xs[m], b = xs[m + half];
            acc += tid == 0 ? a * b : (tid == 1 ? a * a : b * b);
          }
        }
        // Positions [0, d_hi] in halves of HB positions, pipelined over two buffers: in step
        // h, wave 0's lanes 0-2 run the three sequential additions through half h (buffer
        // h & 1: increments in, the states at each position out when the half holds a
        // compared position) while each thread of waves 1-3 forms the metrics of its
        // positions of half h - 1 (the other buffer, states of the step before) and then
        // overwrites the same slots with the increments of half h + 1 (the same positions:
        // no other thread reads them), from samples it loaded a step earlier. The chain is
        // the only sequential work; every other step hides under it.
        constexpr int HB = SCH / 2;
        const int nh = d_hi / HB + 1;  // halves covering [0, d_hi]
        const int h_keep = d_lo / HB;  // the first half holding a compared position
        auto put = [&](int h, int k, float a_out_f, float mid_f, float b_in_f) {
          double *const bp = sm.sc + (h & 1) * 3 * HB;
          const int d = h * HB + k;
          double ip = 0.0, ia = 0.0, ib = 0.0;
          if (d < end) { // zero past `end`: adding +0.0 changes no state at or before `end`
            const double a_out = a_out_f, mid = mid_f, b_in = b_in_f;
            ip = mid * b_in - a_out * mid;
            ia = mid * mid - a_out * a_out;
            ib = b_in * b_in - mid * mid;
          }
          bp[k] = ip; bp[HB + k] = ia; bp[2 * HB + k] = ib;
        };
        auto ld = [&](int d) { return d < N ? xs[d] : 0.f; };
        for (int k = tid; k < HB; k += XT) put(0, k, ld(k), ld(k + half), ld(k + 2 * half));
        // waves 1-3: thread tt owns positions tt, tt + 192, tt + 384 of every half
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
        for (int h = 0; h <= nh; ++h) {
          if (wave == 0) {
            if (h < nh && lane < 3) {
              double2 *const v = reinterpret_cast<double2 *>(sm.sc + (h & 1) * 3 * HB + lane * HB);
              // A rotating pipeline: pair k + Q is requested as pair k is added, so Q loads
              // are always in flight and each add waits only for its own (the adds are the
              // chain; reads past the half land in the next lane's half or other LDS fields
              // and are never used)
              constexpr int Q = AMOD_SC_CQ;
              double2 t[Q];
#pragma unroll
              for (int j = 0; j < Q; ++j) t[j] = v[j];
              if (h < h_keep) { // states not needed: the running sums only
                for (int k = 0; k < HB / 2; k += Q) {
#pragma unroll
                  for (int j = 0; j < Q; ++j) {
                    const double2 c = t[j];
                    t[j] = v[k + Q + j];
                    acc += c.x;
                    acc += c.y;
                  }
                }
              } else {
                for (int k = 0; k < HB / 2; k += Q) {
#pragma unroll
                  for (int j = 0; j < Q; ++j) { // the state at each position, then its update
                    const double2 c = t[j];
                    t[j] = v[k + Q + j];
                    const double s0 = acc;
                    acc += c.x;
                    const double s1 = acc;
                    acc += c.y;
                    v[k + j] = make_double2(s0, s1);
                  }
                }
              }
            }
          } else {
            const int hm = h - 1;
            if (hm >= h_keep) { // metrics of half h - 1, first strict maximum per thread
              const double *const bp = sm.sc + (hm & 1) * 3 * HB;
#pragma unroll
              for (int j = 0; j < PT; ++j) {
                const int k = tt + (XT - 64) * j, d = hm * HB + k;
                if (k < HB && d >= d_lo && d <= d_hi) {
                  const double pp = bp[k], a = bp[HB + k], b = bp[2 * HB + k];
#ifndef AMOD_KO_METRIC
                  // (the division only where the metric may beat bm: with q = fl(pp pp) and
                  // r = fl(a b), q < fl(r bm) (1 - 2^-40) means q / r < bm, so fl(q / r) <= bm)
                  if (a > 0.01 && b > 0.01) {
                    const double q = pp * pp, r = a * b;
                    if (!(q < (r * bm) * (1.0 - 0x1p-40))) {
                      const double metric = q / r;
                      if (metric > bm) { bm = metric; bi = d; }
                    }
                  }
#endif
                }
              }
            }
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
    // The bit stream lives in LDS past the transform's twiddles when it fits (chunk windows
    // and short frames): the demap's ORs, the vote, the parse, the CRC and the payload rows
    // then read and write LDS. In the slot's global words, the vote and frame end waited out
    // a cache round trip per word or byte read (~175 K cycles per 101-symbol chunk window).
    // The voted stream goes to the transform arrays, free once every symbol is demapped.
    constexpr int kTwBytes = (((kFft - 1) * (int)sizeof(double2)) + 15) & ~15;
    // the demap's tables at the chunk area's end: 16 constellation points, then the band's
    // data indices (read per slot and symbol, from global memory they were a cache round
    // trip each inside the symbol loop)
    constexpr int kTabBytes = 16 * (int)sizeof(double2) + kMaxBand * (int)sizeof(int16_t);
    constexpr int kTabOff = ((int)sizeof(sm.chunk) - kTabBytes) & ~15;
    constexpr int kLdsStreamWords = (kTabOff - kTwBytes) / 4;
    static_assert(kLdsStreamWords > 0, "room for a stream past the twiddles");
    const bool lds_stream = nwords + 8 <= kLdsStreamWords;
    if (lds_stream) bits = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(sm.chunk) + kTwBytes);
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
    // Data symbols s = wave, wave + 4, ...: one wave per symbol, the four waves on four
    // symbols at once (a workgroup-wide transform with nine barriers per symbol kept three
    // of the four waves waiting: a frame with 101 data symbols took ~0.8 ms). Per symbol:
    // the reference's radix-2 transform in registers (wave_fft_exact, its transposes
    // through the wave's LDS slot), the equaliser per bin on the lane that holds it, the
    // bins of the band into the same slot, the pilot phase on lane 0 in the pilot list's
    // order, the demap of the band on all lanes.
    {
      double2 *const eqb = (wave < 2 ? reinterpret_cast<double2 *>(sm.re) : reinterpret_cast<double2 *>(sm.er)) +
                           (wave & 1) * kMaxBand;
      static_assert(2 * kMaxBand * sizeof(double2) == 2 * kFft * sizeof(double), "two wave slots per array pair");
      // the transform's twiddles in LDS (the fine stage's sample buffer is free now): read
      // from global memory each of the nine stages waited out an L2 round trip
      double2 *const twl = reinterpret_cast<double2 *>(sm.chunk);
      static_assert(sizeof(sm.chunk) >= (kFft - 1) * sizeof(double2), "twiddles in the chunk area");
      for (int i = tid; i < kFft - 1; i += XT) twl[i] = cfg.t.tw_exact[i];
      double2 *const ptl = reinterpret_cast<double2 *>(reinterpret_cast<char *>(sm.chunk) + kTabOff);
      int16_t *const dil = reinterpret_cast<int16_t *>(ptl + 16);
      if (tid < 16) ptl[tid] = tid < npts ? cfg.t.points[tid] : make_double2(0.0, 0.0);
      for (int b = tid; b < cfg.nband; b += XT) dil[b] = cfg.t.band_di[b];
      __syncthreads();
      float xv[8]; // the next symbol's samples, requested a symbol ahead
      if (wave < M) wave_fft_load(sig + data0 + wave * SYM + CP, xv, lane);
      for (int s = wave; s < M; s += XT / 64) {
        double re[8], im[8];
        // (the debug record's address opaque per symbol: its 32 per-slot store addresses,
        // hoisted out of the loop, held 64 VGPRs across it)
        amod_debug *Ds = D;
        asm volatile("" : "+s"(Ds));
        {
          float cur[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) cur[r] = xv[r];
          if (s + XT / 64 < M) wave_fft_load(sig + data0 + (s + XT / 64) * SYM + CP, xv, lane);
          wave_fft_exact(cur, re, im, twl, lane, reinterpret_cast<double *>(eqb));
        }
        // equalise the lane's bins k = lane + 64 r of the band (demodulateOFDM 386-395)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int k = lane + 64 * r;
          if (k >= cfg.sub_start && k <= cfg.sub_end) {
            const double hr = sm.hr[k], hi = sm.hi[k];
            const double hmag = hr * hr + hi * hi;
            double er, ei;
            if (hmag > 1e-10) {
              er = (re[r] * hr + im[r] * hi) / hmag;
              ei = (im[r] * hr - re[r] * hi) / hmag;
            } else {
              er = re[r]; ei = im[r];
            }
            const int b = k - cfg.sub_start;
            eqb[b] = make_double2(er, ei);
            if (Ds && s == 0) { Ds->x_re[b] = re[r]; Ds->x_im[b] = im[r]; Ds->eq_re[b] = er; Ds->eq_im[b] = ei; }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); // (the wave reads other lanes' bins below)
        __builtin_amdgcn_wave_barrier();
        double ph = 0.0;
        {
          // lane i forms pilot i's quotient eqIm / eqRe (the divisions at once, each the
          // same IEEE operation; npilots <= AMOD_MAX_PILOTS = 32), then every lane adds the
          // used ones in the pilot list's order (modem.js:398-405): the same sum, one
          // dependent add per pilot
          static_assert(AMOD_MAX_PILOTS <= 64, "one lane per pilot");
          double q = 0.0;
          bool used = false;
          if (lane < cfg.npilots) {
            const int p = cfg.pilots[lane];
            if (p >= cfg.sub_start && p <= cfg.sub_end) {
              const double2 e = eqb[p - cfg.sub_start];
              if (fabs(e.x) > 1e-6) { q = e.y / e.x; used = true; }
            }
          }
          uint64_t um = __ballot(used);
          const int pc = __popcll(um);
          double ps = 0.0;
          for (; um; um &= um - 1) ps += readlane_f64(q, __builtin_ctzll(um));
          ph = pc > 0 ? ps / (double)pc : 0.0;
        }
        if (Ds && lane == 0 && s < AMOD_DBG_SYMS) Ds->phase[s] = ph;
        for (int b = lane; b < cfg.nband; b += 64) {
          const int di = dil[b];
          if (di < 0) continue;
          const double2 e = eqb[b];
          const double cr = e.x + e.y * ph;
          const double ci = e.y - e.x * ph;
          double md = __builtin_inf();
          int mi = 0;
          for (int i = 0; i < npts; ++i) {
            const double2 pt = ptl[i];
            const double dr = cr - pt.x, dd = ci - pt.y;
            const double dist = dr * dr + dd * dd;
            if (dist < md) { md = dist; mi = i; }
          }
          const int pos = (s * cfg.ndata + di) * cfg.bps;
          if (sv) {
            // weighted by |H|^2: the equaliser's division amplifies noise where the channel
            // estimate is weak, so each bit counts in proportion to its channel power (MRC)
            const int k = cfg.sub_start + b;
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
          if (val) { // (an LDS-typed pointer: ds_or, not the flat atomic a generic one takes)
            if (lds_stream) atomicOr(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(sm.chunk) + kTwBytes) + (pos >> 5), val);
            else atomicOr(&bits[pos >> 5], val);
          }
        }
        __builtin_amdgcn_wave_barrier(); // (the slot is rewritten by the next symbol)
      }
    }
    wg_global_sync();
    XSTAMP(12);
    if (D && tid == 0) D->nsym = M;
    r.nbits = nbits;
    const uint32_t *v = bits;
    int nv = nbits;
    if (cfg.rep > 1) {
      uint32_t *voted = lds_stream ? reinterpret_cast<uint32_t *>(sm.re) : bits + ((nwords + 3) & ~3);
      static_assert(6 * sizeof(sm.re) / 4 >= sizeof(sm.chunk) / 4, "a voted stream no longer than the raw one fits");
      nv = sv ? soft_vote(sv, nbits, cfg.rep, voted) : block_vote(bits, nbits, cfg.rep, voted);
      wg_global_sync();
      v = voted;
    }
    XSTAMP(17); // (diagnostics: voted)
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
    XSTAMP(16); // (diagnostics: frame end)
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
