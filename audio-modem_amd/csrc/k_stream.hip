// k_stream.hip — GPU pieces of the streaming receiver (app.js StreamingReceiver 706-998).
//
//   k_ema_*      processAudioBlock's DC removal (app.js:751-755): the EMA
//                m_i = 0.999 m_(i-1) + (1 - 0.999) x_i in IEEE double, cleaned_i =
//                f32(x_i - m_i), bit-exact. (1) each 1024-sample chunk's contribution
//                to the state at its end, coalesced; (2) one lane per chunk runs the
//                exact recurrence from an approximate state 4 chunks back (a short
//                geometric sum of those contributions; the map
//                contracts by 0.999 a step, so the chain meets the true one bit for bit)
//                and through its own 8 chunks, samples staged through per-wave LDS tiles
//                (coalesced rows, one row per lane); (3) every chunk whose warm-up state
//                differs from its predecessor's end state is listed, (4) and recomputed
//                from the true state in order. Afterwards every cleaned sample equals the
//                reference's.
//   k_sc_blocks  fp32 32-sample block sums (coalesced, 8-lane DPP reductions), then
//   k_sc_screen  hot-block screening for the fine precompute: the Schmidl-Cox metric
//                at each block start from 8-block window sums; only a hint (the host
//                recomputes anything the hint missed).
//   k_fine       _refineAndCollect's cross-correlation metric (app.js:864-877) for a
//                list of position ranges: corr = sum seg[i] pre1[i] and sEnergy =
//                sum seg[i]^2 in the reference's order, then corr / sqrt(sEnergy E),
//                one lane per position, IEEE double (f32 x f32 products are exact in
//                double; sqrt and the quotient correctly rounded).
//   k_gather     the granules of the cleaned stream the host state machine reads (its
//                scan and refine regions), packed for one device-to-host copy
//   k_window     _demodulateFrame's per-window peak normalisation (app.js:916-925):
//                mx = max |x|, x / mx when mx > 1e-6 (f32 of the double quotient).
// Built with -ffp-contract=off.
#include "amodem_internal.h"

#include <algorithm>
#include <cstdlib>

namespace amod {
namespace {

__device__ __forceinline__ float sample_at(const float *x, int64_t n, int64_t i) { return (i >= 0 && i < n) ? x[i] : 0.f; }

constexpr double kAlpha = 0.999;
constexpr double kOneMinusAlpha = 1.0 - 0.999; // (1 - this.dcAlpha), evaluated in double
constexpr int kL = 1024;                       // EMA chunk (one lane each in k_ema_out)
constexpr int kWarmDefault = 4;                // warm-up chunks before each chunk (the parallel fix
                                               // rounds settle the chunks whose chains had not met)
constexpr int kEmaRounds = 6;                  // parallel fix rounds before the serial safety net
constexpr int kPerDefault = 8;                 // output chunks per k_ema_out lane
constexpr int kTile = 32;                      // samples per lane per LDS tile (36.9 KB per workgroup:
                                               // four per CU; 16 with 8 waves per SIMD measured slower)
constexpr int kLPR = kTile / 4;                // lanes per tile row in the coalesced loads / stores
constexpr int kRPI = 64 / kLPR;                // tile rows per load instruction

// one step of processAudioBlock's DC removal (app.js:753): fl(fl(a m) + fl((1 - a) x))
__device__ __forceinline__ double ema_step(double m, float x) { return kAlpha * m + kOneMinusAlpha * (double)x; }

// (1) c_k = sum_i a^(L-1-i) (1-a) x_(kL+i): chunk k's contribution to the EMA at its end
// from a zero start (fp64, approximate: it only seeds the warm-up). One WAVE per chunk,
// chunks [kbase, kend): lane l takes samples 4 l + 256 u (u < 4) as float4 buffer loads
// (1 KB per wave-instruction; dwords past nx read 0), apow[j] = a^j as double2 pairs. (One
// 256-thread workgroup per chunk with dword loads ran at 4.2 TB/s: 888 K workgroups of
// four loads a thread for a 32k-chunk stream.)
__global__ __launch_bounds__(256) void k_ema_contrib(const float *__restrict__ x, int64_t nx,
                                                     const double *__restrict__ apow, double *__restrict__ c,
                                                     int64_t kbase, int64_t kend) {
  const int lane = threadIdx.x & 63;
  const int64_t k = kbase + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= kend) return;
  const int64_t a0 = k * kL, len = nx - a0 < kL ? (nx - a0 > 0 ? nx - a0 : 0) : kL;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void *)(x + a0), (short)0, (int)(4 * len), 0x00020000);
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  u4 v[kL / 256];
#pragma unroll
  for (int u = 0; u < kL / 256; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * lane + 1024 * u, 0, 0);
  double acc = 0.0;
#pragma unroll
  for (int u = 0; u < kL / 256; ++u) {
    const int i = 4 * lane + 256 * u; // samples i .. i + 3 weigh a^(L-1-i) .. a^(L-4-i)
    const double2 p01 = *reinterpret_cast<const double2 *>(apow + kL - 4 - i); // a^(L-4-i), a^(L-3-i)
    const double2 p23 = *reinterpret_cast<const double2 *>(apow + kL - 2 - i); // a^(L-2-i), a^(L-1-i)
    acc += p23.y * (kOneMinusAlpha * (double)__uint_as_float(v[u][0]));
    acc += p23.x * (kOneMinusAlpha * (double)__uint_as_float(v[u][1]));
    acc += p01.y * (kOneMinusAlpha * (double)__uint_as_float(v[u][2]));
    acc += p01.x * (kOneMinusAlpha * (double)__uint_as_float(v[u][3]));
  }
  acc = wave_sum(acc);
  if (lane == 0) c[k] = acc;
}

// (2) the exact recurrence, one lane per chunk: from the approximate state at the end of
// chunk k - kWarm - 1 (sum_j A^j c_(k - kWarm - 1 - j), A = a^L = 0.36: forty terms leave
// a relative error below 1e-17), kWarm chunks of warm-up (the map contracts by 0.999 a step, so the
// chain reaches the true one bit for bit), then chunk k with its outputs. The samples move
// through a per-wave LDS tile (64 lanes x 32 samples): rows loaded coalesced two tiles
// ahead (registers), each lane walking its own row, output rows stored coalesced.
// warm[k] = the state reached at chunk k's start. A lane outputs `per` consecutive chunks
// after one warm-up (per = 1 read every sample kWarm + 1 times, from HBM: the re-reads are
// other lanes' chunks, long evicted; per = 2 reads them (kWarm + 2) / 2 times).
constexpr int kRow = kTile + 4; // row stride (floats): 16-byte rows for ds_read_b128
__global__ __launch_bounds__(256) void k_ema_out(const float *__restrict__ x, int64_t nx, int64_t n,
                                                 const double *__restrict__ c,
                                                 double A, float *__restrict__ y, double *__restrict__ warm,
                                                 double *__restrict__ end, int64_t nch, int kWarm, int per,
                                                 int64_t wave0, int64_t wave1) {
  __shared__ __attribute__((aligned(16))) float tile[4][64 * kRow];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t gw = wave0 + (int64_t)blockIdx.x * 4 + wv; // waves [wave0, wave1) of this launch
  const int64_t k0 = gw * 64 * per; // the wave's first chunk
  if (gw >= wave1 || k0 >= nch) return;
  const int64_t k = k0 + (int64_t)per * lane;                    // the lane's first output chunk
  const int64_t kw = k - kWarm > 0 ? k - kWarm : 0;           // first warm-up chunk
  double m = 0.0;                                             // zero start: the true one
  if (k < nch && kw > 0) {
    double p = 1.0;
    for (int64_t j = kw - 1; j >= 0 && j > kw - 41; --j) { m += p * c[j]; p *= A; }
  }
  float *const T = tile[wv];
  // lane l's row at step j covers samples [(k - kWarm) L + kTile j, + kTile) (warm-up
  // chunks first, then chunks k .. k + per - 1); rows before the stream start are skipped
  const int steps = (kWarm + per) * kL / kTile, wsteps = kWarm * kL / kTile;
  const int rr = lane / kLPR, c4 = lane % kLPR; // load/store slot: rows rr + kRPI q, column 4 c4
  // the wave's window as raw buffers: out-of-range dwords read 0 / are not written, so no
  // load or store sits under a branch (offsets before the stream start wrap out of range)
  const int64_t wb = (k0 - kWarm) * kL > 0 ? (k0 - kWarm) * kL : 0, yb = k0 * kL;
  const int64_t xlen = nx - wb > 0 ? nx - wb : 0, ylen = n - yb > 0 ? n - yb : 0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(x + wb), (short)0, (int)(4 * (xlen < (1 << 28) ? xlen : (1 << 28))), 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(y + yb), (short)0, (int)(4 * (ylen < (1 << 28) ? ylen : (1 << 28))), 0x00020000);
  // two tiles in flight (pfa: even steps, pfb: odd): with ~7 waves per CU for a C4-sized
  // stream, one tile ahead (8 KB per wave) left each step waiting out most of a load's
  // latency (k_ema_out 2.1 ms for a 3.6 GB stream, 4.3 TB/s of its 9.1 GB)
  float4 pfa[kLPR], pfb[kLPR];
  auto load = [&](int j, float4 (&pf)[kLPR]) {
#pragma unroll
    for (int q = 0; q < kLPR; ++q) {
      const int64_t g = (k0 + (int64_t)per * (rr + kRPI * q) - kWarm) * kL + (int64_t)kTile * j + 4 * c4 - wb;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(4 * g), 0, 0);
      pf[q] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
  };
  auto step = [&](int j, float4 (&pf)[kLPR]) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < kLPR; ++q) *reinterpret_cast<float4 *>(T + (rr + kRPI * q) * kRow + 4 * c4) = pf[q];
    __builtin_amdgcn_wave_barrier();
    if (j + 2 < steps) load(j + 2, pf); // in flight under this tile's and the next one's recurrence
    const int64_t row0 = (k - kWarm) * kL + (int64_t)kTile * j; // first sample of this lane's row
    const bool out = j >= wsteps;                                // chunks k .. k + per - 1
    if (out && (j - wsteps) % (kL / kTile) == 0) { // an output chunk starts
      const int64_t kc = k + (j - wsteps) / (kL / kTile);
      if (kc > k && kc - 1 < nch) end[kc - 1] = m;
      if (kc < nch) warm[kc] = m;
    }
    float *const R = T + lane * kRow;
    if (row0 >= kw * kL) { // warm-up from the chunk kw (its approximate seed), then chunk k
      if (row0 + kTile <= n) {
        // four samples a group: the (1 - a) x products first, then the dependent chain
        // fl(fl(a m) + b) alone, then the outputs from the saved states
        for (int i = 0; i < kTile; i += 4) {
          const float4 v0 = *reinterpret_cast<const float4 *>(R + i);
          const float xv[4] = {v0.x, v0.y, v0.z, v0.w};
          double b[4], ms[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) b[u] = kOneMinusAlpha * (double)xv[u];
#pragma unroll
          for (int u = 0; u < 4; ++u) { m = kAlpha * m + b[u]; ms[u] = m; }
          if (out) {
            float o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) o[u] = (float)((double)xv[u] - ms[u]);
            *reinterpret_cast<float4 *>(R + i) = make_float4(o[0], o[1], o[2], o[3]);
          }
        }
      } else { // the stream's last samples
        for (int i = 0; row0 + i < n; ++i) {
          const float xv = R[i];
          m = ema_step(m, xv);
          if (out) R[i] = (float)((double)xv - m);
        }
      }
    }
    if (out) {
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < kLPR; ++q) {
        const int r = rr + kRPI * q;
        const int64_t g = (int64_t)per * r * kL + (int64_t)kTile * (j - wsteps) + 4 * c4;
        const float4 v = *reinterpret_cast<const float4 *>(T + r * kRow + 4 * c4);
        __amdgpu_buffer_rsrc_t yrr = yr;
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        const u4 w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(w, yrr, (int)(4 * g), 0, 0);
      }
    }
  };
  load(0, pfa);
  if (steps > 1) load(1, pfb);
  for (int j = 0; j < steps; j += 2) {
    step(j, pfa);
    if (j + 1 < steps) step(j + 1, pfb);
  }
  const int64_t kl = k + per - 1 < nch ? k + per - 1 : nch - 1; // the lane's last chunk
  if (kl >= k) end[kl] = m;
}

// (3) chunks whose start state is not bit-equal to the previous chunk's end state
// (warm-up not converged): flagged (lflag) and listed for the fix passes. Chunk 0 starts
// from the true zero; cnt is one round's counter
__global__ __launch_bounds__(256) void k_ema_check_flag(const double *__restrict__ warm, const double *__restrict__ end,
                                                        int64_t nch, unsigned long long *__restrict__ cnt,
                                                        int64_t *__restrict__ list, uint8_t *__restrict__ lflag) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nch) return;
  const bool bad = k > 0 && __double_as_longlong(warm[k]) != __double_as_longlong(end[k - 1]);
  lflag[k] = bad;
  if (bad) list[atomicAdd(cnt, 1ull)] = k;
}

// (4') one round of the parallel fix: one LANE per run of flagged chunks (a flagged chunk
// whose predecessor is not flagged heads one; every verified chunk before a head ends in
// the true state). The lane recomputes the head from its predecessor's end state, then
// walks on while the next chunk is flagged behind it (the same run) or its recorded start
// state differs from the new end (the change propagates), recording each chunk's start
// state in warm[] and its end in end[]; it stops before a chunk another run's lane owns.
// Runs are independent, so 64 of them step in parallel per wave (each lane its own
// exact chain over its own samples, 16 per load); a start state read while another run
// rewrote it is caught by the next round's check. Lanes whose runs end early idle until
// the wave's longest run is done (runs are a chunk or a few).
__global__ __launch_bounds__(256) void k_ema_runs(const float *__restrict__ x, int64_t nx, int64_t n,
                                                  float *__restrict__ y, double *__restrict__ warm,
                                                  double *__restrict__ end, int64_t nch,
                                                  const unsigned long long *__restrict__ cnt,
                                                  const int64_t *__restrict__ list, const uint8_t *__restrict__ lflag,
                                                  unsigned long long *__restrict__ fixed) {
  const int64_t nl = (int64_t)*cnt;
  const int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if ((int64_t)blockIdx.x * 256 >= nl) return; // (whole workgroup past the list)
  bool active = li < nl;
  int64_t t = active ? list[li] : 1;
  if (active && lflag[t - 1]) active = false; // inside a run: its head's lane takes it
  double m = active ? end[t - 1] : 0.0;
  unsigned long long nf = 0;
  while (__ballot(active)) {
    if (active) {
      warm[t] = m; // the start state this chunk's outputs now come from
      const int64_t a = t * kL, b = a + kL < n ? a + kL : n;
      if (b - a == kL && a + kL <= nx) {
        const float4 *src = reinterpret_cast<const float4 *>(x + a);
        float4 *dst = reinterpret_cast<float4 *>(y + a);
        for (int i = 0; i < kL / 4; i += 4) {
          float4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = src[i + u];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float xs[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            float o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { m = ema_step(m, xs[q]); o[q] = (float)((double)xs[q] - m); }
            dst[i + u] = make_float4(o[0], o[1], o[2], o[3]);
          }
        }
      } else { // the stream's last chunk
        for (int64_t g = a; g < b; ++g) {
          const float xv = g < nx ? x[g] : 0.f;
          m = ema_step(m, xv);
          y[g] = (float)((double)xv - m);
        }
      }
      end[t] = m;
      ++nf;
      if (t + 1 >= nch) {
        active = false;
      } else {
        const bool next_flagged = lflag[t + 1] != 0, cur_flagged = lflag[t] != 0;
        if (next_flagged ? !cur_flagged : __double_as_longlong(warm[t + 1]) == __double_as_longlong(m)) active = false;
        else ++t;
      }
    }
  }
  nf = wave_sum(nf);
  if ((threadIdx.x & 63) == 0 && nf) atomicAdd(fixed, nf);
}

// (4) the safety net after the parallel rounds, one wave: the chunks still flagged (lflag,
// from the last k_ema_check_flag), in increasing order (found 64 at a time by a ballot
// over the flags; nothing to do when the count is zero), each recomputed from its
// predecessor's true end state, and the next chunk too while its start state disagrees
// with the new end. Afterwards every cleaned sample equals the reference's. fixed +=
// chunks recomputed. The state is wave-uniform; 64 samples are loaded coalesced, stepped
// lane by lane in order (readlane), and stored coalesced.
__global__ __launch_bounds__(64) void k_ema_fix(const float *__restrict__ x, int64_t nx, int64_t n, float *__restrict__ y,
                                                double *__restrict__ warm, double *__restrict__ end, int64_t nch,
                                                const unsigned long long *__restrict__ cnt,
                                                const uint8_t *__restrict__ lflag,
                                                unsigned long long *__restrict__ fixed) {
  if (blockIdx.x != 0 || *cnt == 0) return;
  const int lane = threadIdx.x;
  unsigned long long nf = 0;
  int64_t done = 0; // chunks below this are final
  for (int64_t b16 = 0; b16 < nch; b16 += 1024) { // 16 flags per lane per load
    uint4 q = make_uint4(0, 0, 0, 0);
    if (b16 + 16 * lane + 16 <= nch) q = *reinterpret_cast<const uint4 *>(lflag + b16 + 16 * lane);
    else for (int i = 0; i < 16 && b16 + 16 * lane + i < nch; ++i) reinterpret_cast<uint8_t *>(&q)[i] = lflag[b16 + 16 * lane + i];
    if (!__ballot((q.x | q.y | q.z | q.w) != 0)) continue;
    for (int sub = 0; sub < 16; ++sub) {
    const int64_t base = b16 + 64 * sub;
    uint64_t fl = __ballot(base + lane < nch && lflag[base + lane] != 0);
    while (fl) {
      int64_t t = base + __builtin_ctzll(fl);
      fl &= fl - 1;
      if (t < done) continue;
      double m = end[t - 1]; // true: every earlier chunk is verified or recomputed
      for (;;) {             // (m carries the state through the chain, no re-read)
        if (lane == 0) warm[t] = m;
        const int64_t a = t * kL, b = a + kL < n ? a + kL : n;
        for (int64_t b0 = a; b0 < b; b0 += 64) {
          const float xv = b0 + lane < b && b0 + lane < nx ? x[b0 + lane] : 0.f;
          const int nj = b - b0 < 64 ? (int)(b - b0) : 64;
          float yv = 0.f;
          for (int j = 0; j < nj; ++j) {
            const float xj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), j));
            m = ema_step(m, xj);
            const float o = (float)((double)xj - m);
            yv = lane == j ? o : yv;
          }
          if (b0 + lane < b) y[b0 + lane] = yv;
        }
        if (lane == 0) end[t] = m; // the chunk's true end state (read back by sharded receivers)
        ++nf;
        if (t + 1 < nch && __double_as_longlong(warm[t + 1]) != __double_as_longlong(m)) { ++t; continue; }
        done = t + 2; // chunk t + 1 started from this true state
        break;
      }
    }
    }
  }
  if (lane == 0 && nf) *fixed += nf;
}

// 32-sample block sums of the cleaned stream: z_b = sum y[k] y[k+256], e_b = sum y[k]^2
// over k in [32 b, 32 b + 32) (a screening hint, any order and precision: the host
// recomputes anything it misses, and hot means a metric >= 0.25 against the reference's
// 0.5). Four samples per lane (float4, coalesced) in fp32, the 8 lanes of a block combined
// by DPP within the row (quad swaps, then the half-row mirror): no LDS. (fp64 sums with
// 8-lane bpermute shuffles: 1.9 ms for a 32k-chunk stream, 1.9 TB/s.) n is a multiple of 4.
__device__ __forceinline__ float dpp_add(float v, int ctrl) {
  const int o = ctrl == 0xB1 ? __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)
              : ctrl == 0x4E ? __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)
                             : __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false);
  return v + __int_as_float(o);
}
__global__ __launch_bounds__(256) void k_sc_blocks(const float *__restrict__ y, int64_t n, int64_t nblk,
                                                   double2 *__restrict__ ze) {
  const int64_t k = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  // raw buffer loads over this workgroup's 1024 + 256 samples (dwords past n read 0): plain
  // float4 reads under the range tests compiled to four dword loads each
  const int64_t base = (int64_t)blockIdx.x * 1024;
  const int64_t len = n - base < 1024 + 256 ? (n - base > 0 ? n - base : 0) : 1024 + 256;
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void *)(y + base), (short)0, (int)(4 * len),
                                                                      0x00020000);
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 av = __builtin_amdgcn_raw_buffer_load_b128(yr, 16 * (int)threadIdx.x, 0, 0);
  const u4 cv = __builtin_amdgcn_raw_buffer_load_b128(yr, 16 * (int)threadIdx.x + 1024, 0, 0);
  const float4 a = make_float4(__uint_as_float(av[0]), __uint_as_float(av[1]), __uint_as_float(av[2]), __uint_as_float(av[3]));
  const float4 c = make_float4(__uint_as_float(cv[0]), __uint_as_float(cv[1]), __uint_as_float(cv[2]), __uint_as_float(cv[3]));
  float z = a.x * c.x, e = a.x * a.x;
  z = fmaf(a.y, c.y, z); e = fmaf(a.y, a.y, e);
  z = fmaf(a.z, c.z, z); e = fmaf(a.z, a.z, e);
  z = fmaf(a.w, c.w, z); e = fmaf(a.w, a.w, e);
  z = dpp_add(z, 0xB1); e = dpp_add(e, 0xB1);   // lanes 0<->1, 2<->3
  z = dpp_add(z, 0x4E); e = dpp_add(e, 0x4E);   // 0<->2, 1<->3: the quad's sum
  z = dpp_add(z, 0x141); e = dpp_add(e, 0x141); // lane i <-> 7 - i: the other quad
  const int64_t b = k >> 5;
  if ((threadIdx.x & 7) == 0 && b < nblk) ze[b] = make_double2((double)z, (double)e);
}

// hot flag per block: the metric at position 32 b (window = 8 blocks) >= thresh
__global__ __launch_bounds__(256) void k_sc_screen(const double2 *__restrict__ ze, int64_t nblk, float thresh,
                                                   uint8_t *__restrict__ hot) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblk) return;
  double p = 0.0, ra = 0.0, rb = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (b + q < nblk) { const double2 v = ze[b + q]; p += v.x; ra += v.y; }
    if (b + 8 + q < nblk) rb += ze[b + 8 + q].y;
  }
  hot[b] = (ra > 0.001 && rb > 0.001 && (p * p) / (ra * rb) >= (double)thresh) ? 1 : 0;
}

// Fine ranges from the hot flags (the host's merge of [32 b - 448, 32 b + 479] over hot
// blocks b, in order): two hot blocks at most kMergeGap apart share a range, so a range
// starts at a hot block with no hot block in the kMergeGap before it and ends at one with
// none in the kMergeGap after it. (1) starts per workgroup, (2) their exclusive scan
// (one workgroup), (3) each start's range written at its rank: ranges in stream order.
constexpr int kMergeGap = 29; // 32 (b - b') <= 2 * 448 + 32
__device__ __forceinline__ bool range_start(const uint8_t *hot, int64_t nhot, int64_t b) {
  if (b >= nhot || !hot[b]) return false;
  for (int64_t j = max<int64_t>(0, b - kMergeGap); j < b; ++j)
    if (hot[j]) return false;
  return true;
}
__global__ __launch_bounds__(256) void k_range_count(const uint8_t *__restrict__ hot, int64_t nhot,
                                                     int32_t *__restrict__ wg_count) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = __popcll(__ballot(range_start(hot, nhot, b)));
  __shared__ int wc[4];
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) wg_count[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}
// in place: wg_count[i] -> sum of wg_count[0 .. i); wg_count[nwg] = the total (one workgroup)
__global__ __launch_bounds__(1024) void k_range_scan(int32_t *__restrict__ wg_count, int nwg) {
  __shared__ int part[1024];
  const int t = threadIdx.x, per = (nwg + 1023) / 1024, a = min(nwg, t * per), b = min(nwg, a + per);
  int sum = 0;
  for (int i = a; i < b; ++i) sum += wg_count[i];
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) { // inclusive scan of the partials
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int i = a; i < b; ++i) { const int v = wg_count[i]; wg_count[i] = run; run += v; }
  if (t == 1023) wg_count[nwg] = part[1023];
}
__global__ __launch_bounds__(256) void k_range_write(const uint8_t *__restrict__ hot, int64_t nhot,
                                                     const int32_t *__restrict__ wg_off, int64_t *__restrict__ first,
                                                     int64_t *__restrict__ count) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool st = range_start(hot, nhot, b);
  const unsigned long long m = __ballot(st);
  __shared__ int wc[4];
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (!st) return;
  const int w = threadIdx.x >> 6;
  int off = wg_off[blockIdx.x] + __popcll(m & ((1ull << (threadIdx.x & 63)) - 1));
  for (int k = 0; k < w; ++k) off += wc[k];
  int64_t last = b; // the range's last hot block: none in the kMergeGap after it
  for (int64_t j = b + 1; j < nhot && j - last <= kMergeGap; ++j)
    if (hot[j]) last = j;
  first[off] = 32 * b - 448;
  count[off] = 32 * (last - b) + 32 + 2 * 448;
}

// fine sums for positions first[r] .. first[r] + count[r] - 1 of range r; out index
// base[r] + j. A thread takes kFineP consecutive positions and slides a register window
// over the staged samples: every tap's 16-byte LDS read feeds its positions' 2 kFineP
// fp64 FMAs (one position per lane read a float per FMA pair: 2.7 ms on the 32k-chunk
// stream, LDS-issue bound). Each position's sums are still the reference's, in its order.
constexpr int kFineMaxSym = 1024; // symbol_len bound of k_fine's LDS window (presets: 576 .. 768)
constexpr int kFineT = 128;       // threads per workgroup
constexpr int kFineP = 4;         // consecutive positions per thread
static_assert(kFineT * kFineP == kFinePositions, "k_fine's workgroup span (amodem_internal.h)");
// barg (optional): per workgroup, the first maximum of its positions' metrics (NaN
// skipped, as the refinement's `metric > best`) as (metric, j), at [r * gridDim.x + bx]
__global__ __launch_bounds__(kFineT) void k_fine(const float *__restrict__ y, int64_t n, const double *__restrict__ pre1,
                                                 int sym, double pre1_energy, const int64_t *__restrict__ first,
                                                 const int64_t *__restrict__ base, const int64_t *__restrict__ count,
                                                 int nranges, double *__restrict__ out, double *__restrict__ out_dev,
                                                 double2 *__restrict__ barg) {
  __shared__ double2 red[kFineT / 64];
  // the workgroup's samples [d0, d0 + kFinePositions + sym), plus the register window's
  // read-ahead (sym is a multiple of 4: amod_config_valid)
  __shared__ __attribute__((aligned(16))) float win[kFinePositions + kFineMaxSym + 8];
  const int r = blockIdx.y;
  if (r >= nranges) return;
  const int64_t j0 = (int64_t)blockIdx.x * kFinePositions, cnt = count[r];
  if (j0 >= cnt) { // (whole workgroup) no position: an empty record
    if (barg && threadIdx.x == 0) barg[(int64_t)r * gridDim.x + blockIdx.x] = make_double2(-__builtin_inf(), (double)j0);
    return;
  }
  {
    const int64_t d0 = first[r] + j0;
    for (int i = threadIdx.x; i < kFinePositions + sym + 8; i += kFineT) win[i] = sample_at(y, n, d0 + i);
    __syncthreads();
  }
  const int p0 = kFineP * (int)threadIdx.x;
  const int64_t jt = j0 + p0; // this thread's first position
  double m = -__builtin_inf(), bj = (double)jt;
  if (jt < cnt) {
    double corr[kFineP], se[kFineP];
#pragma unroll
    for (int k = 0; k < kFineP; ++k) corr[k] = se[k] = 0.0;
    const float *const w = win + p0;
    float4 cur = *reinterpret_cast<const float4 *>(w);
    // f32 x f32 products are exact in double, so fma(s, q, corr) is the reference's
    // corr + s * q with its one rounding: half the fp64 operations of mul + add
    for (int i = 0; i < sym; i += 4) {
      const float4 nxt = *reinterpret_cast<const float4 *>(w + i + 4);
      const double sv[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double q = pre1[i + u];
#pragma unroll
        for (int k = 0; k < kFineP; ++k) {
          corr[k] = __builtin_fma(sv[u + k], q, corr[k]);
          se[k] = __builtin_fma(sv[u + k], sv[u + k], se[k]);
        }
      }
      cur = nxt;
    }
#pragma unroll
    for (int k = 0; k < kFineP; ++k) {
      const int64_t j = jt + k;
      if (j >= cnt) break;
      // the metric the refinement compares (app.js:872-875); NaN: the position is skipped
      const double denom = sqrt(se[k] * pre1_energy);
      const double v = denom > 0.001 ? corr[k] / denom : __builtin_nan("");
      if (out) out[base[r] + j] = v;         // (mapped host memory: the host's lookups)
      if (out_dev) out_dev[base[r] + j] = v; // (the device copy k_gap_refine reads)
      if (v == v && v > m) { m = v; bj = (double)j; } // (in order: the first maximum)
    }
  }
  if (!barg) return;
  for (int o = 32; o > 0; o >>= 1) {
    const double om = __shfl_xor(m, o, 64), oj = __shfl_xor(bj, o, 64);
    if (om > m || (om == m && oj < bj)) { m = om; bj = oj; }
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_double2(m, bj);
  __syncthreads();
  if (threadIdx.x == 0) {
    double2 b = red[0];
    for (int k = 1; k < kFineT / 64; ++k)
      if (red[k].x > b.x || (red[k].x == b.x && red[k].y < b.y)) b = red[k];
    barg[(int64_t)r * gridDim.x + blockIdx.x] = b;
  }
}

// Speculative gap scans (the streaming receiver's _scanForPreamble, app.js:775-847, as
// Receiver::scan in stream.cpp replays it). For fine range r: its first fine-metric
// maximum d is where the refinement would put the frame, so the receiver would reset to
// IDLE with its scan at s0 = d + F (ac sums not initialised) in block ceil(s0 / 4096).
// From that state the scan is a function of the stream alone, run here block by block
// with the host's arithmetic in the host's order (IEEE double, no contraction: this file
// is built with -ffp-contract=off) until a detection; the record holds the state the
// host would then be in. The host adopts a record only when its true state matches the
// start exactly; anything else (no detection within the block limit, the ring's oldest
// sample overtaken) is left to the host (status 0).
// One wave runs kGapG gaps in tiles of 64 positions: (A) lane t forms position t's three
// increments for each gap (coalesced loads), (B) lane g advances gap g's three running
// sums through its tile in order and keeps the sums at every position, (C) lane t tests
// position t of each gap: the metric pre-check, and where it passes (or a detection is
// pending) the running best as an inclusive prefix maximum (a later equal metric never
// replaces the earlier: strict '>') and the 0.7 drop on the sums after the position.
__device__ __forceinline__ double rl_d(double v, int j) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), j), hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int64_t rl_l(int64_t v, int j) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), j) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j));
}
#ifndef AMOD_GAPG
#define AMOD_GAPG 4
#endif
// gaps per wave. With the chain lanes (round 5), on the 32k-gap stream: 1 -> 1.80 ms, 2 ->
// 1.06, 4 -> 0.77, 8 -> 0.98 (the 2000-gap stream: 0.24 / 0.25 / 0.32 / 0.46). Round 4,
// one lane per gap's three sums, 2000 gaps: 8 -> 0.59 ms, 2 -> 0.40, 1 -> 0.57
constexpr int kGapG = AMOD_GAPG;
constexpr int kGapS = 66; // LDS row stride (doubles): 16-byte aligned rows, the chain lanes of phase B on distinct banks
__global__ __launch_bounds__(64) void k_gap_scan(const float *__restrict__ y, int64_t n, int64_t lo,
                                                 const int64_t *__restrict__ first, const double2 *__restrict__ barg,
                                                 int nbx, int nranges, int64_t F, int64_t cap, int64_t nblocks,
                                                 int max_blocks, GapScan *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) double inc[3][kGapG][kGapS]; // phase A -> B: increments of each gap's tile positions
  __shared__ __attribute__((aligned(16))) double stt[3][kGapG][kGapS]; // phase B -> C: sums at each tile position, then the tile's end
  constexpr int64_t kBlk = 4096, half = 256;
  const double min_e = 0.001;
  const int lane = threadIdx.x;
  const int r = blockIdx.x * kGapG + lane;
  auto S = [&](int64_t i) -> double { return (double)sample_at(y, n, i - lo); };
  // ---- per-gap state, lane g = gap g
  bool act = lane < kGapG && r < nranges;
  GapScan rec{};
  int64_t pos = 0, blk = 0, blim = 0, scan_end = 0, best_pos = -1, scanned = 0;
  double p = 0.0, ra = 0.0, rb = 0.0, best = 0.0;
  // the block whose scan call steps position pos (oldest-sample check and block limit as
  // the host's scan calls meet them); false: the record stays status 0
  auto to_block = [&]() -> bool {
    for (;;) {
      if (blk >= blim) return false;
      const int64_t total = (blk + 1) * kBlk;
      if (pos < total - cap + 2 * half) return false; // the host re-positions the scan: its own business
      scan_end = total - 2 * half;
      if (pos <= scan_end) return true;
      ++blk;
    }
  };
  if (act) {
    double2 b = barg[(int64_t)r * nbx];
    for (int k = 1; k < nbx; ++k) {
      const double2 v = barg[(int64_t)r * nbx + k];
      if (v.x > b.x) b = v; // (blocks in position order: ties keep the first)
    }
    if (b.x >= 0.1) { // else the refinement fails there: no frame, no record
      pos = lo + first[r] + (int64_t)b.y + F;
      blk = (pos + kBlk - 1) / kBlk;
      rec.s0 = pos; rec.b1 = blk;
      blim = min(nblocks, blk + max_blocks);
      act = to_block();
    } else {
      act = false;
    }
  }
  // The three running sums of gap g (p, ra, rb) are advanced by three chain lanes, lane
  // q = c kGapG + g for sum c: each reads its own LDS row (inc[c][g]) and writes its own
  // (stt[c][g]), so a position costs one read and one write for every gap of the wave (it
  // was three of each with the gap's lane advancing all three sums: k_gap_scan waited on
  // LDS issue for 58 % of its wave cycles). Gap lane g reads the sums back at the tile end.
  const int cg = lane % kGapG;                            // chain lane: its gap
  const bool chain_lane = lane < 3 * kGapG;
  double *const irow = &inc[0][0][0] + lane * kGapS;     // (chain lanes) row c kGapG + g
  double *const srow = &stt[0][0][0] + lane * kGapS;
  double acc = 0.0;                                       // (chain lanes) the sum
  // ---- the window sums at the start, in order (products on the lanes, sums per chain)
  {
    const unsigned long long am = __ballot(act);
    const bool live_chain = chain_lane && ((am >> cg) & 1);
    for (int c = 0; c < (int)half; c += 64) {
      for (int gi = 0; gi < kGapG; ++gi) {
        if (!((am >> gi) & 1)) continue;
        const int64_t base = rl_l(pos, gi) + c;
        const double a = S(base + lane), bb = S(base + lane + half);
        inc[0][gi][lane] = a * bb; inc[1][gi][lane] = a * a; inc[2][gi][lane] = bb * bb;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      if (live_chain)
        for (int m = 0; m < 64; m += 2) { const double2 v = *reinterpret_cast<const double2 *>(irow + m); acc += v.x; acc += v.y; }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
  }
  // ---- tiles; each tile's samples are loaded during the previous one (a continuing
  // gap's next tile starts where this one ends, whatever happens at the block's end)
  float va[kGapG], vm[kGapG], vb[kGapG];
  auto load_tile = [&](unsigned long long live, int64_t at_lane) { // at_lane: lane g's tile start
#pragma unroll
    for (int gi = 0; gi < kGapG; ++gi) {
      const int64_t x = ((live >> gi) & 1) ? rl_l(at_lane, gi) + lane - lo : -(int64_t)(1 << 20);
      va[gi] = sample_at(y, n, x);
      vm[gi] = sample_at(y, n, x + half);
      vb[gi] = sample_at(y, n, x + 2 * half);
    }
  };
  load_tile(__ballot(act), pos);
  for (;;) {
    const unsigned long long am = __ballot(act);
    if (!am) break;
    const int T = act ? (int)min<int64_t>(64, scan_end - pos + 1) : 0; // lane g: gap g's tile length
    // (A) lane t: increments of position t of each live gap (none at scan_end)
#pragma unroll
    for (int gi = 0; gi < kGapG; ++gi) {
      const bool up = ((am >> gi) & 1) && rl_l(pos, gi) + lane < rl_l(scan_end, gi);
      const double a_out = va[gi], mid = vm[gi], b_in = vb[gi];
      inc[0][gi][lane] = up ? mid * b_in - a_out * mid : 0.0;
      inc[1][gi][lane] = up ? mid * mid - a_out * a_out : 0.0;
      inc[2][gi][lane] = up ? b_in * b_in - mid * mid : 0.0;
    }
    load_tile(am, pos + T); // the next tile's samples, in flight under this one
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // (B) chain lane q: its sum through gap g's tile, in order (the value before each
    // position's update is the sum at that position; T: the sum after the tile)
    {
      const int tu_g = act ? (int)min<int64_t>(T, scan_end - pos) : 0; // (lane g) positions with an update
      int Tq = 0, tq = 0;
#pragma unroll
      for (int gi = 0; gi < kGapG; ++gi) {
        const int Tg = __builtin_amdgcn_readlane(T, gi), ug = __builtin_amdgcn_readlane(tu_g, gi);
        if (cg == gi) { Tq = Tg; tq = ug; }
      }
      if (chain_lane && ((am >> cg) & 1)) {
        int t = 0;
        for (; t + 8 <= tq; t += 8) { // eight increments read ahead of the dependent sum, two per read
          double2 i2[4], s2[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) i2[u] = *reinterpret_cast<const double2 *>(irow + t + 2 * u);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            s2[u].x = acc; acc += i2[u].x;
            s2[u].y = acc; acc += i2[u].y;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) *reinterpret_cast<double2 *>(srow + t + 2 * u) = s2[u];
        }
        for (; t < Tq; ++t) {
          srow[t] = acc;
          if (t < tq) acc += irow[t];
        }
        srow[Tq] = acc;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (act) { p = stt[0][lane][T]; ra = stt[1][lane][T]; rb = stt[2][lane][T]; } // (lane g) the sums after the tile
    // (C) lane t: position t of each live gap
    bool det_here = false; // lane g: gap g detected in this tile
    for (int gi = 0; gi < kGapG; ++gi) {
      if (!((am >> gi) & 1)) continue;
      const int Tg = __builtin_amdgcn_readlane(T, gi);
      const double sp = stt[0][gi][lane], sa = stt[1][gi][lane], sb = stt[2][gi][lane];
      const bool c = lane < Tg && sa > min_e && sb > min_e && sp * sp >= 0.49 * (sa * sb);
      const unsigned long long hits = __ballot(c);
      const double bin = rl_d(best, gi);
      const int64_t bpin = rl_l(best_pos, gi);
      if (!(bin > 0.5 && bpin >= 0) && !hits) continue;
      const int ln = min(lane + 1, 64);
      const double pa = stt[0][gi][ln], raa = stt[1][gi][ln], rba = stt[2][gi][ln]; // sums after position t
      double key = -__builtin_inf();
      int kidx = 64;
      if (c) {
        const double metric = (sp * sp) / (sa * sb);
        if (metric > 0.5) { key = metric; kidx = lane; }
      }
      for (int o = 1; o < 64; o <<= 1) {
        const double ok = __shfl_up(key, o, 64);
        const int oi = __shfl_up(kidx, o, 64);
        if (lane >= o && (ok > key || (ok == key && oi < kidx))) { key = ok; kidx = oi; }
      }
      const int64_t base = rl_l(pos, gi);
      double bj = bin;
      int64_t bpj = bpin;
      if (key > bj) { bj = key; bpj = base + kidx; }
      bool det = false;
      if (lane < Tg && bj > 0.5 && bpj >= 0 && raa > min_e && rba > min_e) det = (pa * pa) / (raa * rba) < bj * 0.7;
      const unsigned long long dm = __ballot(det);
      if (dm) {
        const int j = __builtin_ctzll(dm);
        const int64_t pre = rl_l(bpj, j);
        const double dp = rl_d(pa, j), dra = rl_d(raa, j), drb = rl_d(rba, j);
        if (lane == gi) {
          rec.status = 1; rec.det_block = blk; rec.pre_pos = pre; rec.ac_pos = pos + j + 1;
          rec.p = dp; rec.ra = dra; rec.rb = drb; rec.scanned = scanned + j + 1;
          det_here = true;
        }
      } else {
        const double nb = rl_d(bj, Tg - 1);
        const int64_t nbp = rl_l(bpj, Tg - 1);
        if (lane == gi) { best = nb; best_pos = nbp; }
      }
    }
    __builtin_amdgcn_wave_barrier();
    // (D) lane g: the tile done; at the block's end the commit or the next block
    if (act) {
      if (det_here) {
        act = false;
      } else {
        pos += T; scanned += T;
        if (pos > scan_end) {
          if (best > 0.5 && best_pos >= 0) { // end-of-block commit
            rec.status = 1; rec.det_block = blk; rec.pre_pos = best_pos; rec.ac_pos = pos;
            rec.p = p; rec.ra = ra; rec.rb = rb; rec.scanned = scanned;
            act = false;
          } else {
            ++blk; best = 0.0; best_pos = -1;
            act = to_block();
          }
        }
      }
    }
  }
  if (lane < kGapG && r < nranges) out[r] = rec;
}

// The refinement (_refineAndCollect, app.js:849-898) of each gap record's detection, from
// k_fine's metrics: over d in [pre_pos - radius, pre_pos + radius] the first d whose metric
// is the largest (the reference's `metric > best` from best = -inf: NaN never wins, a later
// equal metric never replaces an earlier one). Valid (ref_ok) only when one fine range holds
// the whole window; the host uses it when its own window is exactly this one (the ring has
// not overtaken the start). One wave per record.
__global__ __launch_bounds__(256) void k_gap_refine(GapScan *__restrict__ g, int nrec, int64_t lo,
                                                    const int64_t *__restrict__ first, const int64_t *__restrict__ base,
                                                    const int64_t *__restrict__ count, int nranges,
                                                    const double *__restrict__ metric, int64_t radius) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= nrec) return;
  const int64_t pre = g[r].pre_pos;
  int ok = g[r].status == 1;
  const int64_t fs = pre - radius - lo, fe = pre + radius - lo; // local positions
  int k = -1;
  if (ok) { // the last range starting at or before fs
    int a = 0, b = nranges; // first[a..b) ascending
    while (a < b) { const int mid = (a + b) >> 1; if (first[mid] <= fs) a = mid + 1; else b = mid; }
    k = a - 1;
    ok = k >= 0 && fe < first[max(k, 0)] + count[max(k, 0)];
  }
  if (!ok) {
    if (lane == 0) g[r].ref_ok = 0;
    return;
  }
  const double *const mv = metric + base[k] + (fs - first[k]);
  double m = -__builtin_inf();
  int64_t mj = INT64_MAX;
  for (int64_t j = lane; j <= fe - fs; j += 64) {
    const double v = mv[j];
    if (v > m) { m = v; mj = j; } // per lane: the first strict maximum of its positions
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double om = __shfl_xor(m, o, 64);
    const int64_t oj = __shfl_xor(mj, o, 64);
    if (om > m || (om == m && oj < mj)) { m = om; mj = oj; }
  }
  if (lane == 0) {
    g[r].ref_best = m;
    g[r].ref_pos = m > -__builtin_inf() ? lo + fs + mj : pre;
    g[r].ref_ok = 1;
  }
}

// the host's sparse copy of the cleaned stream: compact granule j (1024 samples) is stream
// granule src[j]; one workgroup per granule, float4 per thread, coalesced both ways
__global__ __launch_bounds__(256) void k_gather(const float *__restrict__ y, const int32_t *__restrict__ src,
                                                float *__restrict__ out) {
  const int64_t j = blockIdx.x;
  const float4 *const a = reinterpret_cast<const float4 *>(y + (int64_t)src[j] * 1024);
  reinterpret_cast<float4 *>(out + j * 1024)[threadIdx.x] = a[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_window(const float *__restrict__ y, int64_t n, const int64_t *__restrict__ pos,
                                                const int32_t *__restrict__ len, const int64_t *__restrict__ woff,
                                                float *__restrict__ out) {
  __shared__ float red[4];
  __shared__ int red_nan[4];
  const int w = blockIdx.x, tid = threadIdx.x;
  const int64_t p = pos[w], o = woff[w];
  const int L = len[w];
  // Math.max over |x| (app.js:920): a NaN sample makes mx NaN, and then `mx > 1e-6` is false
  // (fmaxf would skip it): tracked beside the max
  float mx = 0.f;
  bool nan = false;
  // a window inside the stream (every one the receiver cuts): float4 buffer loads over it,
  // four in flight per thread (dwords past L read 0; the output offset o is a multiple of 4)
  const bool inside = p >= 0 && p + L <= n;
  const int nq = (L + 3) >> 2;
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void *)(y + (inside ? p : 0)), (short)0, (int)(4 * (int64_t)L), 0x00020000);
  auto ld = [&](int q) {
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(yr, 16 * q, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
  };
  if (inside) {
    for (int q0 = tid; q0 < nq; q0 += 4 * 256) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld(q0 + 256 * u); // (past nq: past L, zeros)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
        nan |= (v[u].x != v[u].x) | (v[u].y != v[u].y) | (v[u].z != v[u].z) | (v[u].w != v[u].w);
      }
    }
  } else {
    for (int i = tid; i < L; i += 256) {
      const float v = sample_at(y, n, p + i);
      mx = fmaxf(mx, fabsf(v));
      nan |= v != v;
    }
  }
  mx = wave_max(mx);
  const bool wnan = __ballot(nan) != 0;
  if ((tid & 63) == 0) { red[tid >> 6] = mx; red_nan[tid >> 6] = wnan; }
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const bool norm = !(red_nan[0] | red_nan[1] | red_nan[2] | red_nan[3]) && (double)mx > 1e-6;
  const double dm = (double)mx;
  if (inside) {
    float4 *const o4 = reinterpret_cast<float4 *>(out + o);
    for (int q = tid; q < nq; q += 256) {
      const float4 v = ld(q);
      o4[q] = norm ? make_float4((float)((double)v.x / dm), (float)((double)v.y / dm), (float)((double)v.z / dm),
                                 (float)((double)v.w / dm))
                   : v;
    }
  } else {
    for (int i = tid; i < L; i += 256) {
      const float v = sample_at(y, n, p + i);
      out[o + i] = norm ? (float)((double)v / dm) : v;
    }
  }
}

} // namespace
} // namespace amod

extern "C" {
int64_t amod_ema_chunk() { return amod::kL; }
// DC removal of x[0, n) from a zero EMA state into y (x read for [0, nx), zero past it); warm / end / scr: nch = ceil(n / L)
// doubles each; list: nch int64; apow: L doubles (a^j); fixed: 2 counters
namespace {
// the EMA's experiment shapes come from the context's knobs (read at amod_open)
int ema_per(const amod::Knobs *kn) { return kn && kn->ema_per > 0 ? kn->ema_per : amod::kPerDefault; }
int ema_warm(const amod::Knobs *kn) { return kn && kn->ema_warm >= 0 ? kn->ema_warm : amod::kWarmDefault; }
int ema_rounds(const amod::Knobs *kn) { return kn && kn->ema_rounds >= 0 ? kn->ema_rounds : amod::kEmaRounds; }
} // namespace

// samples per k_ema_out wave (64 lanes x per chunks): a piece of the stream that is a
// multiple of this can be cleaned as soon as it and the samples before it have landed
int64_t amod_ema_wave_samples(const amod::Knobs *kn) { return (int64_t)64 * ema_per(kn) * amod::kL; }

// stages (1) + (2) for the waves of samples [s0, s1) (s0 a multiple of
// amod_ema_wave_samples(); s1 too, or the end n): their chunk contributions, then their
// outputs; every sample before s1 must have landed (warm-up reads the chunks before s0)
hipError_t amod_launch_ema_part(const float *x, int64_t nx, int64_t n, float *y, double *warm, double *end, double *scr,
                                const double *apow, int64_t s0, int64_t s1, hipStream_t s, const amod::Knobs *kn) {
  const int64_t nch = (n + amod::kL - 1) / amod::kL;
  const int64_t c0 = s0 / amod::kL, c1 = std::min(nch, (s1 + amod::kL - 1) / amod::kL);
  if (c1 <= c0) return hipSuccess;
  double A = 1.0;
  for (int i = 0; i < amod::kL; ++i) A *= amod::kAlpha;
  hipLaunchKernelGGL(amod::k_ema_contrib, dim3((unsigned)((c1 - c0 + 3) / 4)), dim3(256), 0, s, x, nx, apow, scr, c0, c1);
  const int warm_chunks = ema_warm(kn);
  const int per = ema_per(kn);
  const int64_t span = (int64_t)64 * per; // chunks per wave
  const int64_t w0 = c0 / span, w1 = (c1 + span - 1) / span;
  hipLaunchKernelGGL(amod::k_ema_out, dim3((unsigned)((w1 - w0 + 3) / 4)), dim3(256), 0, s, x, nx, n, scr, A, y, warm,
                     end, nch, warm_chunks, per, w0, w1);
  return hipGetLastError();
}

// (3) + (4) once every part is enqueued: the check rounds and the fixes
hipError_t amod_launch_ema_fix(const float *x, int64_t nx, int64_t n, float *y, double *warm, double *end,
                               int64_t *list, unsigned long long *fixed, hipStream_t s, const amod::Knobs *kn) {
  const int64_t nch = (n + amod::kL - 1) / amod::kL;
  if (nch <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(fixed, 0, 2 * sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  uint8_t *const lflag = reinterpret_cast<uint8_t *>((reinterpret_cast<uintptr_t>(list + nch) + 15) & ~uintptr_t(15));
  const int rounds = ema_rounds(kn);
  for (int r = 0; r < rounds; ++r) {
    e = hipMemsetAsync(fixed + 1, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(amod::k_ema_check_flag, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, warm, end, nch,
                       fixed + 1, list, lflag);
    hipLaunchKernelGGL(amod::k_ema_runs, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, x, nx, n, y, warm, end,
                       nch, fixed + 1, list, lflag, fixed);
  }
  e = hipMemsetAsync(fixed + 1, 0, sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(amod::k_ema_check_flag, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, warm, end, nch,
                     fixed + 1, list, lflag);
  hipLaunchKernelGGL(amod::k_ema_fix, dim3(1), dim3(64), 0, s, x, nx, n, y, warm, end, nch, fixed + 1, lflag, fixed);
  return hipGetLastError();
}

hipError_t amod_launch_ema(const float *x, int64_t nx, int64_t n, float *y, double *warm, double *end, double *scr,
                           int64_t *list, const double *apow, unsigned long long *fixed, hipStream_t s,
                           const amod::Knobs *kn) {
  const int64_t nch = (n + amod::kL - 1) / amod::kL;
  if (nch <= 0) return hipSuccess;
  hipError_t e = amod_launch_ema_part(x, nx, n, y, warm, end, scr, apow, 0, n, s, kn);
  if (e != hipSuccess) return e;
  return amod_launch_ema_fix(x, nx, n, y, warm, end, list, fixed, s, kn);
}

hipError_t amod_launch_sc_screen(const float *y, int64_t n, float thresh, double2 *ze, uint8_t *hot, hipStream_t s) {
  const int64_t nblk = (n + 31) / 32;
  if (nblk <= 0) return hipSuccess;
  if (n % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(amod::k_sc_blocks, dim3((unsigned)((32 * nblk + 1023) / 1024)), dim3(256), 0, s, y, n, nblk, ze);
  hipLaunchKernelGGL(amod::k_sc_screen, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, ze, nblk, thresh, hot);
  return hipGetLastError();
}
// the fine ranges of the hot flags: first[r], count[r] for r < *nranges (wg: nhot / 256 + 2
// ints of scratch); first / count hold max_ranges entries
hipError_t amod_launch_ranges(const uint8_t *hot, int64_t nhot, int32_t *wg, int64_t *first, int64_t *count,
                              hipStream_t s) {
  if (nhot <= 0) return hipMemsetAsync(wg, 0, sizeof(int32_t), s);
  const int nwg = (int)((nhot + 255) / 256);
  hipLaunchKernelGGL(amod::k_range_count, dim3((unsigned)nwg), dim3(256), 0, s, hot, nhot, wg);
  hipLaunchKernelGGL(amod::k_range_scan, dim3(1), dim3(1024), 0, s, wg, nwg);
  hipLaunchKernelGGL(amod::k_range_write, dim3((unsigned)nwg), dim3(256), 0, s, hot, nhot, wg, first, count);
  return hipGetLastError();
}
hipError_t amod_launch_fine(const float *y, int64_t n, const double *pre1, int sym, double pre1_energy,
                            const int64_t *first, const int64_t *base, const int64_t *count, int nranges,
                            int64_t maxcount, double *out, double *out_dev, double2 *barg, hipStream_t s) {
  if (nranges <= 0 || maxcount <= 0) return hipSuccess;
  if (sym <= 0 || sym > amod::kFineMaxSym) return hipErrorInvalidValue;
  hipLaunchKernelGGL(amod::k_fine, dim3((unsigned)((maxcount + amod::kFinePositions - 1) / amod::kFinePositions), nranges),
                     dim3(amod::kFineT), 0, s, y, n, pre1, sym,
                     pre1_energy, first, base, count, nranges, out, out_dev, barg);
  return hipGetLastError();
}
hipError_t amod_launch_gap_scan(const float *y, int64_t n, int64_t lo, const int64_t *first, const double2 *barg,
                                int nbx, int nranges, int64_t F, int64_t cap, int64_t nblocks, int max_blocks,
                                amod::GapScan *out, hipStream_t s) {
  if (nranges <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_gap_scan, dim3((unsigned)((nranges + amod::kGapG - 1) / amod::kGapG)), dim3(64), 0, s, y, n,
                     lo, first, barg,
                     nbx, nranges, F, cap, nblocks, max_blocks, out);
  return hipGetLastError();
}
hipError_t amod_launch_gap_refine(amod::GapScan *g, int nrec, int64_t lo, const int64_t *first, const int64_t *base,
                                  const int64_t *count, int nranges, const double *metric, int64_t radius, hipStream_t s) {
  if (nrec <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_gap_refine, dim3((unsigned)((nrec + 3) / 4)), dim3(256), 0, s, g, nrec, lo, first, base,
                     count, nranges, metric, radius);
  return hipGetLastError();
}
hipError_t amod_launch_gather(const float *y, const int32_t *src, int ng, float *out, hipStream_t s) {
  if (ng <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_gather, dim3(ng), dim3(256), 0, s, y, src, out);
  return hipGetLastError();
}
hipError_t amod_launch_window(const float *y, int64_t n, const int64_t *pos, const int32_t *len, const int64_t *woff,
                              int nwin, float *out, hipStream_t s) {
  if (nwin <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_window, dim3(nwin), dim3(256), 0, s, y, n, pos, len, woff, out);
  return hipGetLastError();
}
}
