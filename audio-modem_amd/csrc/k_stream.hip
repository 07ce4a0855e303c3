// k_stream.hip — GPU pieces of the streaming receiver (app.js StreamingReceiver 706-998).
//
//   k_ema        processAudioBlock's DC removal (app.js:751-755): the EMA
//                m_i = 0.999 m_{i-1} + (1 - 0.999) x_i in IEEE double, cleaned_i =
//                f32(x_i - m_i), bit-exact. One lane per chunk of L samples: the lane
//                first runs the recurrence over the W samples before its chunk from 0
//                (the map contracts by 0.999 per step, so chains from different
//                states coalesce bit for bit after ~36k steps), then over its chunk,
//                16 samples per float4 x4 load/store. The state it reached at its
//                chunk start is kept for k_ema_fix.
//   k_ema_fix    one lane walks the chunks in order: a chunk whose warm-up state is
//                not bit-equal to its predecessor's true end state is recomputed from
//                that state. Afterwards every cleaned sample equals the reference's.
//   k_sc_blocks  fp64 32-sample block sums (coalesced, 32-lane reductions), then
//   k_sc_screen  hot-block screening for the fine precompute: the Schmidl-Cox metric
//                at each block start from 8-block window sums; only a hint (the host
//                recomputes anything the hint missed).
//   k_fine       _refineAndCollect's cross-correlation sums (app.js:864-877) for a
//                list of position ranges: corr = sum seg[i] pre1[i] and sEnergy =
//                sum seg[i]^2 in the reference's order, one lane per position, IEEE
//                double (f32 x f32 products are exact in double).
//   k_window     _demodulateFrame's per-window peak normalisation (app.js:916-925):
//                mx = max |x|, x / mx when mx > 1e-6 (f32 of the double quotient).
// Built with -ffp-contract=off.
#include "amodem_internal.h"

namespace amod {
namespace {

__device__ __forceinline__ float sample_at(const float *x, int64_t n, int64_t i) { return (i >= 0 && i < n) ? x[i] : 0.f; }

constexpr double kAlpha = 0.999;
constexpr double kOneMinusAlpha = 1.0 - 0.999; // (1 - this.dcAlpha), evaluated in double

__global__ __launch_bounds__(64) void k_ema(const float *__restrict__ x, int64_t n, int64_t L, int64_t W,
                                            float *__restrict__ y, double *__restrict__ warm,
                                            double *__restrict__ end, int64_t nchunks) {
  const int64_t t = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= nchunks) return;
  const int64_t s = t * L, e = s + L < n ? s + L : n, w0 = s - W > 0 ? s - W : 0;
  double m = 0.0;
  int64_t i = w0;
  // 16-sample steps on float4 loads (x is 16-byte aligned; L, W multiples of 16)
  for (; i + 16 <= s; i += 16) {
    const float4 *p = reinterpret_cast<const float4 *>(x + i);
    const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    const float v[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) m = kAlpha * m + kOneMinusAlpha * (double)v[k];
  }
  for (; i < s; ++i) m = kAlpha * m + kOneMinusAlpha * (double)x[i];
  warm[t] = m;
  for (; i + 16 <= e; i += 16) {
    const float4 *p = reinterpret_cast<const float4 *>(x + i);
    const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    const float v[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    float o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      m = kAlpha * m + kOneMinusAlpha * (double)v[k];
      o[k] = (float)((double)v[k] - m);
    }
    float4 *r = reinterpret_cast<float4 *>(y + i);
    r[0] = make_float4(o[0], o[1], o[2], o[3]);
    r[1] = make_float4(o[4], o[5], o[6], o[7]);
    r[2] = make_float4(o[8], o[9], o[10], o[11]);
    r[3] = make_float4(o[12], o[13], o[14], o[15]);
  }
  for (; i < e; ++i) {
    m = kAlpha * m + kOneMinusAlpha * (double)x[i];
    y[i] = (float)((double)x[i] - m);
  }
  end[t] = m;
}

__global__ void k_ema_fix(const float *__restrict__ x, int64_t n, int64_t L, float *__restrict__ y,
                          const double *__restrict__ warm, double *__restrict__ end, int64_t nchunks,
                          unsigned long long *__restrict__ fixed) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double prev = end[0];
  unsigned long long nf = 0;
  for (int64_t t = 1; t < nchunks; ++t) {
    if (__double_as_longlong(warm[t]) == __double_as_longlong(prev)) {
      prev = end[t];
      continue;
    }
    double m = prev;
    const int64_t s = t * L, e = s + L < n ? s + L : n;
    for (int64_t i = s; i < e; ++i) {
      m = kAlpha * m + kOneMinusAlpha * (double)x[i];
      y[i] = (float)((double)x[i] - m);
    }
    prev = m;
    end[t] = m; // the chunk's true end state (read back by sharded receivers)
    ++nf;
  }
  *fixed = nf;
}

// 32-sample block sums of the cleaned stream in fp64: z_b = sum y[k] y[k+256], e_b =
// sum y[k]^2 over k in [32 b, 32 b + 32); one lane per sample, 32-lane reductions
__global__ __launch_bounds__(256) void k_sc_blocks(const float *__restrict__ y, int64_t n, int64_t nblk,
                                                   double2 *__restrict__ ze) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const double a = sample_at(y, n, k), c = sample_at(y, n, k + 256);
  double z = a * c, e = a * a;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) { z += __shfl_xor(z, o, 32); e += __shfl_xor(e, o, 32); }
  const int64_t b = k >> 5;
  if ((threadIdx.x & 31) == 0 && b < nblk) ze[b] = make_double2(z, e);
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

// fine sums for positions first[r] .. first[r] + count[r] - 1 of range r; out index
// base[r] + j; one lane per position
__global__ __launch_bounds__(256) void k_fine(const float *__restrict__ y, int64_t n, const float *__restrict__ pre1,
                                              int sym, const int64_t *__restrict__ first,
                                              const int64_t *__restrict__ base, const int64_t *__restrict__ count,
                                              int nranges, double2 *__restrict__ out) {
  const int r = blockIdx.y;
  if (r >= nranges) return;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= count[r]) return;
  const int64_t d = first[r] + j;
  double corr = 0.0, se = 0.0;
  for (int i = 0; i < sym; ++i) {
    const double s = sample_at(y, n, d + i);
    corr += s * (double)pre1[i];
    se += s * s;
  }
  out[base[r] + j] = make_double2(corr, se);
}

__global__ __launch_bounds__(256) void k_window(const float *__restrict__ y, int64_t n, const int64_t *__restrict__ pos,
                                                const int32_t *__restrict__ len, const int64_t *__restrict__ woff,
                                                float *__restrict__ out) {
  __shared__ float red[4];
  const int w = blockIdx.x, tid = threadIdx.x;
  const int64_t p = pos[w], o = woff[w];
  const int L = len[w];
  float mx = 0.f;
  for (int i = tid; i < L; i += 256) mx = fmaxf(mx, fabsf(sample_at(y, n, p + i)));
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const double dm = (double)mx;
  for (int i = tid; i < L; i += 256) {
    const float v = sample_at(y, n, p + i);
    out[o + i] = dm > 1e-6 ? (float)((double)v / dm) : v;
  }
}

} // namespace
} // namespace amod

extern "C" {
hipError_t amod_launch_ema(const float *x, int64_t n, int64_t L, int64_t W, float *y, double *warm, double *end,
                           unsigned long long *fixed, hipStream_t s) {
  const int64_t nchunks = (n + L - 1) / L;
  if (nchunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_ema, dim3((unsigned)((nchunks + 63) / 64)), dim3(64), 0, s, x, n, L, W, y, warm, end,
                     nchunks);
  hipLaunchKernelGGL(amod::k_ema_fix, dim3(1), dim3(64), 0, s, x, n, L, y, warm, end, nchunks, fixed);
  return hipGetLastError();
}
hipError_t amod_launch_sc_screen(const float *y, int64_t n, float thresh, double2 *ze, uint8_t *hot, hipStream_t s) {
  const int64_t nblk = (n + 31) / 32;
  if (nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_sc_blocks, dim3((unsigned)((32 * nblk + 255) / 256)), dim3(256), 0, s, y, n, nblk, ze);
  hipLaunchKernelGGL(amod::k_sc_screen, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, ze, nblk, thresh, hot);
  return hipGetLastError();
}
hipError_t amod_launch_fine(const float *y, int64_t n, const float *pre1, int sym, const int64_t *first,
                            const int64_t *base, const int64_t *count, int nranges, int64_t maxcount, double2 *out,
                            hipStream_t s) {
  if (nranges <= 0 || maxcount <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_fine, dim3((unsigned)((maxcount + 255) / 256), nranges), dim3(256), 0, s, y, n, pre1, sym,
                     first, base, count, nranges, out);
  return hipGetLastError();
}
hipError_t amod_launch_window(const float *y, int64_t n, const int64_t *pos, const int32_t *len, const int64_t *woff,
                              int nwin, float *out, hipStream_t s) {
  if (nwin <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_window, dim3(nwin), dim3(256), 0, s, y, n, pos, len, woff, out);
  return hipGetLastError();
}
}
