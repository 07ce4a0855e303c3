// k_tx.hip — GPU transmitter: modulateOFDM + the frame builders, bit-exact (gfx950).
//
// Reference: modulateOFDM (modem.js:322-362), buildTransmitSignal (498-555) and
// buildChunkOFDMFrame (718-756). One 256-thread workgroup per frame:
//
//   data symbols   wave w builds symbols w, w+4, ...: the spectrum of symbol s
//                  (pilots 1+0i, constellation points of the repeated packet bits,
//                  Hermitian mirror with the reference's signed zeros) goes straight
//                  into registers in bit-reversed order; the 9 radix-2 stages of
//                  fftIterative (26-47, inverse) run as three register passes of
//                  three stages with two LDS exchanges per wave, every butterfly the
//                  reference's own operation sequence on the reference's twiddle
//                  recurrence (tabulated on the host); x 1/512, f32 (addCP 202-208)
//   silence        zeros
//   normalise      0.8 / max|signal| over the frame (548-552): the workgroup's max,
//                  then every sample of the frame rescaled as f32(f64(x) * s)
//
// IEEE double without contraction (built with -ffp-contract=off): the output is the
// reference's Float32Array bit for bit. HBM-write bound (4 B per output sample).
#include "amodem_internal.h"

namespace amod {
namespace {

constexpr int TX_WG = 256;
constexpr int TX_NWAVE = TX_WG / 64;

// one radix-2 butterfly of fftIterative (modem.js:36-41), same operation order
__device__ __forceinline__ void bfly(double2 &a, double2 &b, const double2 w) {
  const double tr = w.x * b.x - w.y * b.y;
  const double ti = w.x * b.y + w.y * b.x;
  b.x = a.x - tr;
  b.y = a.y - ti;
  a.x = a.x + tr;
  a.y = a.y + ti;
}

// three consecutive radix-2 stages on the 8 elements a lane holds, element m at index
// base + stride*m: stage half h = stride << s pairs m and m + 2^s; the butterfly
// (i1, i1 + h) takes twiddle j = i1 mod 2h = (base mod stride) + stride * (m & (2^s - 1))
__device__ __forceinline__ void stages3(double2 (&v)[8], int rbase, int stride, const double2 *__restrict__ tw) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int hs = 1 << s, h = stride << s;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (m & hs) continue;
      const int j = rbase + stride * (m & (hs - 1));
      bfly(v[m], v[m + hs], tw[h - 1 + j]);
    }
  }
}

__device__ __forceinline__ int rev3(int m) { return ((m & 1) << 2) | (m & 2) | ((m >> 2) & 1); }
__device__ __forceinline__ int rev6(int g) {
  return ((g & 1) << 5) | ((g & 2) << 3) | ((g & 4) << 1) | ((g & 8) >> 1) | ((g & 16) >> 3) | ((g & 32) >> 5);
}

constexpr int TX_PKT_LDS = 8192; // packet bytes staged in LDS (longer packets read from global)

__global__ __launch_bounds__(TX_WG) void k_tx(const DevCfg cfg, const DevTxWork w) {
  __shared__ double2 xch[TX_NWAVE][kFft];
  __shared__ float wmaxv[TX_NWAVE];
  __shared__ uint32_t pk_s[TX_PKT_LDS / 4];
  __shared__ int16_t di_s[kMaxBand];
  const int f = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint8_t *const pkt = w.pkt + w.pkt_off[f];
  const int plen = w.pkt_len[f], pre = w.pre[f], post = w.post[f];
  float *const out = w.out + w.out_off[f];
  const int SYM = cfg.sym, CP = cfg.cp, rep = cfg.rep, bps = cfg.bps;
  const int per_sym = cfg.ndata * bps;
  const int64_t nbits = (int64_t)plen * 8 * rep;
  const int nsym = (int)((nbits + per_sym - 1) / per_sym);
  const int data0 = pre + 3 * SYM;
  const int64_t total = (int64_t)data0 + (int64_t)nsym * SYM + post;
  // silence before and after (Float32Array zeros; 0 * s stays +0)
  for (int i = tid; i < pre; i += TX_WG) out[i] = 0.f;
  for (int i = tid; i < post; i += TX_WG) out[total - post + i] = 0.f;
  // the packet and the band -> data-index table in LDS: the spectrum build reads them
  // per bit, so their latency must not be a global round trip each
  const bool pk_lds = plen <= TX_PKT_LDS;
  if (pk_lds)
    for (int i = tid; i < (plen + 3) / 4; i += TX_WG) {
      uint32_t v = 0;
      for (int b = 0; b < 4; ++b)
        if (4 * i + b < plen) v |= (uint32_t)pkt[4 * i + b] << (8 * b);
      pk_s[i] = v;
    }
  for (int b = tid; b < cfg.nband; b += TX_WG) di_s[b] = cfg.t.band_di[b];
  __syncthreads();
  const uint8_t *const pk8 = reinterpret_cast<const uint8_t *>(pk_s);

  const double2 *const tw = cfg.t.tw_inv;
  // spectrum value V(k), 1 <= k <= 255: pilot 1 + 0i, data point, 0 elsewhere
  auto value = [&](int s, int k) -> double2 {
    const int b = k - cfg.sub_start;
    if (b < 0 || k > cfg.sub_end) return make_double2(0.0, 0.0);
    const int di = di_s[b];
    if (di < 0) return make_double2(1.0, 0.0);
    int idx = 0;
    for (int q = 0; q < bps; ++q) {
      const int64_t p = (int64_t)s * per_sym + (int64_t)di * bps + q; // position in the repeated stream
      int bit = 0;
      if (p < nbits) {
        const int64_t o = p / rep; // original bit (repeatBits: each bit rep times in a row)
        bit = ((pk_lds ? pk8[o >> 3] : pkt[o >> 3]) >> (7 - (int)(o & 7))) & 1;
      }
      idx = (idx << 1) | bit;
    }
    return cfg.t.points[idx];
  };
  // X[k] after the Hermitian completion of modulateOFDM (modem.js:350-352)
  auto spec = [&](int s, int k) -> double2 {
    if (k == 0 || k == kFft / 2) return make_double2(0.0, 0.0);
    if (k < kFft / 2) return value(s, k);
    const double2 v = value(s, kFft - k);
    return make_double2(v.x, -v.y);
  };

  float lmax = 0.f;
  double2 *const X = xch[wave];
  // exchange layout: element e at e ^ ((e >> 3) & 7) ^ (bit 6 of e, at bit 3). The first
  // store (lane l writes elements 8 l .. 8 l + 7) put every lane of an 8-lane
  // ds_write_b128 group on the same four banks (8-way: 101 M conflict cycles per C2 batch
  // against 38 M LDS-active) and the pass-2 read (64 G + r + 8 m) was 2-way; with the
  // swizzle every ds_write_b128 group covers 8 distinct 16-byte slots and every
  // ds_read_b128 group 16 (all four exchange patterns conflict-free)
  auto sw = [](int e) { return e ^ ((e >> 3) & 7) ^ (((e >> 6) & 1) << 3); };
  for (int s = wave; s < nsym; s += TX_NWAVE) {
    double2 v[8];
    // bitReverse: a[8g + m] = X[rev9(8g + m)] = X[64 rev3(m) + rev6(g)], lane g
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = spec(s, 64 * rev3(m) + rev6(lane));
    stages3(v, 0, 1, tw); // halves 1, 2, 4 inside aligned groups of 8
#pragma unroll
    for (int m = 0; m < 8; ++m) X[sw(8 * lane + m)] = v[m];
    __builtin_amdgcn_wave_barrier();
    const int G = lane >> 3, r = lane & 7; // halves 8, 16, 32: index 64 G + r + 8 m
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = X[sw(64 * G + r + 8 * m)];
    stages3(v, r, 8, tw);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < 8; ++m) X[sw(64 * G + r + 8 * m)] = v[m];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = X[sw(lane + 64 * m)]; // halves 64, 128, 256: index t + 64 m
    stages3(v, lane, 64, tw);
    __builtin_amdgcn_wave_barrier();
    // ifft scale 1/n (exact) and the f32 store of addCP: out[CP + i] = td[i],
    // out[i - (n - CP)] = td[i] for the prefix
    float *const o = out + data0 + s * SYM;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int i = lane + 64 * m;
      const float x = (float)(v[m].x * (1.0 / kFft));
      o[CP + i] = x;
      if (i >= kFft - CP) o[i - (kFft - CP)] = x;
      lmax = fmaxf(lmax, fabsf(x));
    }
  }
  // frame max |signal| (templates: host-computed tmax)
  lmax = wave_max(lmax);
  if (lane == 0) wmaxv[wave] = lmax;
  __syncthreads();
  float fm = cfg.tx_tmax;
  for (int i = 0; i < TX_NWAVE; ++i) fm = fmaxf(fm, wmaxv[i]);
  if (fm > 0.f) {
    const double sc = 0.8 / (double)fm;
    // templates pre1, pre2, CE (modem.js:531-537), scaled
    for (int i = tid; i < 3 * SYM; i += TX_WG) out[pre + i] = (float)((double)cfg.t.tmpl[i] * sc);
    // data symbols: each lane rescales exactly the samples it stored above
    for (int s = wave; s < nsym; s += TX_NWAVE) {
      float *const o = out + data0 + s * SYM;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int i = lane + 64 * m;
        const float x = (float)((double)o[CP + i] * sc);
        o[CP + i] = x;
        if (i >= kFft - CP) o[i - (kFft - CP)] = x;
      }
    }
  } else {
    for (int i = tid; i < 3 * SYM; i += TX_WG) out[pre + i] = cfg.t.tmpl[i];
  }
}

} // namespace
} // namespace amod

extern "C" hipError_t amod_launch_tx(const amod::DevCfg &cfg, const amod::DevTxWork &w, hipStream_t s) {
  if (w.nframes <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::k_tx, dim3(w.nframes), dim3(amod::TX_WG), 0, s, cfg, w);
  return hipGetLastError();
}
