// k_decode_fast.hip — fast path of the OFDM receive chain (gfx950).
//
// Two launches per batch, each shaped for what it does (one HBM pass over the samples,
// then short compute jobs over the few samples the demodulator needs):
//
//   k_detect   one 256-thread workgroup per frame (decodeReceivedSignal frames only):
//              stage 0  stream pass   preprocessSignal (modem.js:213-232) statistics and,
//                                     in the same pass, 32-sample block moments of
//                                     u = x - x[0] (sum u, sum u^2, sum u[k] u[k+256]);
//                                     normalised Schmidl-Cox block sums follow exactly
//                                     from them once mean and peak are known
//              stage 1  Schmidl-Cox   detectPreamble (286-319): window sums at block
//                                     starts, rigorous per-block caps, candidate blocks
//                                     slid position by position (32-lane prefix scans)
//              stage 2  fine timing   inline xcorr (567-588) over the plateau +- 3 CP,
//                                     VALU + DPP, folded on pre1's 256-sample period
//              -> per-frame detection record (start, normalisation, symbols to decode)
//   k_chunk_prep  the same record for decodeChunkFrame windows (modem.js:770-786)
//   k_demod    persistent waves, one frame at a time per wave: CE + data symbols as FFT
//              jobs (two real symbols per complex 512-pt FFT, radix-8 x 3, swizzled LDS
//              exchanges), estimateChannel (421-440), equalise + pilot phase + demap
//              (demodulateOFDM 365-418) into the frame's bit stream in LDS, then
//              majorityVote / bitsToBytes / parse / CRC-32 and the stores; the next
//              job's samples are in flight while the current one computes
//
// Arithmetic is fp32. Every discrete decision carries a guard band sized from an
// error bound; a frame with a decision inside its band is listed
// for k_decode_exact (IEEE double, reference operation order).
#include "amodem_internal.h"
// cache policy of the stream pass's sample loads (experiments: 2 = nt)
#ifndef AMOD_STREAM_CPOL
#define AMOD_STREAM_CPOL 0
#endif

#include <algorithm>
#include <type_traits>

namespace amod {
namespace {

constexpr int WG = 256;                      // 4 waves
constexpr int NWAVE = WG / 64;
constexpr int BLK = 32;                      // Schmidl-Cox block length
constexpr float ACTIVE_EB = 0.05f;           // normalised 32-sample block energy of "signal" (rms ~0.04 of peak)
constexpr int SC_MAXCAND = 256;              // candidate blocks slid per position (else exact)
constexpr int SC_CACHE = 16;                 // candidate blocks whose per-position results stay in LDS
#ifndef AMOD_FIRST_SYMS
#define AMOD_FIRST_SYMS 7
#endif
constexpr int FIRST_SYMS = AMOD_FIRST_SYMS;  // data symbols always decoded (the header's)
#ifndef AMOD_SB
#define AMOD_SB 8
#endif
constexpr int SB = AMOD_SB;                  // stream pass: chunks per load batch
#ifndef AMOD_WPE
#define AMOD_WPE 7                           // waves per SIMD the register budget is sized for (72 VGPRs;
                                             // C2's LDS fits 7 workgroups per CU: 0.277 -> 0.273 ms)
#endif
#ifndef AMOD_SCAN_WPE
#define AMOD_SCAN_WPE 5                      // k_corr_scan (the scan phase alone)
#endif
// Diagnostics only (tools/ko_variants.sh): k_demod knockout builds. With AMOD_KO defined,
// no frame is listed for the exact kernel and every job of every frame runs (the time of
// the same work); bit 1 skips the frame-end CRC, 2 the demap and bit-stream packing, 4 the
// pilot reductions, 8 the window checks, 16 the FFT, 128 only the FFT's LDS exchanges
// (arithmetic kept), 0x200 the whole frame end (vote, parse, CRC, stores), 0x400 the
// header evaluation after each job. The results are
// wrong; only the kernel time matters (0x100 alone: the policy change only, the
// baseline of the others). Undefined in every product build.
#ifdef AMOD_KO
#define KO(b) ((AMOD_KO) & (b))
#else
#define KO(b) 0
#endif
// k_demod's per-frame phase marks (AMOD_STAMPS, tools/demod_profile.py) exist only in a
// diagnostic build (-DAMOD_DEMOD_STAMPS, tools/build_variants.sh): compiled in, their
// pointer and address arithmetic held SGPRs the job loop then spilled to VGPR lanes
#ifdef AMOD_DEMOD_STAMPS
constexpr bool kDemodStamps = true;
#else
constexpr bool kDemodStamps = false;
#endif
#ifndef AMOD_DEMOD_WPE
#define AMOD_DEMOD_WPE 4                     // k_demod: 104 registers, no VGPR spills; LDS (FFT exchange
                                             // rows, twiddles, bit streams) allows 4 workgroups per CU on C2 anyway
#endif

// Dynamic LDS of k_detect, sized per launch (amod_fast_lds_bytes): one region reused
// by the stages, addressed by float / float2 / word index.
//   stages 0-1: s1[nbc] s2[nbc] sx[nbc] (block moments -> caps / E_b / Z_b), cand[256] (int16),
//               cmax[256], pass-1 cache[SC_CACHE][32] (float2: top metric, uncertainty bits)
//   stage 2   : tmpl[T] m[FC + 8] yw[FC + Y] q[FC + 280] (folded window) E[FC + Y] (prefix of
//               squares of yw); FC = the launch's fine-search capacity, T = SYM rounded to 8,
//               Y = max(SYM + 24, 528): the staged span P + SYM + 16 and the fold's reads to
//               qn + 256 (sized from the preset's symbol length: C2's workgroup fits 7 per CU)
extern __shared__ __attribute__((aligned(16))) unsigned char amod_dyn[];
#define LDS_F (reinterpret_cast<float *>(amod_dyn))
#define LDS_F2 (reinterpret_cast<float2 *>(amod_dyn))
#define LDS_U (reinterpret_cast<uint32_t *>(amod_dyn))
#define LDS_I16 (reinterpret_cast<int16_t *>(amod_dyn))
__host__ __device__ constexpr int fine_t(int sym) { return (sym + 7) & ~7; }
__host__ __device__ constexpr int fine_y(int sym) { return ((sym + 24 > 528 ? sym + 24 : 528) + 7) & ~7; }
__host__ __device__ constexpr int fine_m(int, int sym) { return fine_t(sym); }
__host__ __device__ constexpr int fine_yw(int fc, int sym) { return fine_t(sym) + fc + 8; }
__host__ __device__ constexpr int fine_q(int fc, int sym) { return fine_yw(fc, sym) + fc + fine_y(sym); }
__host__ __device__ constexpr int fine_e(int fc, int sym) { return fine_q(fc, sym) + fc + 280; }
__host__ __device__ constexpr int fine_floats(int fc, int sym) { return fine_e(fc, sym) + fc + fine_y(sym); }
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
// the LDS byte address of a pointer into __shared__ memory (the low half of its flat
// address is the offset in the workgroup's LDS)
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }

struct Smem {  // fixed part (static LDS)
  float rf[4 * NWAVE];
  int ri[4 * NWAVE];
  double rd[2 * NWAVE];
  uint32_t ru[16];
  // per-frame scalars (written by one thread, read after a barrier)
  int status, flags, coarse, clo, chi, start, ncand, last_blk;
  float A, B, Bu, errw, cbest, cblo, cbhi, fbest;
  double mean, mx;
};

__device__ __forceinline__ float2 operator+(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 operator-(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// packed-pair forms the demodulator needs (one v_pk_* each, halves picked by op_sel)
// (a.x + b.x, a.y - b.y)
__device__ __forceinline__ f2v pk_add_conj(f2v a, f2v b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// (a.y + b.y, b.x - a.x)
__device__ __forceinline__ f2v pk_add_swap_neg(f2v a, f2v b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// phase derotation (e.x + ph e.y, e.y - ph e.x), ph wave-uniform
__device__ __forceinline__ f2v pk_derot(f2v e, f2v ph) {
  f2v r;
  asm("v_pk_fma_f32 %0, %1, %2, %1 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[1,0,0]" : "=v"(r) : "v"(e), "s"(ph));
  return r;
}
// (a.x b.x - a.y b.y, a.x b.y + a.y b.x)
__device__ __forceinline__ f2v pk_cmul(f2v a, f2v b) {
  f2v t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
// QPSK (Gray, modem.js:107-150) decision as its two stream bits at bits 31, 30:
// [im < 0], [re < 0] xor [im < 0] from the sign bits (a +-0 component lies on a decision
// boundary, where the margin test lists the frame for the exact kernel anyway)
__device__ __forceinline__ uint32_t qpsk_bits(float cr, float ci) {
  const uint32_t a = __float_as_uint(cr), b = __float_as_uint(ci);
  return (b & 0x80000000u) | (((a ^ b) >> 31) << 30);
}
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}

// Radix-8 step on packed pairs (f2v = (re, im) in an aligned register pair): every
// complex add and every multiply by -i or W8 is one v_pk_* with its halves picked by
// op_sel / negated by neg_lo / neg_hi, so no operand is moved between registers. 8-point
// DFT in natural order, v[q] <- sum_m v[m] W8^{mq}: two 4-point DFTs (W4 = -i) after the
// first butterfly, W8 = (1 - i) / sqrt 2 and W8^3 applied as (x + y, y - x) r.
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ f2v pk_add_mi(f2v a, f2v b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ f2v pk_sub_mi(f2v a, f2v b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// (b.x + b.y, b.y - b.x): W8 b / r
__device__ __forceinline__ f2v pk_w8u(f2v b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(b));
  return r;
}
// (b.y - b.x, -b.x - b.y): W8^3 b / r
__device__ __forceinline__ f2v pk_w83u(f2v b) {
  f2v r;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(r) : "v"(b));
  return r;
}
__device__ __forceinline__ void pk_dft4(f2v &a0, f2v &a1, f2v &a2, f2v &a3) {
  const f2v s02 = a0 + a2, d02 = a0 - a2, s13 = a1 + a3, d13 = a1 - a3;
  a0 = s02 + s13;
  a2 = s02 - s13;
  a1 = pk_add_mi(d02, d13);
  a3 = pk_sub_mi(d02, d13);
}
__device__ __forceinline__ void pk_dft8(f2v (&v)[8]) {
  const f2v r = {0.70710678118654752f, 0.70710678118654752f};
  f2v a0 = v[0] + v[4], a1 = v[1] + v[5], a2 = v[2] + v[6], a3 = v[3] + v[7];
  f2v b0 = v[0] - v[4], b1 = v[1] - v[5], b2 = v[2] - v[6], b3 = v[3] - v[7];
  b1 = pk_w8u(b1) * r;
  b3 = pk_w83u(b3) * r;
  pk_dft4(a0, a1, a2, a3);
  // dft4 of (b0, -i b2 folded into the adds, b1, b3)
  const f2v s02 = pk_add_mi(b0, b2), d02 = pk_sub_mi(b0, b2), s13 = b1 + b3, d13 = b1 - b3;
  v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
  v[1] = s02 + s13;
  v[5] = s02 - s13;
  v[3] = pk_add_mi(d02, d13);
  v[7] = pk_sub_mi(d02, d13);
}

// Per-wave exchange buffer of the 512-pt FFT (float2 units): exchanges 1 and 2 use 8 rows
// of XROW = 72 (row q at 72 q), exchange 2 columns at 9 p1 + l1; the spectrum is left at
// spec_idx(n). Every access of a pass is a per-lane base plus an immediate offset (no
// per-access address arithmetic), and the row pad makes each pattern conflict-free:
// ds_read_b64 serves lanes in two groups of 32 with banks (a / 4) mod 64, ds_write_b64 in
// four groups of 16 with banks (a / 4) mod 32 (MI355X_MICROARCH.md, LDS), and
// 72 q2 + l1 resp. 72 q2 + 9 p1 (q2 < 4 inside a group) are distinct mod 32.
constexpr int XROW = 72;
constexpr int XCH_F2 = 8 * XROW; // float2 per wave
// spec_idx: bits 4-5 of n XOR-ed into bits 1-2. The pass-3 store of lane (p1, q2) writes
// n = q2 + 8 p1 (+ 64 p2): in each 16-lane ds_write_b64 group (q2 in {2g, 2g + 1}) the
// float2 slots mod 16 are then (q2 ^ 2 (p1 >> 1)) + 8 (p1 & 1), all distinct (the
// round-2 swizzle, bit 5 into bit 2, left them 2-way); the band reads (consecutive n)
// stay 2-way only in groups that straddle a 16-bin boundary
__device__ __forceinline__ int spec_idx(int n) { return n ^ (((n >> 4) & 3) << 1); }

// One wave: 512-pt complex FFT of z (lane l holds z[l + 64 m] in v[m]); X[n] is
// left in the wave's exchange buffer X2 at spec_idx(n).
// tw1: rows 1-7 of e^{-2 pi i l q / 512} (row q at tw1[64 q]); tw2: [8][8] pass-2 twiddles
__device__ void fft512_wave(f2v (&v)[8], float2 *const X2f, const float2 *__restrict__ tw1f,
                            const float2 *__restrict__ tw2f) {
  f2v *const X2 = reinterpret_cast<f2v *>(X2f);
  const f2v *const tw1 = reinterpret_cast<const f2v *>(tw1f), *const tw2 = reinterpret_cast<const f2v *>(tw2f);
  int l = wave_lane();
  asm volatile("" : "+v"(l)); // keep lane-derived bases inside the job loop
  const int l1 = l & 7, q2 = l >> 3;
  // each pass's twiddles are requested before its butterflies, so their LDS latency hides
  // under the arithmetic (the compiler reads them after it, one exposed wait per read pair);
  // the wait is explicit, with the twiddle registers as its operands
  f4v t01, t23, t45;
  f2v t6;
  {
    const uint32_t a = lds_addr(tw1 + 64 + l); // rows 1 .. 7, 512 B apart
    asm volatile("ds_read2st64_b64 %0, %1 offset0:0 offset1:1" : "=v"(t01) : "v"(a));
    asm volatile("ds_read2st64_b64 %0, %1 offset0:2 offset1:3" : "=v"(t23) : "v"(a));
    asm volatile("ds_read2st64_b64 %0, %1 offset0:4 offset1:5" : "=v"(t45) : "v"(a));
    asm volatile("ds_read_b64 %0, %1 offset:3072" : "=v"(t6) : "v"(a));
  }
  pk_dft8(v);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t01), "+v"(t23), "+v"(t45), "+v"(t6));
  v[1] = pk_cmul(v[1], t01.xy); v[2] = pk_cmul(v[2], t01.zw);
  v[3] = pk_cmul(v[3], t23.xy); v[4] = pk_cmul(v[4], t23.zw);
  v[5] = pk_cmul(v[5], t45.xy); v[6] = pk_cmul(v[6], t45.zw);
  v[7] = pk_cmul(v[7], t6);
  // exchange 1: Y1[q][l] at row q, column l
  f2v *const w1 = X2 + l;
#ifdef AMOD_KO
  if ((AMOD_KO) & 128) { // (diagnostics: the FFT's arithmetic without its LDS exchanges)
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(v[q]));
      pk_dft8(v);
#pragma unroll
      for (int q = 1; q < 8; ++q) v[q] = pk_cmul(v[q], tw1[q * 64 + l]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) asm volatile("" ::"v"(v[q]));
    return;
  }
#endif
#pragma unroll
  for (int q = 0; q < 8; ++q) w1[q * XROW] = v[q];
  __builtin_amdgcn_wave_barrier();
  // pass 2, lane (l1, q2): the 64-pt DFT of row q2 over l = l1 + 8 l2, radix-8 over l2
  f2v *const r1 = X2 + q2 * XROW + l1;
#pragma unroll
  for (int l2 = 0; l2 < 8; ++l2) v[l2] = r1[8 * l2];
  {
    const uint32_t a = lds_addr(tw2 + l1); // p1 = 1 .. 7, 64 B apart
    asm volatile("ds_read2_b64 %0, %1 offset0:8 offset1:16" : "=v"(t01) : "v"(a));
    asm volatile("ds_read2_b64 %0, %1 offset0:24 offset1:32" : "=v"(t23) : "v"(a));
    asm volatile("ds_read2_b64 %0, %1 offset0:40 offset1:48" : "=v"(t45) : "v"(a));
    asm volatile("ds_read_b64 %0, %1 offset:448" : "=v"(t6) : "v"(a));
  }
  // (the row's samples above are compiler-issued reads: pk_dft8 waits for them itself; the
  // twiddle reads behind them are only waited for below)
  pk_dft8(v);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t01), "+v"(t23), "+v"(t45), "+v"(t6));
  v[1] = pk_cmul(v[1], t01.xy); v[2] = pk_cmul(v[2], t01.zw);
  v[3] = pk_cmul(v[3], t23.xy); v[4] = pk_cmul(v[4], t23.zw);
  v[5] = pk_cmul(v[5], t45.xy); v[6] = pk_cmul(v[6], t45.zw);
  v[7] = pk_cmul(v[7], t6);
  __builtin_amdgcn_wave_barrier();
  // exchange 2: U[p1] of lane (l1, q2) at row q2, column 9 p1 + l1 (same base as r1)
#pragma unroll
  for (int p1 = 0; p1 < 8; ++p1) r1[9 * p1] = v[p1];
  __builtin_amdgcn_wave_barrier();
  const int p1 = l & 7; // pass-3 lane = (p1, q2), same row as pass 2
  const f2v *const r2 = X2 + q2 * XROW + 9 * p1;
#pragma unroll
  for (int a = 0; a < 8; ++a) v[a] = r2[a];
  pk_dft8(v); // v[p2] = X[q2 + 8 p1 + 64 p2]
  __builtin_amdgcn_wave_barrier();
  f2v *const w3 = X2 + spec_idx(q2 + 8 * p1); // spec_idx(n + 64 p2) = spec_idx(n) + 64 p2
#pragma unroll
  for (int p2 = 0; p2 < 8; ++p2) w3[64 * p2] = v[p2];
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ float2 spec_read(const float2 *X2, int n) { return X2[spec_idx(n & 511)]; }

// Symbol rows (one word-aligned row of wsym words per data symbol, MSB-first) ->
// the frame's contiguous MSB-first bit stream (bitsToBytes order, modem.js:468-476):
// word W takes bits [32 W, 32 W + 32) across as many rows as it spans. Bits past
// nsym rows are zero. Row storage needs one readable word past the last row.
__device__ void repack_rows(const uint32_t *rows, int wsym, int per_sym, int nsym, uint32_t *out) {
  const int nw = (nsym * per_sym + 31) >> 5;
  for (int W = ltid(); W < nw; W += WG) {
    const int g = 32 * W;
    int s = g / per_sym, l = g - s * per_sym;
    uint32_t acc = 0;
    int got = 0;
    while (got < 32 && s < nsym) {
      const int n = min(32 - got, per_sym - l);
      const uint32_t *rw = rows + s * wsym + (l >> 5);
      const int o = l & 31;
      uint32_t x = o ? (rw[0] << o) | (rw[1] >> (32 - o)) : rw[0];
      x &= n >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> n);
      acc |= x >> got;
      got += n;
      ++s;
      l = 0;
    }
    out[W] = acc;
  }
}
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

// v_rcp_f32 / v_sqrt_f32 / v_rsq_f32 without the IEEE scaling and fix-up sequences
// (<= 1 ulp). Used only for bounds and metrics whose guards carry a relative slack of
// >= 1e-4 (caps, brackets) or an absolute one of >= 1e-3 (metric guards).
__device__ __forceinline__ float rcp_a(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sqrt_a(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float rsq_a(float x) { return __builtin_amdgcn_rsqf(x); }

// min/max of three without the NaN canonicalisation fminf/fmaxf add (a NaN sample
// is caught through the sum instead)
__device__ __forceinline__ float min3_raw(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Whole-wave reductions to a wave-uniform value: DPP butterflies inside each row of
// 16 lanes (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror),
// then the four rows combined through readlane. No LDS round trips. Whole wave active.
#define AMOD_DPP_I(v, ctrl) __builtin_amdgcn_update_dpp(0, (v), (ctrl), 0xF, 0xF, true)
#define AMOD_DPP_F(v, ctrl) __int_as_float(AMOD_DPP_I(__float_as_int(v), (ctrl)))
__device__ __forceinline__ float rlane(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float wsum(float v) {
  v += AMOD_DPP_F(v, 0xB1); v += AMOD_DPP_F(v, 0x4E); v += AMOD_DPP_F(v, 0x141); v += AMOD_DPP_F(v, 0x140);
  return (rlane(v, 0) + rlane(v, 16)) + (rlane(v, 32) + rlane(v, 48));
}
__device__ __forceinline__ float wmax(float v) {
  v = fmaxf(v, AMOD_DPP_F(v, 0xB1)); v = fmaxf(v, AMOD_DPP_F(v, 0x4E));
  v = fmaxf(v, AMOD_DPP_F(v, 0x141)); v = fmaxf(v, AMOD_DPP_F(v, 0x140));
  return fmaxf(fmaxf(rlane(v, 0), rlane(v, 16)), fmaxf(rlane(v, 32), rlane(v, 48)));
}
__device__ __forceinline__ int wmin_i(int v) {
  v = min(v, AMOD_DPP_I(v, 0xB1)); v = min(v, AMOD_DPP_I(v, 0x4E));
  v = min(v, AMOD_DPP_I(v, 0x141)); v = min(v, AMOD_DPP_I(v, 0x140));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int wmax_i(int v) {
  v = max(v, AMOD_DPP_I(v, 0xB1)); v = max(v, AMOD_DPP_I(v, 0x4E));
  v = max(v, AMOD_DPP_I(v, 0x141)); v = max(v, AMOD_DPP_I(v, 0x140));
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ int wor_i(int v) {
  v |= AMOD_DPP_I(v, 0xB1); v |= AMOD_DPP_I(v, 0x4E); v |= AMOD_DPP_I(v, 0x141); v |= AMOD_DPP_I(v, 0x140);
  return (__builtin_amdgcn_readlane(v, 0) | __builtin_amdgcn_readlane(v, 16)) |
         (__builtin_amdgcn_readlane(v, 32) | __builtin_amdgcn_readlane(v, 48));
}

// Whole-wave sum / max to a wave-uniform value with one readlane: row reductions by DPP,
// then row_bcast:15 (rows 1, 3 take rows 0, 2) and row_bcast:31 (rows 2, 3 take lane 31),
// so lane 63 holds the total. Whole wave active.
__device__ __forceinline__ float wsum_b(float v) {
  v += AMOD_DPP_F(v, 0xB1); v += AMOD_DPP_F(v, 0x4E); v += AMOD_DPP_F(v, 0x141); v += AMOD_DPP_F(v, 0x140);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return rlane(v, 63);
}
// four wsum_b reductions interleaved step by step: a DPP read of a value the previous VALU
// instruction wrote needs two wait states, which the three other chains fill (one chain
// alone pays an s_nop per step)
__device__ __forceinline__ void wsum_b4(float &a, float &b, float &c, float &d) {
  asm volatile("s_nop 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)); // (see AMOD_DPP_GUARD)
#define AMOD_W4(ctrl)                                                                   \
  { const float ta = AMOD_DPP_F(a, ctrl), tb = AMOD_DPP_F(b, ctrl), tc = AMOD_DPP_F(c, ctrl), td = AMOD_DPP_F(d, ctrl); \
    a += ta; b += tb; c += tc; d += td; }
  AMOD_W4(0xB1) AMOD_W4(0x4E) AMOD_W4(0x141) AMOD_W4(0x140)
#undef AMOD_W4
  // the two row broadcasts as DPP adds into the value itself: the rows a broadcast does
  // not enable keep their sums (the builtin form moved a zero and the broadcast into a
  // scratch register first, then added: three VALU per step instead of one). The s_nop
  // covers the DPP read of a value the compiler's last VALU may have just written;
  // inside the block each chain's previous write is three instructions back
  asm volatile("s_nop 1\n"
               "v_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
               "v_add_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
               "v_add_f32_dpp %2, %2, %2 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
               "v_add_f32_dpp %3, %3, %3 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
               "v_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
               "v_add_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
               "v_add_f32_dpp %2, %2, %2 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
               "v_add_f32_dpp %3, %3, %3 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
               "s_nop 1" // (the readlanes below: a VALU write of a VGPR needs a wait state before
                         // v_readlane reads it, which the compiler cannot see inside the block)
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  a = rlane(a, 63); b = rlane(b, 63); c = rlane(c, 63); d = rlane(d, 63);
}
// the same four sums over row 0 only (lanes 0 .. 15; the pilot lanes of every built-in
// preset): the row reductions alone, then lane 0
__device__ __forceinline__ void wsum16_4(float &a, float &b, float &c, float &d) {
  asm volatile("s_nop 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  // row 1 of a (b) takes row 0 of c (d) (v_permlane16_swap: odd rows of the first operand
  // with even rows of the second), so one row-local butterfly sums a and c (b and d) at
  // once: the same lanes in the same order as four separate sums over row 0
  float ac = __uint_as_float(__builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(c), false, false)[0]);
  float bd = __uint_as_float(__builtin_amdgcn_permlane16_swap(__float_as_uint(b), __float_as_uint(d), false, false)[0]);
#define AMOD_W2(ctrl)                                                                   \
  { const float t0 = AMOD_DPP_F(ac, ctrl), t1 = AMOD_DPP_F(bd, ctrl); ac += t0; bd += t1; }
  AMOD_W2(0xB1) AMOD_W2(0x4E) AMOD_W2(0x141) AMOD_W2(0x140)
#undef AMOD_W2
  a = rlane(ac, 0); c = rlane(ac, 16); b = rlane(bd, 0); d = rlane(bd, 16);
}
__device__ __forceinline__ float wmax_b(float v) {
  v = fmaxf(v, AMOD_DPP_F(v, 0xB1)); v = fmaxf(v, AMOD_DPP_F(v, 0x4E));
  v = fmaxf(v, AMOD_DPP_F(v, 0x141)); v = fmaxf(v, AMOD_DPP_F(v, 0x140));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x142, 0xA, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x143, 0xC, 0xF, false)));
  return rlane(v, 63);
}

// max over the wave of non-negative floats (or NaN): their bit patterns order like the
// values, so the reduction runs on integers (v_max_i32 with DPP fused, no NaN
// canonicalisation steps); a wave-uniform result via one readlane. Whole wave active.
// (inputs of the DPP reductions below may come from inline asm, e.g. max3_raw: the
// compiler's hazard check does not count an asm block as the VALU write a DPP read must
// wait two states for, so each reduction starts with its own s_nop tied to the value)
#define AMOD_DPP_GUARD(x) asm volatile("s_nop 1" : "+v"(x))
__device__ __forceinline__ float wmax_nn(float x) {
  AMOD_DPP_GUARD(x);
  int v = __float_as_int(x);
  v = max(v, AMOD_DPP_I(v, 0xB1)); v = max(v, AMOD_DPP_I(v, 0x4E));
  v = max(v, AMOD_DPP_I(v, 0x141)); v = max(v, AMOD_DPP_I(v, 0x140));
  // the row broadcasts as DPP maxima into v itself (see wsum_b4)
  asm volatile("s_nop 1\n"
               "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
               "s_nop 1\n"
               "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
               "s_nop 1" // (before the readlane: see wsum_b4)
               : "+v"(v));
  return __int_as_float(__builtin_amdgcn_readlane(v, 63));
}

// inclusive prefix sum inside each aligned 32-lane group: row_shr 1/2/4/8 inside rows of
// 16, then row_bcast:15 carries row 0 (2) into row 1 (3). The group's lanes all active.
__device__ __forceinline__ float scan32(float v) {
  v += AMOD_DPP_F(v, 0x111); v += AMOD_DPP_F(v, 0x112); v += AMOD_DPP_F(v, 0x114); v += AMOD_DPP_F(v, 0x118);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  return v;
}

// inclusive prefix sum over the whole wave: scan32, then row_bcast:31 carries lane 31
// into rows 2 and 3. Whole wave active.
__device__ __forceinline__ float scan64(float v) {
  v = scan32(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return v;
}

// sum over each aligned group of 8 lanes, result in every lane of the group (DPP:
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror). Whole wave active.
// three dpp_sum8 interleaved (each DPP read of a fresh VALU result needs wait states)
__device__ __forceinline__ void dpp_sum8x3(float &a, float &b, float &c) {
  a += AMOD_DPP_F(a, 0xB1); b += AMOD_DPP_F(b, 0xB1); c += AMOD_DPP_F(c, 0xB1);
  a += AMOD_DPP_F(a, 0x4E); b += AMOD_DPP_F(b, 0x4E); c += AMOD_DPP_F(c, 0x4E);
  a += AMOD_DPP_F(a, 0x141); b += AMOD_DPP_F(b, 0x141); c += AMOD_DPP_F(c, 0x141);
}
__device__ __forceinline__ float dpp_sum8(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, true));
  return v;
}

// Why a frame skips the fast path (0: it does not). Depends on the frame, the options and
// the launch's fast-path length only (never on other frames of the batch).
__device__ __forceinline__ int frame_route(const DevCfg &cfg, const DevWork &w, int N) {
  if (w.options & AMOD_OPT_FORCE_EXACT) return AMOD_FLAG_FORCED;
  if ((int64_t)N > w.fast_len) return AMOD_FLAG_BIG; // longer than the launch's fast-path workspace
  return 0;
}

// append frame f to k_decode_exact's list (one thread); [sc_lo, sc_hi]: the positions
// that can hold detectPreamble's argmax when the coarse stage proved that (else -1)
__device__ __forceinline__ void list_exact(const DevWork &w, int f, int flags, int sc_lo = -1, int sc_hi = -1) {
  const int i = atomicAdd(w.fb_count, 1);
  w.fb_list[i] = f;
  w.fb_flags[i] = flags;
  if (w.det) {
    w.det[f].sc_lo = sc_lo;
    w.det[f].sc_hi = sc_hi;
    w.det[f].route = ROUTE_EXACT;
  }
}

// scalar (SMEM) load of a wave-uniform record: waits on lgkmcnt, not behind vector loads
template <typename T> __device__ __forceinline__ T sload(const T *p) {
  static_assert(sizeof(T) % 4 == 0, "whole dwords");
  typedef const __attribute__((address_space(4))) uint32_t *cptr;
  const cptr q = reinterpret_cast<cptr>(reinterpret_cast<uintptr_t>(p));
  uint32_t v[sizeof(T) / 4];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) v[i] = q[i];
  T out;
  __builtin_memcpy(&out, v, sizeof(T));
  return out;
}

// chunk q of the frame in k-space (k = i + ph; 64 float4 = 256 samples); lanes
// past the frame's last float4 read nothing, the last float4 reads only its
// in-frame samples (no access past the frame)
__device__ __forceinline__ float4 ld_chunk(const float *base, int q, int lane, int nvec, int K) {
  const int v = 64 * q + lane;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (v < nvec - 1 || (v == nvec - 1 && (K & 3) == 0)) {
    t = reinterpret_cast<const float4 *>(base)[v];
  } else if (v == nvec - 1) {
    const int r = K & 3;
    t.x = base[4 * v];
    if (r > 1) t.y = base[4 * v + 1];
    if (r > 2) t.z = base[4 * v + 2];
  }
  return t;
}

// Kernel arguments re-read through a fresh (opaque) kernarg-segment pointer at each
// stage: the loads become scalar loads next to their uses instead of ~100 SGPRs of
// configuration held (and spilled) across the whole kernel.
struct KArgs {
  DevCfg cfg;
  DevWork w;
};
__device__ __forceinline__ const KArgs &kargs() {
  auto p = (__attribute__((address_space(4))) const KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const KArgs *)p;
}
#define FRESH_ARGS                                                                      \
  const DevCfg &cfg = kargs().cfg;                                                      \
  const DevWork &w = kargs().w;                                                         \
  (void)cfg;                                                                            \
  (void)w

// diagnostics only (AMOD_STAMPS): wave 0's shader-clock timeline of a frame
#define STAMP(k)                                                                        \
  do {                                                                                  \
    if (w.stamps && tid == 0) w.stamps[(int64_t)f * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// SCAN_ONLY: the same code stopped after the Schmidl-Cox decision (k_corr_scan, the
// correlation-scan phase measured on its own; nothing is written).
// DBG: parity-test build that also records intermediates (amod_decode_device_debug);
template <bool SCAN_ONLY, bool DBG> __device__ __forceinline__ void detect() {
  __shared__ Smem sm;
  FRESH_ARGS;
  const int nbc = w.nb_cap; // dynamic LDS capacity of this launch
  const int f = w.f0 + (int)blockIdx.x; // frames [f0, f1) of this launch
  const int tid = ltid(), lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6); // wave-uniform (SGPR)
  // frame geometry in SGPRs: every branch and loop bound below is wave-uniform
  const int64_t off_l = w.off[f];
  const int64_t off = ((int64_t)__builtin_amdgcn_readfirstlane((int)(off_l >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off_l);
  const int N = __builtin_amdgcn_readfirstlane(w.len[f]);
  const int ph = (int)(off & 3);
  const int K = ph + N;                      // k-space end (exclusive)
  const float *const X = w.samples + off;    // frame sample i at X[i]
  const int SYM = cfg.sym, CP = cfg.cp;
  constexpr bool dbg = DBG;
  amod_debug *D = dbg ? w.dbg + f : nullptr;
  STAMP(0);
  {
    const int route = frame_route(cfg, w, N);
    if (route) {
      if (tid == 0) list_exact(w, f, route);
      return;
    }
  }
  int start = 0;
  const float eps_c = 2e-3f * cfg.guard; // Schmidl-Cox metric guard (absolute)
  const float eps_g = 1e-3f * cfg.guard; // energy-gate guard (relative)
  const float eps_f = 1e-3f * cfg.guard; // fine metric guard (absolute)
  if (tid == 0) {
    sm.status = AMOD_OK; sm.flags = 0; sm.coarse = -1; sm.clo = -1; sm.chi = -1; sm.start = 0;
    sm.fbest = 0.f; sm.A = 1.f; sm.B = 0.f; sm.mean = 0.0; sm.mx = 0.0;
    // detectPreamble never runs its loop below 512 samples: coarse index -1 whatever
    // the samples hold (modem.js:288-319, 564)
    if (cfg.mode == AMOD_MODE_RECEIVED && N < 512) sm.status = AMOD_E_PREAMBLE;
  }
  __syncthreads();
  if (sm.status != AMOD_OK) goto finish_error;

  {
    // ------------------------------------------------ stage 0: stream pass
    const int nch = (K + 255) >> 8;
    const int NB = (K + BLK - 1) / BLK;
    const int bz_edge = max(0, (K - 256) >> 5); // blocks >= this have pairs past the frame end
    // Samples of the blocks whose pairs leave the frame (and of block 0 when the frame
    // starts mid-float4), summed directly below: requested now, so their latency hides
    // under the stream pass. Edge slot e: block 0 (e = 0) or bz_edge + e - 1; there are
    // at most NB - bz_edge <= 9 such blocks, so two rounds of 8 32-lane groups cover them.
    float ex0[2], ex1[2];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int e = 2 * wave + (lane >> 5) + 2 * NWAVE * it;
      const int b = e == 0 ? 0 : bz_edge + e - 1;
      const int i = BLK * b + (lane & 31) - ph;
      const bool use = b < NB && !(e == 0 && (ph == 0 || bz_edge == 0)) && i >= 0 && i + 256 < N;
      ex0[it] = use ? X[i] : 0.f;
      ex1[it] = use ? X[i + 256] : 0.f;
    }
    {
      FRESH_ARGS;
      // Vector pass over the float4s wholly inside the frame's k-range (k < kfull);
      // the <= 3 samples of a trailing partial float4 are added by thread 0 below.
      // A lane past the last full float4 reloads it (masked below), so no load sits
      // under a branch.
      // frame as a raw buffer over its whole float4s: lanes past the end read zeros
      const int nfull = K >> 2, kfull = 4 * nfull;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void *)(X - ph), (short)0, 16 * nfull, 0x00020000);
      const float c0 = X[0];
      // the <= 3 samples of a trailing partial float4, requested now (lanes 0-2) so that
      // thread 0's tail step below does not wait for memory after the pass
      float tailv = 0.f;
      {
        const int k = kfull + (lane & 3);
        if (lane < 3 && k < K && k >= ph) tailv = X[k - ph];
      }
      const int q0 = (wave * nch) / NWAVE, q1 = ((wave + 1) * nch) / NWAVE;
      float sacc = 0.f;
      float mn = INFINITY, mxv = -INFINITY;
      auto LD = [&](int q) -> float4 {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 1024 * q, AMOD_STREAM_CPOL);
        return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
      };
      // per-sample work on packed pairs (v_pk_add/mul/fma_f32): u = x - x[0] of a chunk is
      // computed once, when the chunk is its predecessor's partner, and carried in
      // registers to its own step
      const f2v c0v = {c0, c0};
      auto u_of = [&](const float4 v, f2v &lo, f2v &hi) {
        lo = f2v{v.x, v.y} - c0v;
        hi = f2v{v.z, v.w} - c0v;
      };
      // chunk q (raw a, u in u01/u23) with its partner chunk q + 1 (raw nb -> n01/n23);
      // block moments stored through pb[0..2] (block 8 q + lane / 8 of each array)
      auto step = [&](int q, const float4 a, f2v u01, f2v u23, const float4 nb, f2v &n01, f2v &n23,
                      float *const pb0, float *const pb1, float *const pb2) {
        const int kq = 256 * q;
        u_of(nb, n01, n23);
        if (kq >= ph && kq + 256 <= kfull) { // whole chunk inside the frame (wave-uniform)
          mn = min3_raw(mn, min3_raw(a.x, a.y, a.z), a.w);
          mxv = max3_raw(mxv, max3_raw(a.x, a.y, a.z), a.w);
        } else {
          const int k0 = kq + 4 * lane;
          const float av[4] = {a.x, a.y, a.z, a.w};
          float ua[4] = {u01.x, u01.y, u23.x, u23.y};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (k0 + j >= ph && k0 + j < kfull) { mn = fminf(mn, av[j]); mxv = fmaxf(mxv, av[j]); }
            else ua[j] = 0.f;
          }
          u01 = f2v{ua[0], ua[1]};
          u23 = f2v{ua[2], ua[3]};
        }
        const f2v p1 = u01 + u23;
        const f2v p2 = __builtin_elementwise_fma(u23, u23, u01 * u01);
        const f2v px = __builtin_elementwise_fma(u23, n23, u01 * n01);
        float s1 = p1.x + p1.y, s2 = p2.x + p2.y, sx = px.x + px.y;
        dpp_sum8x3(s1, s2, sx);
        sacc += s1; // every lane of a group holds its block's sum: lane 0 of the group counts it
        if ((lane & 7) == 0) { *pb0 = s1; *pb1 = s2; *pb2 = sx; }
      };
      // a ring of R chunk registers kept full: chunk q is stepped with its partner q + 1
      // (next slot), then its slot is refilled with chunk q + R, so about R - 1 loads per
      // wave stay in flight through the whole pass (no drain between batches). The
      // wave's last chunk q1 - 1 takes chunk q1 as partner; refills past q1 re-read
      // chunk q1 (a cache hit): every load is unconditional, so the in-order vmcnt
      // accounting stays exact and each step waits only for its own two chunks.
      constexpr int R = SB + 1;
      float4 c[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        c[j] = LD(min(q0 + j, q1));
        __builtin_amdgcn_sched_barrier(0);
      }
      f2v cu01, cu23; // u of the chunk stepped next
      u_of(c[0], cu01, cu23);
      for (int qb = q0; qb < q1; qb += R) {
        // one moment address per array and ring turn; the steps use immediate offsets
        float *const pb = LDS_F + 8 * qb + (lane >> 3);
        float *const pb1 = pb + nbc, *const pb2 = pb1 + nbc;
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const int q = qb + j;
          if (q < q1) step(q, c[j], cu01, cu23, c[(j + 1) % R], cu01, cu23, pb + 8 * j, pb1 + 8 * j, pb2 + 8 * j);
          c[j] = LD(min(q + R, q1));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      double sacc_d = (lane & 7) == 0 ? (double)sacc : 0.0;
      sacc_d = wave_sum(sacc_d);
      mn = -wmax(-mn);
      mxv = wmax(mxv);
      const float tail0 = rlane(tailv, 0), tail1 = rlane(tailv, 1), tail2 = rlane(tailv, 2);
      if (lane == 0) { sm.rd[wave] = sacc_d; sm.rf[wave] = mn; sm.rf[NWAVE + wave] = mxv; }
      __syncthreads();
      if (tid == 0) {
        double S = 0.0;
        float MN = INFINITY, MX = -INFINITY;
        for (int i = 0; i < NWAVE; ++i) { S += sm.rd[i]; MN = fminf(MN, sm.rf[i]); MX = fmaxf(MX, sm.rf[NWAVE + i]); }
        for (int k = max(kfull, ph); k < K; ++k) { // trailing partial float4
          const float x = k == kfull ? tail0 : (k == kfull + 1 ? tail1 : tail2), u = x - c0;
          S += (double)u; MN = fminf(MN, x); MX = fmaxf(MX, x);
          LDS_F[k >> 5] += u;
          LDS_F[nbc + (k >> 5)] = fmaf(u, u, LDS_F[nbc + (k >> 5)]);
        }
        int flags = 0;
        float A = 1.f, B = 0.f, Bu = 0.f;
        double mean = 0.0, mx = 0.0;
        if (!isfinite(S) || !isfinite(MN) || !isfinite(MX)) {
          flags = AMOD_FLAG_NONFINITE; // NaN/Inf anywhere reaches the mean: exact path
        } else if (N > 0) {
          mean = (double)c0 + S / (double)N;
          // max |f32(x - mean)| is reached at the extremes: rounding to f32 is monotone
          mx = fmax(fabs((double)(float)((double)MX - mean)), fabs((double)(float)((double)MN - mean)));
          if (fabs(mx - 1e-6) <= 1e-6 * 1e-4) flags |= AMOD_FLAG_THRESH; // mean from fp32 block sums
          if (mx > 1e-6) { A = (float)(1.0 / mx); B = (float)(-mean / mx); Bu = (float)(((double)c0 - mean) / mx); }
          else { A = 1.f; B = (float)(-mean); Bu = (float)((double)c0 - mean); }
        }
        sm.flags = flags; sm.A = A; sm.B = B; sm.Bu = Bu; sm.mean = mean; sm.mx = mx; sm.last_blk = -1;
        if (dbg) { D->mean = mean; D->mx = mx; }
      }
      __syncthreads();
    }
    if (sm.flags) goto to_exact;
    // moments -> normalised block sums: y = A u + Bu, so over a block
    //   E_b = A^2 S2 + 2 A Bu S1 + n Bu^2,   Z_b = A^2 Sx + A Bu (S1_b + S1_{b+8}) + 32 Bu^2
    {
      FRESH_ARGS;
      const float A = sm.A, Bu = sm.Bu, AA = A * A, AB = A * Bu, BB = Bu * Bu, aAB = fabsf(AB);
      float tmax = 0.f;
      for (int b = tid; b < NB; b += WG) { // Z first: it reads s1/s2 of block b + 8
        const float s2b = fmaxf(LDS_F[nbc + b], 0.f);
        if (b < bz_edge && (b > 0 || ph == 0)) {
          const float s1b = LDS_F[b], s1p = LDS_F[b + 8], s2p = fmaxf(LDS_F[nbc + b + 8], 0.f);
          LDS_F[2 * nbc + b] = fmaf(AA, LDS_F[2 * nbc + b], fmaf(AB, s1b + s1p, 32.f * BB));
          tmax = fmaxf(tmax, AA * sqrt_a(s2b * s2p) + aAB * (sqrt_a(32.f * s2b) + sqrt_a(32.f * s2p)) + 32.f * BB);
        }
      }
      __syncthreads();
      int last = -1; // last block with signal energy (sizes the first FFT round only)
      for (int b = tid; b < NB; b += WG) {
        const float s1b = LDS_F[b], s2b = fmaxf(LDS_F[nbc + b], 0.f);
        const int nv = min(BLK * b + BLK, K) - max(BLK * b, ph);
        const float eb = fmaf(AA, s2b, fmaf(2.f * AB, s1b, (float)nv * BB));
        LDS_F[nbc + b] = eb;
        if (eb > ACTIVE_EB) last = b;
        tmax = fmaxf(tmax, AA * s2b + 2.f * aAB * sqrt_a(32.f * s2b) + 32.f * BB);
      }
      last = wmax_i(last);
      if (lane == 0 && last >= 0) atomicMax(&sm.last_blk, last);
      // blocks whose pairs leave the frame (and block 0 when the frame starts mid-float4):
      // summed directly from the samples, one 32-lane group per block
      const float Af = sm.A, Bf = sm.B;
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int e = 2 * wave + (lane >> 5) + 2 * NWAVE * it;
        const int b = e == 0 ? 0 : bz_edge + e - 1;
        if (b >= NB || (e == 0 && (ph == 0 || bz_edge == 0))) continue; // uniform per 32-lane group
        const int i = BLK * b + (lane & 31) - ph;
        float z = 0.f;
        if (i >= 0 && i + 256 < N) z = fmaf(ex0[it], Af, Bf) * fmaf(ex1[it], Af, Bf);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) z += __shfl_xor(z, o, 32);
        if ((lane & 31) == 0) LDS_F[2 * nbc + b] = z;
      }
      tmax = wmax(tmax);
      if (lane == 0) sm.rf[wave] = tmax;
      __syncthreads();
      if (tid == 0) {
        float T = 0.f;
        for (int i = 0; i < NWAVE; ++i) T = fmaxf(T, sm.rf[i]);
        // a block sum carries <= ~13 roundings of terms bounded by T; a window adds 8 blocks
        sm.errw = 8.f * 16.f * 5.9604645e-8f * (1.0001f * T) + 1e-30f;
      }
      __syncthreads();
    }
    STAMP(1);
    if (cfg.stop_after == 0) return;

    // ---------------------------------------------- stage 1: Schmidl-Cox scan
    {
      FRESH_ARGS;
      const int E = N - 512;
      if (E < 0) {
        if (tid == 0) sm.status = AMOD_E_PREAMBLE;
        __syncthreads();
        goto finish_error;
      }
      const float errw = sm.errw;
      const float A = sm.A, B = sm.B;
      const float gate_lo = 0.01f * (1.f - eps_g) - errw, gate_hi = 0.01f * (1.f + eps_g) + errw;
      const float *const Eb = LDS_F + nbc, *const Zb = LDS_F + 2 * nbc;
      const int CMAX = 3 * nbc + SC_MAXCAND / 2;   // per-candidate max metric (after cand[])
      const int PCACHE = CMAX + SC_MAXCAND;        // pass-1 results of the first SC_CACHE blocks
      float *const cap = LDS_F;
      const int ncb = (E + ph) / BLK + 1; // blocks holding at least one position d in [0, E]
      // (a) window sums at block starts: a rigorous lower bound Lb on the best metric,
      //     and every block's cap (upper bound of the metric over its 32 positions)
      float lmax = -1.f;
      for (int c = tid; c < ncb; c += WG) {
        float p = 0.f, ra = 0.f, rb = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) { p += Zb[c + q]; ra += Eb[c + q]; rb += Eb[c + 8 + q]; }
        if (BLK * c - ph >= 0 && ra - errw > gate_hi && rb - errw > gate_hi) {
          const float pl = fmaxf(fabsf(p) - errw, 0.f);
          lmax = fmaxf(lmax, (pl * pl) * rcp_a((ra + errw) * (rb + errw)) * 0.9999f);
        }
        const float e0 = fmaxf(Eb[c], 0.f) + errw, e8 = fmaxf(Eb[c + 8], 0.f) + errw;
        const float e16 = (c + 16 < NB ? fmaxf(Eb[c + 16], 0.f) : 0.f) + errw;
        const float ra_lo = ra - e0 - errw, rb_lo = rb - e8 - errw;
        float cv;
        if (!(ra + e8 + errw > gate_lo && rb + e16 + errw > gate_lo)) cv = -2.f; // gated out throughout
        else if (ra_lo > 0.f && rb_lo > 0.f) {
          // |p(d) - p_c| <= sum|z| over blocks c and c+8 <= sqrt(E_c E_c+8) + sqrt(E_c+8 E_c+16)
          const float pm = fabsf(p) + errw + sqrt_a(e0 * e8) + sqrt_a(e8 * e16);
          cv = (pm * pm) * rcp_a(ra_lo * rb_lo) * 1.0001f;
        } else cv = INFINITY;
        cap[c] = cv;
      }
      lmax = wmax(lmax);
      if (tid == 0) sm.ncand = 0;
      if (lane == 0) sm.rf[wave] = lmax;
      __syncthreads();
      STAMP(2);
      if (cfg.stop_after == 10) return;
      float Lb = -1.f;
      for (int i = 0; i < NWAVE; ++i) Lb = fmaxf(Lb, sm.rf[i]);
      // (b) blocks whose cap reaches Lb - eps_c
      //     compacted per wave with a ballot: one LDS atomic per wave and 64 blocks
      for (int c0 = 64 * wave; c0 < ncb; c0 += WG) {
        const int c = c0 + lane;
        const bool pred = c < ncb && cap[c] >= Lb - eps_c;
        const uint64_t mask = __ballot(pred);
        if (mask) {
          int base = 0;
          if (lane == 0) base = atomicAdd(&sm.ncand, (int)__popcll(mask));
          base = __shfl(base, 0);
          const int slot = base + (int)__popcll(mask & ((1ull << lane) - 1ull));
          if (pred && slot < SC_MAXCAND) LDS_I16[6 * nbc + slot] = (int16_t)c;
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
      // (c) every position of a candidate block: one 32-lane group per block; window
      // sums at d0 + j are the block-start sums plus an exclusive prefix (across the
      // group) of the per-position slide increments. m_lo/m_hi bracket the metric
      // given the block-sum error errw.
      // raw samples of candidate block cidx at d, d + 256, d + 512 (0 outside the frame)
      auto cand_load = [&](int cidx, float (&xr)[3]) {
        const int d = BLK * (int)LDS_I16[6 * nbc + cidx] - ph + (lane & 31);
#pragma unroll
        for (int t = 0; t < 3; ++t) xr[t] = (d + 256 * t >= 0 && d + 256 * t < N) ? X[d + 256 * t] : 0.f;
      };
      auto cand_eval = [&](int cidx, const float (&xr)[3], float &m, float &mlo, float &mhi, int &d, float &ra,
                           float &rb) -> bool {
        const int j = lane & 31;
        const int c = LDS_I16[6 * nbc + cidx];
        float p = 0.f;
        ra = 0.f; rb = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) { p += Zb[c + q]; ra += Eb[c + q]; rb += Eb[c + 8 + q]; }
        d = BLK * c - ph + j;
        const float y0 = (d >= 0 && d < N) ? fmaf(xr[0], A, B) : 0.f;
        const float y1 = (d + 256 >= 0 && d + 256 < N) ? fmaf(xr[1], A, B) : 0.f;
        const float y2 = (d + 512 >= 0 && d + 512 < N) ? fmaf(xr[2], A, B) : 0.f;
        const float z0 = (d >= 0 && d < N - 256) ? y0 * y1 : 0.f;
        const float z1 = (d + 256 >= 0 && d + 256 < N - 256) ? y1 * y2 : 0.f;
        const float vp = z1 - z0, va = fmaf(y1, y1, -y0 * y0), vb = fmaf(y2, y2, -y1 * y1);
        // exclusive prefix (inclusive scan minus own term) over the 32-lane group
        p += scan32(vp) - vp; ra += scan32(va) - va; rb += scan32(vb) - vb;
        const bool ok = d >= 0 && d <= E && ra > gate_lo && rb > gate_lo;
        m = ok ? (p * p) * rcp_a(ra * rb) : -1.f;
        const float pl = fmaxf(fabsf(p) - errw, 0.f), ph2 = fabsf(p) + errw;
        mlo = ok ? (pl * pl) * rcp_a((ra + errw) * (rb + errw)) * 0.9999f : -1.f;
        mhi = ok ? ((ra > errw && rb > errw) ? (ph2 * ph2) * rcp_a((ra - errw) * (rb - errw)) * 1.0001f : INFINITY) : -1.f;
        return ok;
      };
      float best = -1.f, blo = -1.f, bhi = -1.f;
      int bidx = 0x7fffffff;
      // the samples of a group's first two blocks (16 per workgroup: the usual plateau
      // neighbourhood) are requested together, one memory latency for both
      const int g0 = 2 * wave + (lane >> 5);
      float xq[2][3];
#pragma unroll
      for (int it = 0; it < 2; ++it)
        if (g0 + 2 * NWAVE * it < ncand) cand_load(g0 + 2 * NWAVE * it, xq[it]);
      for (int g = g0, it = 0; g - (lane >> 5) < ncand; g += 2 * NWAVE, ++it) {
        if (g < ncand) {
          float m, mlo, mhi, ra, rb;
          int d;
          float xr[3];
          if (it < 2) {
#pragma unroll
            for (int t = 0; t < 3; ++t) xr[t] = it == 0 ? xq[0][t] : xq[1][t];
          } else {
            cand_load(g, xr);
          }
          const bool ok = cand_eval(g, xr, m, mlo, mhi, d, ra, rb);
          if (ok) {
            if (m > best || (m == best && d < bidx)) { best = m; bidx = d; }
            blo = fmaxf(blo, mlo);
            bhi = fmaxf(bhi, mhi);
          }
          // pass 2 reads the first SC_CACHE blocks' positions from LDS instead of memory
          if (g < SC_CACHE) {
            const int u = (ra <= gate_hi || rb <= gate_hi) | (((mhi - mlo) > eps_c) << 1);
            LDS_F[PCACHE + 2 * (32 * g + (lane & 31))] = ok ? fmaxf(m, mhi) : -INFINITY;
            LDS_U[PCACHE + 2 * (32 * g + (lane & 31)) + 1] = (uint32_t)u;
          }
          // the block's highest possible metric, for pass 2's filter
          float top = ok ? fmaxf(m, mhi) : -2.f;
          top = fmaxf(top, AMOD_DPP_F(top, 0xB1)); top = fmaxf(top, AMOD_DPP_F(top, 0x4E));
          top = fmaxf(top, AMOD_DPP_F(top, 0x141)); top = fmaxf(top, AMOD_DPP_F(top, 0x140));
          top = fmaxf(top, __shfl_xor(top, 16, 32));
          if ((lane & 31) == 0) LDS_F[CMAX + g] = top;
        } // a group's 32 lanes share g, so its DPP/shuffles stay inside active lanes
      }
      {
        const float bw = wmax(best);
        const int iw = wmin_i(best == bw ? bidx : 0x7fffffff);
        const float lw = wmax(blo), hw = wmax(bhi);
        if (lane == 0) { sm.rf[wave] = bw; sm.ri[wave] = iw; sm.rf[NWAVE + wave] = lw; sm.rf[2 * NWAVE + wave] = hw; }
        __syncthreads();
        if (tid == 0) {
          float B2 = -1.f, L2 = -1.f, H2 = -1.f;
          int I2 = 0x7fffffff;
          for (int i = 0; i < NWAVE; ++i) {
            if (sm.rf[i] > B2 || (sm.rf[i] == B2 && sm.ri[i] < I2)) { B2 = sm.rf[i]; I2 = sm.ri[i]; }
            L2 = fmaxf(L2, sm.rf[NWAVE + i]);
            H2 = fmaxf(H2, sm.rf[2 * NWAVE + i]);
          }
          sm.cbest = B2; sm.coarse = I2; sm.cblo = L2; sm.cbhi = H2;
        }
        __syncthreads();
      }
      STAMP(4);
      if (cfg.stop_after == 12) return;
      const float CB = sm.cbest, CBL = sm.cblo, CBH = sm.cbhi;
      // positions that may hold the reference's argmax: metric possibly within eps_c of the best
      int lo = 0x7fffffff, hi = -1, unc = 0;
      if (CBH >= 0.5f - eps_c) {
        for (int g = 2 * wave + (lane >> 5); g - (lane >> 5) < ncand; g += 2 * NWAVE) {
          if (g < ncand && LDS_F[CMAX + g] >= CBL - eps_c) { // blocks that can reach the band
            float v;
            int d, u;
            if (g < SC_CACHE) {
              v = LDS_F[PCACHE + 2 * (32 * g + (lane & 31))];
              u = (int)LDS_U[PCACHE + 2 * (32 * g + (lane & 31)) + 1];
              d = BLK * (int)LDS_I16[6 * nbc + g] - ph + (lane & 31);
            } else {
              float m, mlo, mhi, ra, rb, xr[3];
              cand_load(g, xr);
              const bool ok = cand_eval(g, xr, m, mlo, mhi, d, ra, rb);
              v = ok ? fmaxf(m, mhi) : -INFINITY;
              u = (ra <= gate_hi || rb <= gate_hi) | (((mhi - mlo) > eps_c) << 1);
            }
            if (v >= CBL - eps_c) {
              lo = min(lo, d); hi = max(hi, d);
              unc |= u != 0; // near the energy gate, or a metric interval wider than the guard
            }
          }
        }
      }
      lo = wmin_i(lo); hi = wmax_i(hi); unc = wor_i(unc);
      if (lane == 0) { sm.ri[wave] = lo; sm.ri[NWAVE + wave] = hi; sm.ri[2 * NWAVE + wave] = unc; }
      __syncthreads();
      if (tid == 0) {
        int LO = 0x7fffffff, HI = -1, U = 0;
        for (int i = 0; i < NWAVE; ++i) { LO = min(LO, sm.ri[i]); HI = max(HI, sm.ri[NWAVE + i]); U |= sm.ri[2 * NWAVE + i]; }
        int flags = sm.flags;
        if (CBH < 0.5f - eps_c) sm.status = AMOD_E_PREAMBLE;          // confidently not detected
        else if (CBL <= 0.5f + eps_c || U) flags |= AMOD_FLAG_COARSE;  // threshold, gate or error ambiguous
        else if (HI - LO > 2 * 3 * CP) flags |= AMOD_FLAG_COARSE;      // no common fine window
        sm.flags = flags; sm.clo = LO; sm.chi = HI;
#ifdef AMOD_DIAG
        if (w.stamps) { // diagnostics build only: the coarse decision's inputs
          unsigned long long *st = w.stamps + (int64_t)f * 32 + 20;
          st[0] = __float_as_uint(CB); st[1] = __float_as_uint(CBL); st[2] = __float_as_uint(CBH);
          st[3] = (unsigned)U; st[4] = (unsigned)LO; st[5] = (unsigned)HI; st[6] = (unsigned)ncand;
          st[7] = __float_as_uint(sm.errw);
        }
#endif
        if (dbg) { D->coarse_metric = CB; D->coarse_lo = LO; D->coarse_hi = HI; }
      }
      __syncthreads();
    }
    if (sm.flags) goto to_exact;
    if (sm.status != AMOD_OK) goto finish_error;
    STAMP(5);
    if (SCAN_ONLY || cfg.stop_after == 1) return;

    // ---------------------------------------------- stage 2: fine timing
    {
      FRESH_ARGS;
      const int FC = w.fine_cap; // positions the launch's LDS holds (>= 12 CP + 1: every window the
                                 // coarse stage lets through)
      const int FM = fine_m(FC, SYM), FYW = fine_yw(FC, SYM), FQ = fine_q(FC, SYM), FE = fine_e(FC, SYM);
      const float A = sm.A, B = sm.B;
      const int R = 3 * CP;
      const int c_lo = sm.clo, c_hi = sm.chi;
      const int w0 = max(0, c_lo - R), w1 = min(N - SYM, c_hi + R);
      const int P = w1 - w0 + 1;
      if (P > FC) {
        if (tid == 0) sm.flags |= AMOD_FLAG_FINE;
        __syncthreads();
        goto to_exact;
      }
      if (P <= 0) {
        if (tid == 0) sm.status = AMOD_E_LOW_CORR;
        __syncthreads();
        goto finish_error;
      }
      // template + the normalised search window, staged once in LDS; a thread issues a
      // batch of loads before its first store (one memory latency per batch): raw buffer
      // loads past the frame end return 0 without a branch
      const int span = P + SYM + 16;
      {
        constexpr int TR = (768 + WG - 1) / WG, YB = 8;
        const __amdgpu_buffer_rsrc_t rx =
            __builtin_amdgcn_make_buffer_rsrc((void *)(X + w0), (short)0, 4 * (N - w0), 0x00020000);
        const __amdgpu_buffer_rsrc_t rt =
            __builtin_amdgcn_make_buffer_rsrc((void *)cfg.t.pre1, (short)0, 4 * SYM, 0x00020000);
        float tv[TR];
#pragma unroll
        for (int r = 0; r < TR; ++r)
          tv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rt, 4 * (tid + r * WG), 0, 0));
        for (int j0 = 0; j0 < span; j0 += YB * WG) {
          float yv[YB];
#pragma unroll
          for (int r = 0; r < YB; ++r)
            yv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, 4 * (j0 + tid + r * WG), 0, 0));
          if (j0 == 0) {
#pragma unroll
            for (int r = 0; r < TR; ++r)
              if (tid + r * WG < SYM) LDS_F[tid + r * WG] = tv[r];
          }
#pragma unroll
          for (int r = 0; r < YB; ++r) {
            const int j = j0 + tid + r * WG;
            if (j < span) LDS_F[FYW + j] = (w0 + j < N) ? fmaf(yv[r], A, B) : 0.f;
          }
        }
      }
      __syncthreads();
      const float te = cfg.te_f;
      const int noct = (P + 7) >> 3;
      const float *yw = LDS_F + FYW;
      const float *tm = LDS_F;
      const float *qw = LDS_F + FQ;
      const int fold = cfg.fold;
      if (fold) {
        // corr(d) = sum_{i<256} t[i] (y[d+i] + fold y[d+i+256]) + sum_{i<CP} t[i] y[d+i+512]
        // (t[i+256] = fold t[i]): 256 + CP taps instead of SYM
        const int qn = 8 * noct + 264;
        for (int j = tid; j < qn; j += WG) LDS_F[FQ + j] = fmaf((float)fold, yw[j + 256], yw[j]);
      }
      // window energies from a prefix of squares: E[j] = sum_{i<j} y[i]^2, en(d) = E[d+SYM] - E[d],
      // built 2048 entries at a time with a carried base. Each E[j] carries <= ~40 roundings of
      // partial sums <= E[span]: |err en| <= en_err.
      float en_err;
      {
        float carry = 0.f;
        for (int base = 0; base <= span; base += 8 * WG) {
          float sq[8], s = 0.f;
          const int b0 = base + 8 * tid;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float v = b0 + k < span ? yw[b0 + k] : 0.f;
            sq[k] = v * v;
            s += sq[k];
          }
          const float inc = scan64(s);
          if (lane == 63) sm.rf[wave] = inc;
          __syncthreads();
          float run = carry - s + inc, tot = 0.f;
          for (int i = 0; i < NWAVE; ++i) {
            const float wv = sm.rf[i];
            if (i < wave) run += wv;
            tot += wv;
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (b0 + k <= span) LDS_F[FE + b0 + k] = run;
            run += sq[k];
          }
          carry += tot;
          __syncthreads(); // sm.rf is reused by the next chunk
        }
        en_err = 6e-6f * carry + 1e-30f;
      }
      // metric of window position d from its correlation cj; energies from the prefix E
      auto fine_metric = [&](int d, float cj) {
        float en = LDS_F[FE + d + SYM] - LDS_F[FE + d];
        if (en < 1e4f * en_err) { // low-energy window: the difference is not accurate enough
          en = 0.f;
          for (int i = 0; i < SYM; ++i) en = fmaf(yw[d + i], yw[d + i], en);
        }
        // den = sqrt(en te) against the 0.001 gate, compared as squares; m = cj / den
        const float et = fmaxf(en, 0.f) * te;
        const float g_hi = 0.001f * (1.f + eps_g), g_lo = 0.001f * (1.f - eps_g);
        float m;
        if (et > g_hi * g_hi) m = cj * rsq_a(et);
        else if (et > g_lo * g_lo) m = cj * rsq_a(et) + 4.f; // uncertain gate: tagged
        else m = -8.f;                                      // gated out
        LDS_F[FM + d] = m;
      };
      // lane = (octet of 8 positions, one of 8 tap ranges): per tap one window read,
      // one template read, 8 correlations. The 8 ranges of an octet are 8 aligned
      // lanes, combined by DPP; energies come from the prefix E.
      for (int task = tid; task < noct * 8; task += WG) {
        const int oc = task >> 3, sp = task & 7;
        const int j0 = 8 * oc; // window offset of the octet's first position
        float c[8], yv[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) c[r] = 0.f;
        // correlation segments: (array, window offset, first tap, taps)
        auto corr = [&](const float *arr, int base, int i0, int n) {
#pragma unroll
          for (int r = 0; r < 7; ++r) yv[r] = arr[base + i0 + r];
#pragma unroll 8
          for (int i = i0; i < i0 + n; ++i) {
            yv[7] = arr[base + i + 7];
            const float t = tm[i];
#pragma unroll
            for (int r = 0; r < 8; ++r) c[r] = fmaf(yv[r], t, c[r]);
#pragma unroll
            for (int r = 0; r < 7; ++r) yv[r] = yv[r + 1];
          }
        };
        // tap range n split 8 ways with an odd length L (banks of the 8 splits differ)
        auto split = [&](int n, int &i0, int &cnt) {
          const int L = (n >> 3) | 1;
          i0 = sp * L;
          cnt = sp < 7 ? L : n - 7 * L;
        };
        int i0, cnt;
        if (fold) {
          split(256, i0, cnt);
          corr(qw, j0, i0, cnt);                    // folded body
          split(CP, i0, cnt);
          corr(yw, j0 + 512, i0, cnt);              // tail taps at offset 512
        } else {
          split(SYM, i0, cnt);
          corr(yw, j0, i0, cnt);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) c[r] = dpp_sum8(c[r]);
        if (j0 + sp < P) {
          // lane sp finishes position j0 + sp
          float cj = c[0];
#pragma unroll
          for (int r = 1; r < 8; ++r) cj = sp == r ? c[r] : cj;
          fine_metric(j0 + sp, cj);
        }
      }
      __syncthreads();
      // argmax (first index), second best and the best uncertain-gate candidate in one
      // pass: per lane its best (first index), the best of its other positions and its
      // best tagged metric; per wave the same with the second best taken over everything
      // but the wave's argmax; thread 0 combines the waves (the global argmax belongs to
      // exactly one wave, whose second best then stands in for its best)
      float b1 = -8.f, b2 = -8.f, mt = -INFINITY;
      int i1x = 0x7fffffff;
      for (int k = tid; k < P; k += WG) {
        float m = LDS_F[FM + k];
        const bool tagged = m > 2.f;
        if (tagged) { m -= 4.f; mt = fmaxf(mt, m); }
        if (m > b1) { b2 = b1; b1 = m; i1x = k; }
        else b2 = fmaxf(b2, m);
      }
      {
        const float bw = wmax(b1);
        const int iw = wmin_i(b1 == bw ? i1x : 0x7fffffff);
        const float sw = wmax(i1x == iw ? b2 : b1);
        const float tw = wmax(mt);
        if (lane == 0) {
          sm.rf[wave] = bw; sm.ri[wave] = iw; sm.rf[NWAVE + wave] = sw; sm.rf[2 * NWAVE + wave] = tw;
        }
      }
      __syncthreads();
      if (tid == 0) {
        float FB = -8.f;
        int kst = 0x7fffffff;
        for (int i = 0; i < NWAVE; ++i)
          if (sm.rf[i] > FB || (sm.rf[i] == FB && sm.ri[i] < kst)) { FB = sm.rf[i]; kst = sm.ri[i]; }
        float B2 = -8.f, MT = -INFINITY;
        for (int i = 0; i < NWAVE; ++i) {
          B2 = fmaxf(B2, sm.ri[i] == kst ? sm.rf[NWAVE + i] : sm.rf[i]);
          MT = fmaxf(MT, sm.rf[2 * NWAVE + i]);
        }
        const int U = MT >= FB - eps_f; // a tagged (uncertain-gate) metric near the best
        sm.fbest = FB;
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
  }

  // the detection record the demodulation launches read
  if (tid == 0) {
    const int data0 = start + 3 * SYM;
    const int M = (N - data0) / SYM; // whole data symbols (demodulateOFDM numSym)
    int T = M;
    // symbols up to the end of the frame's signal energy (the trailing silence is not
    // demodulated; k_finish sends a frame whose parse reads past them to the exact path)
    if (!dbg && sm.last_blk >= 0) {
      const int act_end = BLK * (sm.last_blk + 1) - ph; // first sample after the last active block
      const int tact = (act_end - data0 + SYM - 1) / SYM;
      T = min(M, max(min(M, FIRST_SYMS), tact));
    }
    T = min(T, w.mcap); // the k_demod bit stream's capacity (a parse past it: exact path)
    DetRec d;
    d.route = ROUTE_DEMOD; d.flags = 0; d.start = start; d.M = M; d.T = T; d.coarse = sm.coarse;
    d.A = sm.A; d.B = sm.B; d.fbest = sm.fbest; d.sc_lo = d.sc_hi = -1; d.pad = 0.f;
    w.det[f] = d;
    // opt-in soft combining (not reference behaviour): k_demod's soft instance, or the exact
    // kernel where that does not apply (a parity-debug launch)
    if (soft_combine_applies(w.options, cfg.rep, cfg.mod) && !soft_fast(w.options, cfg, w.dbg != nullptr))
      list_exact(w, f, AMOD_FLAG_SOFT);
  }
  return;

finish_error:
  if (tid == 0) {
    amod_result r;
    init_result(r);
    r.status = sm.status;
    r.coarse_idx = sm.status == AMOD_E_PREAMBLE ? -1 : sm.coarse;
    r.fine_metric = sm.status == AMOD_E_PREAMBLE ? 0.f : sm.fbest;
    r.preamble_idx = -1;
    w.res[f] = r;
    if (w.det) w.det[f].route = ROUTE_DONE;
  }
  return;

to_exact:
  // past the coarse stage, [clo, chi] holds every position whose metric can reach the
  // best (the others' upper bounds are below its lower bound): the exact replica's
  // recurrence stops at chi and compares metrics only there
  if (tid == 0) {
    const bool hull = sm.clo >= 0 && sm.chi >= sm.clo;
    list_exact(w, f, sm.flags, hull ? sm.clo : -1, hull ? sm.chi : -1);
  }
}

// ------------------------------------------------------------ detection kernels
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(AMOD_WPE))) void k_detect(const DevCfg cfg_arg, const DevWork w_arg) {
  (void)cfg_arg;
  tl_init(w_arg);
  detect<false, false>();
}
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(AMOD_WPE))) void k_detect_dbg(const DevCfg cfg_arg, const DevWork w_arg) {
  (void)cfg_arg;
  tl_init(w_arg);
  detect<false, true>();
}
// stream pass + Schmidl-Cox only (diagnostics: AMOD_STOP_AFTER=1); launched with the same
// dynamic LDS as k_detect, so the same number of workgroups share a CU
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(AMOD_SCAN_WPE))) void k_corr_scan(const DevCfg cfg_arg, const DevWork w_arg) {
  (void)cfg_arg;
  tl_init(w_arg);
  detect<true, false>();
}

// decodeChunkFrame (modem.js:770-786): no preprocessing, the frame starts at pre1;
// one thread per window writes its detection record (or its geometry error)
__global__ __launch_bounds__(WG) void k_chunk_prep(const DevCfg cfg, const DevWork w) {
  tl_init(w);
  const int f = w.f0 + (int)(blockIdx.x * WG + threadIdx.x);
  if (f >= w.f1) return;
  const int N = w.len[f], SYM = cfg.sym;
  const int route = frame_route(cfg, w, N);
  if (route) { list_exact(w, f, route); return; }
  if (3 * SYM >= N) {
    amod_result r;
    init_result(r);
    r.status = 3 * SYM > N ? AMOD_E_FRAME_SHORT_CE : AMOD_E_NO_DATA;
    w.res[f] = r;
    w.det[f].route = ROUTE_DONE;
    return;
  }
  DetRec d;
  d.route = ROUTE_DEMOD; d.flags = 0; d.start = 0; d.M = (N - 3 * SYM) / SYM; d.T = min(d.M, w.mcap); d.coarse = -1;
  d.A = 1.f; d.B = 0.f; d.fbest = 0.f; d.sc_lo = d.sc_hi = -1; d.pad = 0.f;
  w.det[f] = d;
  if (soft_combine_applies(w.options, cfg.rep, cfg.mod) && !soft_fast(w.options, cfg, w.dbg != nullptr))
    list_exact(w, f, AMOD_FLAG_SOFT);
}

// ------------------------------------------------------------ demodulation
// k_demod: persistent waves, one frame at a time per wave (frames last-first: the ones
// k_detect streamed last are the likeliest to still sit in the Infinity Cache), no
// workgroup barrier after the twiddle staging. A frame is a sequence of FFT jobs:
// job 0 = (CE, data symbol 0), job j = (2j-1, 2j); two real symbols share one complex
// 512-pt FFT (X1 = (Z[k] + conj Z[-k]) / 2, X2 = (Z[k] - conj Z[-k]) / 2i). Job 0's CE
// half gives the channel estimate (estimateChannel, modem.js:421-440) kept in registers
// as G = 1/H for the lane's band subcarriers; every data symbol is equalised, pilot-phase
// corrected and demapped (demodulateOFDM 365-418) with decision margins and its
// decisions OR-ed into the frame's MSB-first bit stream in the wave's LDS. The next
// job's samples (the next frame's first job at a frame's end) are in flight while the
// current one computes. At the frame's end the wave runs majorityVote, the parse, the
// CRC-32 and the stores (modem.js:468-495, 605-654, 805-849). A decision inside its
// guard band (or a parse that reads past the demodulated symbols) lists the frame for
// the exact kernel instead.

// Wave-level CRC-32 (modem.js:443-457) of bytes [0, L) of stream v. The message is cut
// into 16-byte chunks (wave_crc32: left-aligned, the last one zero-padded; wave_crc32_long:
// right-aligned, the first one zero-padded and started from t.crc_pre[pad], the register
// that the pad's zero bytes advance to the reference's initial ~0). Each chunk's register
// comes from slice-by-4 lookups in the workgroup's copy of the table in LDS (t4l: 4 KB,
// staged once at the kernel start; round 2 staged it per frame into the wave's exchange
// buffer: 2.6 K cycles of global loads per frame), is moved to the message end by the
// GF(2) matrix of its zero-byte shift and the images are XOR-combined (CRC linearity).
// Lane l takes chunks l, l + 64, ..., CRC_ILP of them interleaved, so the dependent
// lookups of different chunks overlap; the whole message is one pass (the frame-end CRC
// was a chain of global-memory lookups: 13.5k cycles per C2 frame, 24.7k per C4 window,
// tools/demod_profile.py).
// bytes i .. i + 3 of an MSB-first stream as one little-endian word (CRC byte order);
// bytes before the stream start (i >= -15) read as zero
__device__ __forceinline__ uint32_t le_word_pad(const uint32_t *v, int i) {
  const int wi = i >> 2, sh = 8 * (i & 3);
  const uint32_t lo = wi >= 0 ? v[max(wi, 0)] : 0u;
  const uint32_t hi = wi >= -1 ? v[max(wi + 1, 0)] : 0u;
  return __builtin_bswap32(sh ? (lo << sh) | (hi >> (32 - sh)) : lo);
}
// the same product with the matrix's 32 columns already in registers
__device__ __forceinline__ uint32_t crc_apply_rows(const uint4 (&m)[8], uint32_t c) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r ^= m[k].x & (uint32_t)((int32_t)(c << (31 - 4 * k)) >> 31);
    r ^= m[k].y & (uint32_t)((int32_t)(c << (30 - 4 * k)) >> 31);
    r ^= m[k].z & (uint32_t)((int32_t)(c << (29 - 4 * k)) >> 31);
    r ^= m[k].w & (uint32_t)((int32_t)(c << (28 - 4 * k)) >> 31);
  }
  return r;
}
__device__ __forceinline__ uint32_t crc_shift(const uint32_t *mat, int q, uint32_t c) {
  const uint4 *const mq = reinterpret_cast<const uint4 *>(mat + 32 * q);
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 m = mq[k];
    r ^= m.x & (uint32_t)((int32_t)(c << (31 - 4 * k)) >> 31);
    r ^= m.y & (uint32_t)((int32_t)(c << (30 - 4 * k)) >> 31);
    r ^= m.z & (uint32_t)((int32_t)(c << (29 - 4 * k)) >> 31);
    r ^= m.w & (uint32_t)((int32_t)(c << (28 - 4 * k)) >> 31);
  }
  return r;
}
// XOR over the wave to a wave-uniform value: DPP row reductions, then the two row
// broadcasts as DPP xors into v itself (the rows a broadcast does not enable keep theirs)
__device__ __forceinline__ uint32_t wave_xor_dpp(uint32_t x) {
  int v = (int)x;
  AMOD_DPP_GUARD(v);
  v ^= AMOD_DPP_I(v, 0xB1); v ^= AMOD_DPP_I(v, 0x4E); v ^= AMOD_DPP_I(v, 0x141); v ^= AMOD_DPP_I(v, 0x140);
  asm volatile("s_nop 1\n"
               "v_xor_b32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
               "s_nop 1\n"
               "v_xor_b32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
               "s_nop 1" // (before the readlane: see wsum_b4)
               : "+v"(v));
  return (uint32_t)__builtin_amdgcn_readlane(v, 63);
}
// chunks are LEFT-aligned (chunk j = bytes [16 j, 16 j + 16), the last one zero-padded to a
// whole chunk), read as one ds_read_b128 each. Lane l hashes the CONTIGUOUS chunks
// [n l, n l + n) (n = ceil(nch / 64)) in sequence, the register carried from chunk to chunk,
// so each lane moves its register to the message end once, by the GF(2) zero-shift matrix
// of the chunks after its range (round 4 gave lane l the chunks l, l + 64, ... and shifted
// each: three matrix products per lane on C4, each behind eight global reads of its
// matrix; the frame-end CRC was 15.7 k of a frame's 201 k wave cycles there). Chunk 0 starts
// from the reference's ~0; the register of the padded message is moved back over the pad's
// zero bytes at the end by crc_unpad[pad] (the inverse zero-byte operator, the workgroup's
// LDS copy of t.crc_unpad).
__device__ __forceinline__ uint32_t wave_crc32(const uint32_t *v, int L, const DevTables &t, const uint32_t *t4l,
                                               const uint32_t *crc_unpad, unsigned long long *stp = nullptr) {
  const int lane = wave_lane();
  if (stp && lane == 0) stp[30] = __builtin_amdgcn_s_memtime(); // (diagnostics: table staged)
  const uint32_t *const t4 = t4l;
  const int nch = (L + kCrcChunk - 1) / kCrcChunk;
  const int pad = kCrcChunk * nch - L;
  const int n = (nch + 63) >> 6; // chunks per lane (wave-uniform)
  const int j0 = n * lane, j1 = min(j0 + n, nch);
  // this lane's shift matrix (global memory) requested before the chunk steps, so its
  // reads fly under them
  uint4 sm[8];
  {
    const uint4 *const mq = reinterpret_cast<const uint4 *>(t.crc_mat + 32 * max(0, nch - j1));
#pragma unroll
    for (int k = 0; k < 8; ++k) sm[k] = mq[k];
  }
  uint32_t c = lane == 0 ? 0xFFFFFFFFu : 0u;
  for (int q = 0; q < n; ++q) { // (wave-uniform trip count; a lane past its range idles)
    const int j = j0 + q;
    if (j < nch) {
      uint4 wd = reinterpret_cast<const uint4 *>(v)[j];
      if (j == nch - 1 && pad) { // bytes past L read as zero (MSB-first words)
        const int nv = kCrcChunk - pad; // valid bytes of this chunk, 1 .. 15
        const auto keep = [&](int st) -> uint32_t {
          const int b = nv - 4 * st;
          return b >= 4 ? 0xFFFFFFFFu : b <= 0 ? 0u : ~(0xFFFFFFFFu >> (8 * b));
        };
        wd.x &= keep(0); wd.y &= keep(1); wd.z &= keep(2); wd.w &= keep(3);
      }
#pragma unroll
      for (int st = 0; st < kCrcChunk / 4; ++st) {
        const uint32_t wv = st == 0 ? wd.x : st == 1 ? wd.y : st == 2 ? wd.z : wd.w;
        const uint32_t x = c ^ __builtin_bswap32(wv);
        c = t4[768 + (x & 0xFF)] ^ t4[512 + ((x >> 8) & 0xFF)] ^ t4[256 + ((x >> 16) & 0xFF)] ^ t4[x >> 24];
      }
    }
  }
  if (stp && lane == 0) stp[31] = __builtin_amdgcn_s_memtime(); // (chunk registers)
  const uint32_t acc = j0 < nch ? crc_apply_rows(sm, c) : 0u;
  const uint32_t reg = wave_xor_dpp(acc);
  return (pad ? crc_shift(crc_unpad, pad, reg) : reg) ^ 0xFFFFFFFFu;
}

// the same over messages longer than kCrcMats chunks (8 KB): kCrcMats-chunk blocks in
// sequence, each block's first chunk carrying the register of the blocks before it
__device__ __forceinline__ uint32_t wave_crc32_long(const uint32_t *v, int L, const DevTables &t) {
  const int lane = wave_lane();
  const uint32_t *t4 = t.crc_s4;
  constexpr int BLOCKB = kCrcMats * kCrcChunk; // bytes per block
  uint32_t reg = 0xFFFFFFFFu; // carried between blocks (uniform)
  for (int p0 = 0; p0 < L; p0 += BLOCKB) {
    const int plen = min(BLOCKB, L - p0);
    const int nch = (plen + kCrcChunk - 1) / kCrcChunk; // chunks, right-aligned
    uint32_t acc = 0;
    for (int j = lane; j < nch; j += 64) {
      const int end = plen - (nch - 1 - j) * kCrcChunk; // exclusive, relative to p0
      const int beg = max(0, end - kCrcChunk);
      uint32_t c = j == 0 ? reg : 0u;
      int i = p0 + beg;
      for (; i + 4 <= p0 + end; i += 4) {
        c ^= le_word_pad(v, i);
        c = t4[768 + (c & 0xFF)] ^ t4[512 + ((c >> 8) & 0xFF)] ^ t4[256 + ((c >> 16) & 0xFF)] ^ t4[c >> 24];
      }
      for (; i < p0 + end; ++i) c = t4[(c ^ stream_byte(v, i)) & 0xFF] ^ (c >> 8);
      acc ^= crc_shift(t.crc_mat, nch - 1 - j, c);
    }
    reg = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_xor(acc));
  }
  return reg ^ 0xFFFFFFFFu;
}

// Majority vote (modem.js:487-495) of the first nbits of `bits` into `voted`, one wave:
// voted word wd is the vote over raw words [REP wd, REP wd + REP), which each lane reads
// once; the bit extraction is unrolled (REP known at compile time), no per-bit LDS reads.
// Bits of the last word past the voted count are zero.
template <int REP> __device__ __forceinline__ void wave_vote_t(const uint32_t *bits, int nbits, uint32_t *voted) {
  const int nv = nbits / REP;
  const int nw = (nv + 31) >> 5;
  constexpr int thr = (REP + 1) >> 1; // sum >= rep/2  <=>  sum >= ceil(rep/2)
  for (int wd = wave_lane(); wd < nw; wd += 64) {
    uint32_t raw[REP];
#pragma unroll
    for (int u = 0; u < REP; ++u) raw[u] = bits[REP * wd + u];
    uint32_t word = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      int sum = 0;
#pragma unroll
      for (int u = 0; u < REP; ++u) {
        const int pos = b * REP + u;
        sum += (raw[pos >> 5] >> (31 - (pos & 31))) & 1;
      }
      word |= (uint32_t)(sum >= thr) << (31 - b);
    }
    const int valid = nv - 32 * wd;
    if (valid < 32) word &= ~(0xFFFFFFFFu >> valid);
    voted[wd] = word;
  }
}
__device__ __forceinline__ void wave_vote(const uint32_t *bits, int nbits, int rep, uint32_t *voted) {
  switch (rep) {
  case 2: wave_vote_t<2>(bits, nbits, voted); return;
  case 3: wave_vote_t<3>(bits, nbits, voted); return;
  case 4: wave_vote_t<4>(bits, nbits, voted); return;
  case 5: wave_vote_t<5>(bits, nbits, voted); return;
  default: break;
  }
  const int nv = nbits / rep;
  const int nw = (nv + 31) >> 5;
  const int thr = (rep + 1) >> 1;
  for (int wd = wave_lane(); wd < nw; wd += 64) {
    uint32_t word = 0;
    for (int b = 0; b < 32; ++b) {
      const int j = wd * 32 + b;
      if (j >= nv) break;
      int sum = 0;
      for (int u = 0; u < rep; ++u) {
        const int pos = j * rep + u;
        sum += (bits[pos >> 5] >> (31 - (pos & 31))) & 1;
      }
      word |= (uint32_t)(sum >= thr) << (31 - b);
    }
    voted[wd] = word;
  }
}

// parse_stream (amodem_internal.h: modem.js:605-654, 805-849, 793-802) with the same
// decisions in the same order, reading words instead of bytes: the first 16 bytes in one
// ds_read_b128, then each field at a data-dependent offset as one pair of words, so a parse
// is two (chunk / metadata) or three (legacy) dependent LDS round trips (the byte reads
// were one per field byte)
__device__ __forceinline__ uint32_t be32_word(const uint32_t *v, int i) {
  const int wi = i >> 2, sh = 8 * (i & 3);
  const uint32_t a = v[wi], b = v[wi + 1];
  return sh ? (a << sh) | (b >> (32 - sh)) : a;
}
__device__ __forceinline__ int parse_fast(const uint32_t *v, int nbytes, int mode, amod_result &r) {
  r.nbytes = nbytes;
  const int min_bytes = mode == AMOD_MODE_CHUNK ? 6 : 10;
  if (nbytes < min_bytes) { r.status = AMOD_E_DECODED_SHORT; r.frame_type = -1; return -1; }
  const uint4 h = *reinterpret_cast<const uint4 *>(v); // bytes 0 .. 15 (MSB-first words)
  const int t = (int)(h.x >> 24);
  if (t == 0xFE) {
    r.frame_type = 0xFE;
    if (nbytes < 16) { r.status = AMOD_E_META_SHORT; return -1; }
    r.total_chunks = (int32_t)((h.x << 8) | (h.y >> 24));
    r.total_size = (int32_t)((h.y << 8) | (h.z >> 24));
    r.chunk_size = (int32_t)((h.z >> 8) & 0xFFFFu);
    const int nl = (int)(h.z & 0xFFu);
    int off = 12;
    if (off + nl + 4 > nbytes) { r.status = AMOD_E_META_TRUNC; return -1; }
    r.name_off = off; r.name_len = nl;
    off += nl;
    r.expected_crc = be32_word(v, off);
    r.status = AMOD_OK;
    return off;
  }
  if (t == 0xFF) {
    r.frame_type = 0xFF;
    if (nbytes < 11) { r.status = AMOD_E_CHUNK_SHORT; return -1; }
    r.seq_num = (int32_t)((h.x << 8) | (h.y >> 24));
    const int dl = (int)((h.y >> 8) & 0xFFFFu);
    int off = 7;
    if (off + dl + 4 > nbytes) { r.status = AMOD_E_CHUNK_TRUNC; return -1; }
    r.data_off = off; r.data_len = dl;
    off += dl;
    r.expected_crc = be32_word(v, off);
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
  const int32_t dl = (int32_t)be32_word(v, off);
  off += 4;
  if (dl <= 0 || (int64_t)off + dl + 4 > nbytes) { r.status = AMOD_E_INVALID_LEN; r.aux = dl; return -1; }
  r.data_off = off; r.data_len = dl;
  off += dl;
  r.expected_crc = be32_word(v, off);
  r.status = AMOD_OK;
  return off;
}

// the longest prefix parse_need reads: a legacy header (1 + 255 + 4 bytes)
constexpr int kHeaderMaxBytes = 1 + 255 + 4;

struct FrameS {  // wave-uniform facts of one frame on the demodulation path (SGPRs: the
                // frame-end-only fields are re-read from the detection record there; the
                // normalisation A, B with one scalar load per job: held here they were two of
                // the SGPRs the full file spilled and read back every job)
  int f, T, M, start;
  const float *X;
};
__device__ __forceinline__ int frame_jobs(const FrameS &F) { return F.T > 0 ? 1 + F.T / 2 : 0; }

// MOD: the launch's modulation as a template argument (decisions and packing unroll)
// NS: band slots per lane, ceil(nband / 64) (slot rr < NS - 1 is full on every lane)
// SOFT: opt-in soft combining (AMOD_OPT_SOFT_COMBINE, BPSK / QPSK, repetition > 1; not
// reference behaviour): each repeat group is decided by the sign of its
// |H|^2-weighted soft sum, per symbol as the symbol is demodulated (below)
template <bool DBG, int MOD, int NS, bool SOFT = false> __device__ __forceinline__ void demod_loop() {
  constexpr int BPS = MOD == AMOD_BPSK ? 1 : (MOD == AMOD_QPSK ? 2 : 4);
  __shared__ __attribute__((aligned(16))) float2 xch[NWAVE][XCH_F2];
  __shared__ float2 twl[512];   // tw1 rows 1-7 (row q at 64 (q - 1)), then tw2[64]
  __shared__ __attribute__((aligned(16))) uint32_t crc_t4[1024]; // CRC slice-by-4 table (frame ends)
  __shared__ __attribute__((aligned(16))) uint32_t crc_up[16 * 32]; // inverse zero-byte operators
  FRESH_ARGS;
  const int tid = ltid();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  {
    const float2 t1a = cfg.t.tw1[64 + tid], t1b = cfg.t.tw1[64 + min(tid + WG, 447)], t2 = cfg.t.tw2[tid & 63];
    const uint4 c4 = reinterpret_cast<const uint4 *>(cfg.t.crc_s4)[tid];
    twl[tid] = t1a;
    if (tid + WG < 7 * 64) twl[WG + tid] = t1b;
    if (tid < 64) twl[7 * 64 + tid] = t2;
    reinterpret_cast<uint4 *>(crc_t4)[tid] = c4;
    if (tid < 128) reinterpret_cast<uint4 *>(crc_up)[tid] = reinterpret_cast<const uint4 *>(cfg.t.crc_unpad)[tid];
  }
  __syncthreads();
  const int lane = tid & 63;
  const int SYM = cfg.sym, CP = cfg.cp, nband = cfg.nband, sub_start = cfg.sub_start;
  const int ndata = cfg.ndata, per_sym = ndata * BPS, origin_idx = cfg.origin_idx;
  const bool chunk_mode = cfg.mode == AMOD_MODE_CHUNK;
  const float guard = cfg.guard;
  // frames [f0, f1) of this launch, or the list of frames whose detection the exact
  // kernel replayed
  const int nfr = w.dm_list ? __builtin_amdgcn_readfirstlane(*w.dm_count) : w.f1 - w.f0;
  // the wave's bit stream (and voted stream) in dynamic LDS
  uint32_t *const bits = LDS_U + wave * w.stream_words;
  uint32_t *const voted = bits + w.vote_off;
  // the wave's exchange buffer, its base held in a VGPR: as a scalar it was one of the
  // values the full SGPR file spilled to a VGPR lane and read back (v_readlane, VALU) five
  // times a job
  int xoff = wave * XCH_F2;
  asm volatile("" : "+v"(xoff));
  float2 *const X2 = &xch[0][0] + xoff;
  const float2 *const tw1 = twl - 64, *const tw2 = twl + 7 * 64;
  // per-lane band facts for its 4 subcarriers b = bo + 64 rr, bo = (lane - sub_start) mod
  // 64: the bin k = sub_start + b of slot 0 is congruent to the lane mod 64, so each 16-
  // or 32-lane group of a band read covers whole aligned residue blocks of the spectrum
  // (conflict-free under spec_idx; lane l on subcarrier l had every group 2-way, in both
  // halves Z[k] and Z[512 - k]: 16 of k_demod's ~40 conflict cycles per job on C4); the
  // mirrored half stays 2-way in one lane pair per group. The bit offset of its decision
  // in a symbol, di * BPS (di = data index). A slot without a data subcarrier holds
  // BPS * (jk + lane) (a pilot) or BPS * (jk + 64 + lane) (none): its decision store then
  // lands in a junk dword past any job's decision run (jk: two symbols' decisions plus
  // two stream words) by the same address arithmetic as a data slot's, so a store is one
  // add and one shift-add (it was five VALU with the select of a scratch dword)
  // (two 16-bit fields per register: registers bound k_demod's occupancy)
  const int bo0 = (lane - sub_start) & 63;
  const int jk = 2 * ndata + 64;
  uint32_t di_pk[2] = {0u, 0u};
#pragma unroll
  for (int rr = 3; rr >= 0; --rr) {
    const int di = bo0 + 64 * rr < nband ? (int)cfg.t.band_di[bo0 + 64 * rr] : -2;
    const int dib = di >= 0 ? di * BPS : BPS * (jk + lane + (di == -2 ? 64 : 0));
    di_pk[rr >> 1] |= ((uint32_t)dib & 0xFFFFu) << (16 * (rr & 1));
  }
  auto dib_of = [&](int rr) { return (int)(int16_t)(di_pk[rr >> 1] >> (16 * (rr & 1))); };
  // kn_neg bit rr: the CE sign of the lane's band subcarrier rr is -1 (generateChannelEstSymbol);
  // bit 4 + rr: slot rr holds no data subcarrier (a pilot, or none: its decision margin is
  // passed over); bit 8: the lane holds a pilot, bit 9: that pilot's CE sign is -1
  uint32_t kn_neg = 0;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    kn_neg |= (uint32_t)(bo0 + 64 * rr < nband && cfg.t.known[bo0 + 64 * rr] < 0.f) << rr;
    kn_neg |= (uint32_t)(dib_of(rr) >= BPS * jk) << (4 + rr);
  }
  // The pilots are evaluated on lanes of their own: lane p < npilots takes the list's pilot
  // p (the reference loops over OFDM.PILOTS, duplicates included, and skips pilots outside
  // the band: modem.js:398-405), reading its two bins Z[k], Z[512 - k] from the spectrum, so
  // the phase sums reduce over the first 16 lanes (row 0) for every built-in preset and no
  // lane selects its pilot slot out of four. paddr: the LDS byte addresses of the two bins
  // (16 bits each); gp: 1/H at the pilot, set by job 0 like a band slot's G
  uint32_t paddr;
  {
    const int np = cfg.npilots;
    const int kp = lane < np ? cfg.pilots[min(lane, AMOD_MAX_PILOTS - 1)] : -1;
    const bool pin = kp >= sub_start && kp <= cfg.sub_end;
    const int kq = pin ? kp : sub_start; // (a lane without a pilot reads a valid bin)
    const uint32_t a0 = lds_addr(X2 + spec_idx(kq)), a1 = lds_addr(X2 + spec_idx((kFft - kq) & (kFft - 1)));
    paddr = a0 | (a1 << 16);
    kn_neg |= (uint32_t)pin << 8;
    kn_neg |= (uint32_t)(pin && cfg.t.known[kq - sub_start] < 0.f) << 9;
  }
  // bit 10: (wave-uniform) the pilot sums reduce over row 0; bit 11: chunk mode. Read per
  // job from the VGPR with one v_readfirstlane: as scalars the two flags were 64-bit lane
  // masks the full SGPR file spilled and read back (four v_readlane a job)
  kn_neg |= (cfg.npilots <= 16 ? 1u << 10 : 0u) | (chunk_mode ? 1u << 11 : 0u);

  // Frames (last-first: frame f1 - 1 - k for the k-th) by a static stride for the first
  // rounds, then one at a time from the claim counter (w.claim). Waves on one SIMD do not
  // progress alike: VALU issue goes by priority, then age, so the youngest waves get the
  // slots the older ones leave (MI355X_MICROARCH.md, issue arbitration) and under a purely
  // static split they ran the kernel's tail alone (C4: the last-dispatched workgroups'
  // waves lived 2.16 M cycles against 1.67 M for the rest). A wave claims the frame after
  // its current one when it starts the current one, so the atomic's return is long back
  // when it is read (a claim read at once holds up the in-order vmcnt waits of the sample
  // loads: per-frame claims measured slower in round 2)
  int nblk = (int)gridDim.x;
  if (w.yield_blocks > 0 && w.yield_blocks < nblk && __builtin_amdgcn_readfirstlane(*w.yield_count) > 0)
    nblk = w.yield_blocks;
  if ((int)blockIdx.x >= nblk) { // (before any frame: the grid's frames are strided over nblk)
    if (w.tl && lane == 0) w.tl[kTlHead + (int)blockIdx.x * NWAVE + wave] = 0ull;
    return;
  }
  const int wstride = nblk * NWAVE;
  // (at least claim_min frames per wave: a short batch's waves would all claim at once, and
  // same-address device-scope atomics serialise at the memory side: C2, 2.44 frames per
  // wave, lost 59 us that way)
  const int rounds = nfr / wstride;
  const bool dyn = w.claim != nullptr && !DBG && rounds >= w.claim_min;
  const int kstat = dyn ? max(1, rounds - w.claim_rounds) * wstride : nfr; // k < kstat: static
  auto claim = [&]() -> int { // lane 0: the next claimed k - kstat (not waited for here)
    int v = 0;
    if (lane == 0) v = atomicAdd(w.claim, 1);
    return v;
  };
  int pend = 0; // (lane 0) the claim for the frame after the current one
  // the first frame on the demodulation path from candidate k on
  auto next_frame = [&](int k, FrameS &F) -> int {
    FRESH_ARGS;
    while (k < nfr) {
      const int f = w.dm_list ? __builtin_amdgcn_readfirstlane(w.dm_list[k]) : w.f1 - 1 - k;
      const DetRec d = sload(w.det + f);
      if (d.route == (w.dm_list ? ROUTE_REPLAY : ROUTE_DEMOD)) { // (the list launch: replayed frames)
        F.f = f; F.T = d.T; F.M = d.M; F.start = d.start;
        F.X = w.samples + sload(w.off + f);
        return k;
      }
      k = (!dyn || k + wstride < kstat) ? k + wstride : kstat + __builtin_amdgcn_readfirstlane(claim());
    }
    return nfr;
  };
  // symbols of job j: s1 (-2 = the CE symbol), s2 (-1 = none)
  auto job_syms = [](const FrameS &F, int j, int &s1, int &s2) {
    if (j == 0) { s1 = -2; s2 = 0; }
    else { s1 = 2 * j - 1; s2 = 2 * j < F.T ? 2 * j : -1; }
  };
  // the job's samples as buffer loads: the frame is the resource (SGPRs), the window start
  // the scalar offset, 4 lane the vector offset and 256 m the instruction's immediate, so a
  // job's 16 loads cost no address arithmetic (global loads took three VALU each)
  int lane4 = 4 * lane;
  asm volatile("" : "+v"(lane4));
  auto job_loads = [&](const FrameS &F, int j, f2v (&r)[8]) {
    // job j's first symbol window starts 2 (j + 1) symbols after the frame start (the CE
    // symbol for j = 0, data symbol 2j - 1 after it), its second one symbol later when
    // there is one (symbol 2j < T; job 0's data symbol 0 always): job_syms' windows, in
    // three scalar operations
    const int p1 = F.start + CP + 2 * SYM * (j + 1);
    const int p2 = (j == 0 || 2 * j < F.T) ? p1 + SYM : p1;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)F.X, (short)0, 0x7FFFFFFF, 0x00020000);
    int vo = lane4;
    asm volatile("" : "+v"(vo)); // (one offset register: 256 m goes to the immediate, not 8 hoisted copies)
#pragma unroll
    for (int m = 0; m < 8; ++m)
      r[m] = f2v{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo + 256 * m, 4 * p1, 0)),
                 __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo + 256 * m, 4 * p2, 0))};
  };

  f2v gl[4];                  // G = 1/H of the lane's band subcarriers (job 0)
  f2v gp = {0.f, 0.f};        // G = 1/H at the lane's pilot (job 0)
  float wl[4] = {0.f, 0.f, 0.f, 0.f}; // SOFT: the soft weights |H|^2 of the lane's band subcarriers (job 0)
  float wmax = 0.f, dW = 0.f;  // SOFT: the frame's largest weight, and the error bound of every weight
  float gmax = 0.f, zce = 0.f; // guard scales of the frame (job 0)
  // state of the frame being demodulated (wave-uniform): jobs it takes (shrinks once the
  // header says how many bytes the parse reads), those bytes (-1: not yet known), the
  // first data symbol with a decision inside its guard band, flags
  int live_f = -1, fnj = 0, fneed = -1, flag_sym = 0x7fffffff;
  int wflags = 0;  // NONFINITE / CHANNEL: the whole frame goes to the exact kernel
  int sflags = 0;  // DEMAP / PHASE of flag_sym and later: only if the parse reads them
  const int rep = cfg.rep;
  // bytes the parse reads once `dsym` data symbols are demodulated (-1: more needed)
  // (-1 - need: more bytes needed; with *hdr = 1 the header is decoded, so `need` is final)
  // (rep > 1: the known prefix, up to the longest header parse_need reads, is voted by the
  // whole wave first, so lane 0 parses a plain byte stream)
  auto eval_need = [&](const FrameS &F, int dsym, int *hdr = nullptr) -> int {
    const int nbits = F.M * per_sym;
    const int known = min(dsym * per_sym, nbits);
    const int avail = (known / rep) >> 3;
    const uint32_t *src = bits;
    if (SOFT) {
      src = voted; // (built symbol by symbol: every complete group of the known symbols)
    } else if (rep > 1) {
      wave_vote(bits, min(known, kHeaderMaxBytes * 8 * rep), rep, voted);
      __builtin_amdgcn_wave_barrier();
      src = voted;
    }
    int need = 0, fin = 0;
    if (lane == 0) {
      bool f = false;
      need = parse_need(src, 1, avail, (nbits / rep) >> 3, cfg.mode, &f);
      fin = f;
      if (need > avail) need = -1 - need;
    }
    if (hdr) *hdr = __builtin_amdgcn_readfirstlane(fin);
    return __builtin_amdgcn_readfirstlane(need);
  };
  // the last data symbol holding bits of the first `need` parsed bytes. need * 8 * rep is
  // at most the frame's bit count (eval_need never returns more than the decoded bytes), an
  // int: 32-bit unsigned arithmetic (the int64 division was a ~140-SALU software routine)
  auto last_sym_of = [&](int need) -> int {
    const uint32_t nb = (uint32_t)need * 8u * (uint32_t)rep;
    return (int)((nb + (uint32_t)per_sym - 1u) / (uint32_t)per_sym) - 1;
  };
  // one job of frame `cur` (jcur = 0 starts the frame; a frame without data symbols has
  // one empty job, so every frame passes through its frame end)
  // c1 / c2: the job's samples; issue_next() refills them with the next job's once they
  // are folded into the FFT input, so those loads fly under this job's FFT, equalise, demap, finish
  auto run_job = [&](const FrameS &cur, const int jcur, f2v (&c)[8], auto &&issue_next) {
#ifdef AMOD_DEMOD_STAMPS
#define DSTAMP(k, cond)                                                                   \
  do {                                                                                  \
    if (w.stamps && (cond) && lane == 0) w.stamps[(int64_t)cur.f * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define DSTAMP(k, cond) do { } while (0)
#endif
    const int f = cur.f;
    amod_debug *const D = DBG ? w.dbg + f : nullptr;
    if (jcur == 0) { // a new frame: clear its bit stream (SOFT: its voted stream, built by ORs)
      const int nwz = SOFT ? (int)(((uint32_t)(cur.T * per_sym / rep) + 31) >> 5) + 3 : (int)(((uint32_t)(cur.T * per_sym) + 31) >> 5) + 2;
      uint32_t *const zs = SOFT ? voted : bits;
      for (int i = lane; i < nwz; i += 64) zs[i] = 0u;
      live_f = f; fnj = max(frame_jobs(cur), 1); fneed = -1; flag_sym = 0x7fffffff;
      wflags = 0; sflags = 0;
    } else if (jcur >= fnj) { // prefetched before the header showed the frame was complete
      issue_next();
      return;
    }
    // ---------------------------------------------------------------- job (cur, jcur)
    if (cur.T <= 0) issue_next();
    if (cur.T > 0) {
      int s1, s2;
      job_syms(cur, jcur, s1, s2);
      const bool ce = s1 == -2;
      const float first1 = rlane(c[0].x, 0), first2 = rlane(c[0].y, 0);
      f2v v[8];
      // no second symbol: A = B = 0 zeroes the imaginary half (its samples are finite: the
      // last job re-reads the first symbol's, checked below in chunk mode)
      const f2v ab = sload(reinterpret_cast<const f2v *>(&w.det[__builtin_amdgcn_readfirstlane(f)].A)); // scalar: f is wave-uniform
      const float cA = ab.x, cB = ab.y;
      const f2v Av = {cA, s2 >= 0 ? cA : 0.f}, Bv = {cB, s2 >= 0 ? cB : 0.f};
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = __builtin_elementwise_fma(c[m], Av, Bv);
      // a window is constant iff every raw sample equals its first one (all-zero spectrum).
      // One sample per lane settles it for any real signal (some lane differs); only when
      // all 64 agree are the other 448 compared (wave-uniform branch)
      bool const1 = false, const2 = false;
      if (!KO(8)) {
        int ne1 = c[0].x != first1, ne2 = c[0].y != first2;
        const bool q1 = __ballot(ne1) == 0, q2 = __ballot(ne2) == 0;
        if (q1 || q2) {
#pragma unroll
          for (int m = 1; m < 8; ++m) { ne1 |= c[m].x != first1; ne2 |= c[m].y != first2; }
          const1 = q1 && __ballot(ne1) == 0;
          const2 = q2 && __ballot(ne2) == 0;
        }
      }
      DSTAMP(16, jcur == 1);
      DSTAMP(27, jcur == 2); // (job 2 samples ready: minus mark 21 = the wait for its loads)
      // the FFT input is formed before the next job's loads are issued (the compiler
      // otherwise issued the loads first and copied the samples out of their target
      // registers: eight v_mov_b64 per job; C4 k_demod -1.6 %, C5 -2.5 %)
      asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                   "+v"(v[7])::"memory");
      issue_next(); // the samples are in v: the next job's loads fly under this FFT too
      if (!KO(16)) fft512_wave(v, X2, tw1, tw2);
      DSTAMP(17, jcur == 1);
      int ln = lane;
      asm volatile("" : "+v"(ln)); // per-job lane (keeps debug/bit addresses out of registers)
      // per-job copies of the lane's slot facts: their comparisons are made where they are
      // used instead of held as lane masks across the loop (SGPR pairs that spill)
      asm volatile("" : "+v"(di_pk[0]), "+v"(di_pk[1]), "+v"(kn_neg), "+v"(paddr));
      const uint32_t kmode = __builtin_amdgcn_readfirstlane(kn_neg);
      const bool pil16 = (kmode >> 10) & 1, chunk_j = (kmode >> 11) & 1;
      // the band: slot rr of lane ln is subcarrier b = bo + 64 rr, bins k = k0 + 64 rr and
      // 512 - k (spec_idx(n +- 64) = spec_idx(n) +- 64: one base per side, immediate offsets)
      const int bo = (ln - sub_start) & 63; // (recomputed per job: no VGPR held across the loop)
      const int k0 = sub_start + bo;
      const f2v *const zkp = reinterpret_cast<const f2v *>(X2 + spec_idx(k0));
      const f2v *const znp = reinterpret_cast<const f2v *>(X2 + spec_idx(kFft - 192 - k0));
      // this lane's pilot bins (lanes without one read a valid bin and mask it)
      f2v zpk, zpn;
      {
        const uint32_t pa = paddr & 0xFFFFu, pb = paddr >> 16;
        asm volatile("ds_read_b64 %0, %2\n ds_read_b64 %1, %3" : "=v"(zpk), "=v"(zpn) : "v"(pa), "v"(pb));
      }
      float zm = 0.f;
      // twice the reference's X1, X2 (Z = x1 + i x2: X1 = (Z[k] + conj Z[-k]) / 2,
      // X2 = (Z[k] - conj Z[-k]) / 2i); the 1/2 is folded into G below (exact: powers of 2)
      f2v x1[4], x2[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        x1[rr] = x2[rr] = f2v{0.f, 0.f};
        if (rr >= NS) continue; // no subcarrier in this slot
        const f2v zk = zkp[64 * rr], zn = znp[64 * (3 - rr)];
        f2v a = pk_add_conj(zk, zn), c = pk_add_swap_neg(zk, zn);
        float zz = max3_raw(fabsf(zk.x) + fabsf(zk.y), fabsf(zn.x) + fabsf(zn.y), zm);
        // chunk mode, `x || 0` semantics on the exact path: a NaN/Inf sample makes every bin
        // of Z non-finite (each bin is a sum over all 512 inputs with non-zero weights, and
        // Inf * 0 is NaN), so one bin pair per lane stands in for the 1024 samples
        if (rr == 0 && chunk_j && !KO(8) && __ballot(!isfinite(zk.x + zk.y + zn.x + zn.y)))
          wflags |= AMOD_FLAG_NONFINITE;
        if (rr == NS - 1) { // the last slot may be partly filled
          const bool in = bo + 64 * rr < nband;
          a = in ? a : f2v{0.f, 0.f};
          c = in ? c : f2v{0.f, 0.f};
          zz = in ? zz : zm;
        }
        x1[rr] = a; x2[rr] = c; zm = zz;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(zpk), "+v"(zpn));
      const f2v x1p = pk_add_conj(zpk, zpn), x2p = pk_add_swap_neg(zpk, zpn);
      if (ce) {
        // channel estimate from the CE symbol: H = Y * known (X = +-1, modem.js:431-438).
        // Here h = 2H and g = G / 2 (so x g = X G); |h|^2 = 4 |H|^2 against 4 x the thresholds
        zce = wmax_nn(zm);
        float gm = 0.f;
        int ch = 0;
        auto inv = [&](f2v x, bool neg) -> float2 {
          const float kn = neg ? -1.f : 1.f;
          const float2 h = const1 ? make_float2(0.f, 0.f) : make_float2(x.x * kn, x.y * kn);
          const float m2 = h.x * h.x + h.y * h.y;
          float2 g;
          if (m2 > 4.f * 1e-10f) { const float im2 = __builtin_amdgcn_rcpf(m2); g = make_float2(h.x * im2, -h.y * im2); } // 1 ulp: inside the eq bound
          else g = make_float2(0.5f, 0.f); // G = 1 (passthrough)
          return g;
        };
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int b = bo + 64 * rr;
          const float2 g = inv(x1[rr], (kn_neg >> rr) & 1);
          const float2 h = make_float2(x1[rr].x, x1[rr].y);
          const float m2 = const1 ? 0.f : h.x * h.x + h.y * h.y;
          // |H|^2 close to 1e-10 (or tiny but non-zero) decides passthrough differently
          ch |= b < nband && !const1 && m2 < 4.f * 1e-6f;
          // a slot without a data subcarrier (pilot or none) gets G = NaN, so its eq and
          // margins are NaN: v_min / v_max pass NaN over, so the QPSK margin needs no
          // per-slot select and em no mask (the pilots' |eq| enter em from the pilot lanes
          // below). gm above takes the real G. (parity-debug launches keep the real G:
          // they report every band slot's eq)
          const float gx = !DBG && ((kn_neg >> (4 + rr)) & 1) ? __builtin_nanf("") : g.x;
          const float gy = !DBG && ((kn_neg >> (4 + rr)) & 1) ? __builtin_nanf("") : g.y;
          gl[rr] = f2v{gx, gy};
          if (SOFT) wl[rr] = b < nband ? 0.25f * m2 : 0.f; // |H|^2 = |h|^2 / 4
          if (b < nband) gm = fmaxf(gm, fabsf(g.x) + fabsf(g.y));
          if (DBG && b < nband) { const float kn = (kn_neg >> rr) & 1 ? -1.f : 1.f;
            D->h_re[b] = const1 ? 0.f : 0.5f * h.x * kn; D->h_im[b] = const1 ? 0.f : 0.5f * h.y * kn; }
        }
        { const float2 g = inv(x1p, (kn_neg >> 9) & 1); gp = f2v{g.x, g.y}; }
        gmax = wmax_nn(gm); // half of max |G|
        if (__ballot(ch)) wflags |= AMOD_FLAG_CHANNEL;
        if (SOFT) {
          // |H_fast - H| <= 2e-6 guard zce (the FFT bound of the guards, |H| <= zce), so the
          // weight's error is <= (|H_fast| + |H|) |dH| <= 4.1e-6 guard zce^2, plus the fp32
          // rounding of |h|^2 / 4
          wmax = wmax_nn(max3_raw(wl[0], wl[1], fmaxf(wl[2], wl[3])));
          dW = 4.1e-6f * guard * zce * zce + 2.4e-7f * wmax;
        }
      }
      // equalise both halves (the CE half of job 0 is not a data symbol); em bounds |eq| of
      // both symbols of the job
      f2v e1[4], e2[4];
      float em = 0.f;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const f2v g = gl[rr];
        e1[rr] = pk_cmul(x1[rr], g);
        e2[rr] = pk_cmul(x2[rr], g);
        em = max3_raw(em, fabsf(e1[rr].x) + fabsf(e1[rr].y), fabsf(e2[rr].x) + fabsf(e2[rr].y));
        const int b = bo + 64 * rr;
        if (DBG && b < nband && (s1 == 0 || s2 == 0)) {
          const bool one = s1 == 0;
          const f2v xx = one ? x1[rr] : x2[rr], ee = one ? e1[rr] : e2[rr];
          const bool c = one ? const1 : const2;
          D->x_re[b] = c ? 0.f : 0.5f * xx.x; D->x_im[b] = c ? 0.f : 0.5f * xx.y;
          D->eq_re[b] = c ? 0.f : ee.x; D->eq_im[b] = c ? 0.f : ee.y;
        }
      }
      DSTAMP(18, jcur == 1);
      // the pilots' eq (pilot lanes; a lane without one has its sub_start bin's, a data
      // subcarrier's: harmless in the max). Their |eq| joins em: the band slots that hold
      // pilots pass NaN over (above)
      const f2v q1e = pk_cmul(x1p, gp), q2e = pk_cmul(x2p, gp);
      if (!DBG) em = max3_raw(em, fabsf(q1e.x) + fabsf(q1e.y), fabsf(q2e.x) + fabsf(q2e.y));
      // error bound of eq for both symbols (fp32 FFT + channel estimate), DESIGN.md "guards"
      // (gmax is half of max |G|, hence 4e-6)
      float d = 4e-6f * guard * gmax * (zm + em * zce);
      d = wmax_nn(d) + 1e-12f;
      const bool live1 = !ce && !const1, live2 = s2 >= 0 && !const2;
      // pilot phase: mean of eqIm/eqRe over pilots with |eqRe| > 1e-6 (modem.js:398-405), on
      // the pilot lanes
      float ps1, pe1, ps2, pe2;
      int pc1, pc2;
      unsigned long long ph_b1, ph_b2; // pilot lanes whose |eqRe| lies within the band of 1e-6
      {
        const bool pil = (kn_neg >> 8) & 1;
        const float a1 = fabsf(q1e.x), a2 = fabsf(q2e.x);
        const bool w1 = pil && a1 > 1e-6f, w2 = pil && a2 > 1e-6f;
        // (the counts as two 32-bit popcounts: __popcll's 64-bit result compiled to a 64-bit
        // integer-to-float conversion sequence below)
        const unsigned long long bw1 = __ballot(w1), bw2 = __ballot(w2);
        pc1 = __builtin_popcount((uint32_t)bw1) + __builtin_popcount((uint32_t)(bw1 >> 32));
        pc2 = __builtin_popcount((uint32_t)bw2) + __builtin_popcount((uint32_t)(bw2 >> 32));
        // v_rcp_f32 (1 ulp): its error is covered by the 1e-6 |ph| term of tau below
        const float q1 = w1 ? __builtin_amdgcn_rcpf(q1e.x) : 0.f;
        const float q2 = w2 ? __builtin_amdgcn_rcpf(q2e.x) : 0.f;
        ps1 = q1 * q1e.y;
        ps2 = q2 * q2e.y;
        pe1 = fabsf(q1) * fmaf(fabsf(q1e.y), fabsf(q1), 1.f);
        pe2 = fabsf(q2) * fmaf(fabsf(q2e.y), fabsf(q2), 1.f);
        // a pilot |eqRe| near 1e-6 makes that symbol's phase (and every decision) uncertain
        ph_b1 = __ballot(pil && fabsf(a1 - 1e-6f) <= 2.f * d + 1e-7f);
        ph_b2 = __ballot(pil && fabsf(a2 - 1e-6f) <= 2.f * d + 1e-7f);
      }
      if (KO(4)) { ps1 = rlane(ps1, 0); pe1 = rlane(pe1, 0); ps2 = rlane(ps2, 0); pe2 = rlane(pe2, 0); }
      else if (pil16) wsum16_4(ps1, pe1, ps2, pe2);
      else wsum_b4(ps1, pe1, ps2, pe2);
      const float ip1 = pc1 > 0 ? __builtin_amdgcn_rcpf((float)(int32_t)pc1) : 0.f;
      const float ip2 = pc2 > 0 ? __builtin_amdgcn_rcpf((float)(int32_t)pc2) : 0.f;
      const float ph1 = ps1 * ip1, ph2 = ps2 * ip2;
      const float dp1 = d * pe1 * ip1 + 1e-6f * fabsf(ph1), dp2 = d * pe2 * ip2 + 1e-6f * fabsf(ph2);
      const float tau1 = 4.f * (d * (1.f + fabsf(ph1)) + em * dp1) + 1e-9f;
      const float tau2 = 4.f * (d * (1.f + fabsf(ph2)) + em * dp2) + 1e-9f;
      DSTAMP(19, jcur == 1);
      if (DBG && ln == 0) {
        if (s1 >= 0 && s1 < AMOD_DBG_SYMS) D->phase[s1] = const1 ? 0.f : ph1;
        if (s2 >= 0 && s2 < AMOD_DBG_SYMS) D->phase[s2] = const2 ? 0.f : ph2;
      }
      // a constant FFT window has an all-zero spectrum in the reference: every data
      // subcarrier takes the origin decision (ties resolve to the first point).
      // The job's decisions (symbols s1, s2: a contiguous run [gs, ge) of the frame's
      // decision sequence) go to the exchange buffer, free again once the band is in
      // registers: one dword per decision (conflict-free ds_write_b32, consecutive data
      // indices on consecutive lanes), its bits already at their place in the stream word
      // (BPS divides 32, so a decision never straddles a word; v_lshrrev takes the
      // position mod 32). Word wfirst + i of the stream is then the OR of dwords
      // [DPW i, DPW i + DPW), one lane per word, one ds_or into the stream (the first
      // word's top bits belong to the previous job).
      constexpr int DPW = 32 / BPS; // decisions per stream word
      uint32_t *const dec = reinterpret_cast<uint32_t *>(X2);
      const int nd = kargs().cfg.ndata; // (a fresh scalar load: ndata itself is spilled by here)
      const int gs = (ce ? 0 : s1) * nd, ge = ((s2 >= 0 ? s2 : s1) + 1) * nd;
      // (non-negative: unsigned shifts and masks, not the signed division's sign fix-ups)
      const int wfirst = (int)((uint32_t)gs / DPW), g0 = wfirst * DPW;
      const int gend = (int)(((uint32_t)ge + DPW - 1) & ~(uint32_t)(DPW - 1));
      asm volatile("" ::: "memory"); // (the band reads above are float2 accesses of the same LDS)
      // the first and last words' dwords outside [gs, ge) are zeroed (lanes < DPW); every
      // other lane stores into a junk dword past any decision or junk dword of the job, so
      // the stores take no exec-mask block
      if (!SOFT) {
        const int jz = jk + ndata + DPW + 128 + ln; // (< 1152 dwords: the exchange buffer)
        const int z1 = ln < DPW && g0 + ln < gs ? ln : jz;
        const int z2 = ln < DPW && ge + ln < gend ? ge - g0 + ln : jz;
        dec[z1] = 0u;
        dec[z2] = 0u;
      }
      const uint32_t org_bits = (uint32_t)origin_idx << (32 - BPS);
      char *const decg = reinterpret_cast<char *>(dec) - 4 * g0; // (byte base of decision index 0)
      // the guard: each symbol's smallest decision margin over the lane's data slots (a slot
      // without a data subcarrier counts as +inf), compared once with the symbol's band
      const f2v phv1 = f2v{ph1, ph1}, phv2 = f2v{ph2, ph2};
      const uint32_t lm31a = live1 ? 0x80000000u : 0u, lm30a = live1 ? 0x40000000u : 0u; // (QPSK, BPSK)
      const uint32_t lm31b = live2 ? 0x80000000u : 0u, lm30b = live2 ? 0x40000000u : 0u;
      const int sbase1 = s1 * per_sym, sbase2 = s2 * per_sym;
      float mm1 = __builtin_inff(), mm2 = __builtin_inff();
      // one slot's decision for symbol `which` (0: s1, 1: s2)
      auto slot_dec = [&](int rr, auto which_c) {
        constexpr int which = decltype(which_c)::value;
        const bool nd = (kn_neg >> (4 + rr)) & 1; // a pilot slot, or no subcarrier
        const f2v c = pk_derot(which == 0 ? e1[rr] : e2[rr], which == 0 ? phv1 : phv2);
        uint32_t db;
        float margin;
        float &mm = which == 0 ? mm1 : mm2;
        if (MOD == AMOD_QPSK) {
          // the sign-bit decision with the symbol's liveness folded into its two masks:
          // QPSK's origin decision is index 0 (four equidistant points, the first kept:
          // runtime.cpp demap_exact(QPSK, 0, 0)), so a dead symbol's bits are 0 and no
          // per-slot select is needed
          const uint32_t a = __float_as_uint(c.x), b = __float_as_uint(c.y);
          db = (b & (which == 0 ? lm31a : lm31b)) | (((a ^ b) >> 1) & (which == 0 ? lm30a : lm30b));
          if (!DBG) {
            // the symbol's smallest margin min(|re|, |im|) in one v_min3_f32 with |.| source
            // modifiers; a slot without a data subcarrier has NaN components (G = NaN at the
            // CE), which v_min passes over
            asm("v_min3_f32 %0, %0, |%1|, |%2|" : "+v"(mm) : "v"(c.x), "v"(c.y));
          } else {
            // min(|re|, |im|) as one v_min_f32 with |.| source modifiers (fminf, and
            // fmed3 folded into it, canonicalised both inputs first: two more VALU per slot)
            asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(margin) : "v"(c.x), "v"(c.y));
            margin = nd ? __builtin_inff() : margin;
            asm("v_min_f32 %0, %1, %2" : "=v"(mm) : "v"(mm), "v"(margin));
          }
        } else if (MOD == AMOD_BPSK && !DBG) {
          // BPSK: index 1 iff re < 0, the origin decision is index 0: the sign bit under the
          // liveness mask (re = -0 decides 1 here but has margin 0, inside every band: the
          // frame goes to the exact kernel); the margin |re| straight into the symbol's
          // minimum (NaN for a slot without a data subcarrier: passed over)
          db = __float_as_uint(c.x) & (which == 0 ? lm31a : lm31b);
          asm("v_min_f32_e64 %0, %0, |%1|" : "+v"(mm) : "v"(c.x));
        } else {
          db = (uint32_t)decide(MOD, c.x, c.y, margin) << (32 - BPS);
          db = (which == 0 ? live1 : live2) ? db : org_bits;
          margin = nd ? __builtin_inff() : margin;
          // (v_min_f32 without fminf's canonicalisation: a NaN margin is passed over, as the
          // comparison of the per-slot form was false for it)
          asm("v_min_f32 %0, %1, %2" : "=v"(mm) : "v"(mm), "v"(margin));
        }
        // dword pos / BPS - g0 of the buffer (a lane without a data subcarrier in this slot
        // stores into its junk dword: no exec-mask block per store); pos is a multiple of
        // BPS, so the byte offset is pos * (4 / BPS): one shift-add from the job's base
        const uint32_t pos = (uint32_t)((which == 0 ? sbase1 : sbase2) + dib_of(rr));
        *reinterpret_cast<uint32_t *>(decg + pos * (4 / BPS)) = db >> (pos & 31);
      };
      using W0 = std::integral_constant<int, 0>;
      using W1 = std::integral_constant<int, 1>;
      if constexpr (SOFT) {
        // Soft combining, one symbol at a time: every data subcarrier's soft values (BPSK: the
        // phase-corrected real part; QPSK: the imaginary part for the first bit, the max-log
        // min(|re|, |im|), negative where the signs differ, for the second; each times the
        // weight |H|^2 of its subcarrier, as the exact kernel forms them) go to the exchange
        // buffer at their bit offset in the symbol; then lane l sums repeat group jS + l
        // (every bit of it in this symbol, plus the carried partial sum of a group that
        // began in the previous one) and the signs of the complete groups are ORed into the
        // voted stream by one ballot per 64 groups. The error of each soft value is bounded
        // by the symbol's decision band tau (2 tau for QPSK's max-log value: a sign change
        // of a component within tau moves it by at most 2 tau), the weight's dW and the
        // fp32 roundings; a group whose sum lies within the sum of its values' bounds is
        // uncertain, and its symbol routes the frame to the exact kernel.
        // (value, error bound) per bit of the symbol: the bound per value, from the value's own
        // |eq| (the symbol band tau takes the largest |eq| of the job: several times looser)
        f2v *const sb = reinterpret_cast<f2v *>(X2);
        float *const carry = reinterpret_cast<float *>(bits); // (the raw stream is unused here)
        constexpr float KS = MOD == AMOD_QPSK ? 2.f : 1.f;
        auto soft_sym = [&](auto which_c, int s, bool live, float ph, float dp) {
          constexpr int which = decltype(which_c)::value;
          const f2v phv = f2v{ph, ph};
          const float aph = 1.f + fabsf(ph);
#pragma unroll
          for (int rr = 0; rr < NS; ++rr) {
            const bool nd = (kn_neg >> (4 + rr)) & 1;
            const f2v e = which == 0 ? e1[rr] : e2[rr];
            const f2v c = pk_derot(e, phv);
            const float w = live ? wl[rr] : 0.f; // (a constant window: the exact values are 0)
            const float ea = fabsf(e.x) + fabsf(e.y);
            // this value's |c - c_exact| bound: the guards' tau with its own |eq| in the phase
            // term (d stays the wave's: the FFT error is set by the whole spectrum's scale)
            const float tau = 4.f * (d * aph + ea * dp) + 1e-9f;
            const float ca = ea * aph; // bounds |re|, |im| of c
            const float ev = live ? KS * tau * (w + dW) + ca * dW + 2.4e-7f * ca * w : 0.f;
            const int o = nd ? BPS * ndata + 8 + BPS * ln : dib_of(rr); // bit offset (junk past the symbol)
            if (MOD == AMOD_BPSK) {
              sb[o] = f2v{c.x * w, ev};
            } else {
              float m;
              asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(m) : "v"(c.x), "v"(c.y));
              sb[o] = f2v{c.y * w, ev};
              sb[o + 1] = f2v{((__float_as_uint(c.x) ^ __float_as_uint(c.y)) >> 31 ? -m : m) * w, ev};
            }
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
          const int P0 = s * per_sym, P1 = P0 + per_sym;
          const int jS = P0 / rep, jE = P1 / rep; // groups [jS, jE) complete here; jE partial
          const bool strad = jS * rep < P0;
          const float c0 = carry[0], ce0 = carry[1]; // (the previous symbol's partial group)
          bool unc = false;
          for (int g0 = jS; g0 <= jE; g0 += 64) { // (one pass for every built-in preset)
            const int j = g0 + ln;
            float sum = 0.f, E = 0.f, sa = 0.f;
            if (j <= jE) {
              const int b0 = j * rep;
              for (int u = 0; u < rep; ++u) {
                const int b = b0 + u;
                if (b >= P0 && b < P1) { const f2v t = sb[b - P0]; sum += t.x; E += t.y; sa += fabsf(t.x); }
              }
              if (j == jS && strad) { sum += c0; E += ce0; sa += fabsf(c0); }
            }
            E += 6e-8f * (float)rep * sa; // (the fp32 sum of at most rep values)
            const bool full = j < jE;
            const uint64_t m = __ballot(full && sum < 0.f);
            unc |= __ballot(full && fabsf(sum) <= E) != 0;
            if (j == jE && jE * rep < P1) { carry[0] = sum; carry[1] = E; } // (one lane)
            // groups g0 + l, MSB-first in the voted words: word (g0 >> 5), bit 31 - (g0 & 31) on
            const uint64_t R = __builtin_bitreverse64(m);
            const int ob = g0 & 31, W = g0 >> 5;
            if (ln < 3) {
              const uint32_t wv = ln == 0 ? (uint32_t)(R >> (32 + ob))
                                : ln == 1 ? (uint32_t)(R >> ob) : (ob ? (uint32_t)(R << (32 - ob)) : 0u);
              atomicOr(voted + W + ln, wv);
            }
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
          return live && unc;
        };
        if (s1 >= 0 && soft_sym(W0{}, s1, live1, ph1, dp1)) mm1 = -1.f; // (mm <= tau: the flags below)
        if (s2 >= 0 && soft_sym(W1{}, s2, live2, ph2, dp2)) mm2 = -1.f;
      } else if (!KO(2)) {
        // (wave-uniform) both halves data symbols: every job but a frame's first (the CE
        // half) and, for an even symbol count, its last, as one straight-line block
        if (s1 >= 0 && s2 >= 0) {
#pragma unroll
          for (int rr = 0; rr < NS; ++rr) { slot_dec(rr, W0{}); slot_dec(rr, W1{}); }
        } else if (s2 >= 0) {
#pragma unroll
          for (int rr = 0; rr < NS; ++rr) slot_dec(rr, W1{});
        } else {
#pragma unroll
          for (int rr = 0; rr < NS; ++rr) slot_dec(rr, W0{});
        }
      }
      // the job's guard events as lane masks, tested once: any of them is rare, and only
      // then are the symbols' flags worked out (one scalar test per job, not a chain of
      // scalar selects per symbol and flag)
      const unsigned long long dm_b1 = __ballot(mm1 <= tau1), dm_b2 = __ballot(mm2 <= tau2);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      // (lane i reads its NQ 16-byte pieces starting at piece i / (16 / NQ) mod NQ: the 16
      // lanes of each ds_read_b128 group then cover 16 distinct 16-byte bank slots; in
      // order, lanes i and i + 16 / NQ hit the same slot: 4-way for QPSK). A job's run is
      // at most 2 ndata / DPW + 2 words: one pass of the wave for BPSK and QPSK.
      constexpr int NQ = DPW / 4;
      const int rot = (int)(((uint32_t)ln / (16 / NQ)) & (NQ - 1));
      const int nwj = (KO(2) || SOFT) ? 0 : (int)((uint32_t)(gend - g0) / DPW);
      for (int i = ln; i < nwj; i += 64) {
        const uint4 *const q = reinterpret_cast<const uint4 *>(dec + DPW * i);
        uint4 t[NQ]; // (every piece requested before the first is combined: one LDS wait)
#pragma unroll
        for (int k = 0; k < NQ; ++k) t[k] = q[(k + rot) & (NQ - 1)];
        uint32_t word = 0u;
#pragma unroll
        for (int k = 0; k < NQ; ++k) word |= (t[k].x | t[k].y) | (t[k].z | t[k].w);
        atomicOr(bits + wfirst + i, word);
        if (BPS <= 2) break; // (one pass covers a BPSK or QPSK run: <= 2 * 255 / DPW + 2 words)
      }
      asm volatile("" ::: "memory"); // (the next FFT rewrites the buffer)
      {
        // (live1 / live2 imply s1 / s2 >= 0)
        if (!KO(0xFFFF) && ((live1 ? dm_b1 | ph_b1 : 0ull) | (live2 ? dm_b2 | ph_b2 : 0ull)) != 0) {
          const bool d1u = live1 && dm_b1 != 0, d2u = live2 && dm_b2 != 0;
          const bool p1u = live1 && ph_b1 != 0, p2u = live2 && ph_b2 != 0;
          if (d1u || p1u) {
            flag_sym = min(flag_sym, s1);
            sflags |= (d1u ? AMOD_FLAG_DEMAP : 0) | (p1u ? AMOD_FLAG_PHASE : 0);
          }
          if (d2u || p2u) {
            flag_sym = min(flag_sym, s2);
            sflags |= (d2u ? AMOD_FLAG_DEMAP : 0) | (p2u ? AMOD_FLAG_PHASE : 0);
          }
        }
      }
      DSTAMP(20, jcur == 1);
      __builtin_amdgcn_wave_barrier();
      DSTAMP(21, jcur == 1);
      // once the header is decoded the parse's byte range is known: the frame takes only
      // the jobs that demodulate it (trailing silence or noise is never transformed)
      if (!DBG && fneed < 0 && !wflags && !KO(0x400)) { // (parity-debug launches demodulate every symbol)
        const int dsym = jcur == 0 ? 1 : min(2 * jcur + 1, cur.T);
        // (the job count only ever shrinks, once the answer is final: the next job was
        // chosen before this one ran, so a frame whose count grew would lose jobs)
        int hdr = 0;
        int need = eval_need(cur, dsym, &hdr);
        if (need < 0 && hdr) need = -1 - need; // header decoded: the byte count is final
        if (need >= 0) {
          // jobs holding the last data symbol the parse reads (job j: symbols 2j-1, 2j)
          const int ls = need > 0 ? last_sym_of(need) : 0;
          const int jn = ls <= 0 ? 1 : (ls + 1) / 2 + 1;
          const int availT = (min(cur.T * per_sym, cur.M * per_sym) / rep) >> 3;
          if (need > availT) {
            wflags |= AMOD_FLAG_SPAN; // past the demodulated symbols: the exact kernel
            fnj = jcur + 1;
          } else {
            fneed = need;
            if (!KO(0xFFFF)) fnj = min(fnj, max(jcur + 1, jn));
          }
        }
      }
    }
    // ---------------------------------------------------------------- frame end
    if (jcur + 1 >= fnj && !KO(0x200)) {
      FRESH_ARGS; // the finish's tables and outputs: scalar loads here, not held across the loop
      DSTAMP(22, true);
      const int nbits = cur.M * per_sym;
      const int decoded = cur.T * per_sym;
      int need = fneed;
      if (need < 0 && !wflags) {
        need = eval_need(cur, cur.T); // no job (T = 0), or the symbols ran out first
        if (need < 0) wflags |= AMOD_FLAG_SPAN;
      }
      // the last data symbol whose bits the parse reads
      const int last_sym = need > 0 ? last_sym_of(need) : -1;
      if (flag_sym <= last_sym) wflags |= sflags;
      DSTAMP(23, true);
      if (KO(0xFFFF)) wflags = 0;
      if (wflags) {
        if (lane == 0) list_exact(w, f, wflags);
      } else {
        {
          const uint32_t *v = SOFT ? voted : bits;
          if (!SOFT && rep > 1) { // vote only the decoded prefix the parse reads
            wave_vote(bits, min(decoded, need * 8 * rep), rep, voted);
            __builtin_amdgcn_wave_barrier();
            v = voted;
          }
          // parse (modem.js:605-654, 793-849), CRC over [0, off), payload prefix
          amod_result r;
          init_result(r);
          r.nbits = nbits;
          if (cfg.mode == AMOD_MODE_RECEIVED) {
            const DetRec dr = sload(w.det + f);
            r.fine_metric = dr.fbest; r.coarse_idx = dr.coarse; r.preamble_idx = cur.start;
            r.flags = dr.flags; // AMOD_FLAG_REPLAY (+ why) for a replayed detection, else 0
          }
          const int nbytes = (nbits / rep) >> 3;
          const int crc_len = parse_fast(v, nbytes, cfg.mode, r); // every lane: the same bytes
          if (cfg.mode == AMOD_MODE_RECEIVED) {
            // preambleIdx is reported on legacy success and on every 0xFE/0xFF result (609-620)
            const bool keep = (r.frame_type == 0xFE || r.frame_type == 0xFF) || (r.frame_type == 0 && r.status == AMOD_OK);
            if (!keep) r.preamble_idx = -1;
          } else {
            r.preamble_idx = -1;
          }
          DSTAMP(24, true);
          if (crc_len >= 0) {
            // slice-by-4 lookups in the workgroup's LDS copy of the table
            r.actual_crc = KO(1) ? r.expected_crc : crc_len <= kCrcMats * kCrcChunk
                               ? wave_crc32(v, crc_len, cfg.t, crc_t4, crc_up,
                                            kDemodStamps && w.stamps ? w.stamps + (int64_t)f * 32 : nullptr)
                               : wave_crc32_long(v, crc_len, cfg.t);
            r.crc_valid = r.expected_crc == r.actual_crc;
          }
          DSTAMP(25, true);
          const int store_bytes = min(need, nbytes);
          r.payload_valid = store_bytes;
          // payload bytes, big-endian words -> memory order, 16 bytes per lane and store
          // (the slot stride is a multiple of 16; bytes past store_bytes in the last 16 are
          // written as zero, the value the slot holds past payload_valid)
          const int nq = (store_bytes + 15) >> 4;
          uint4 *const dst = reinterpret_cast<uint4 *>(w.payload + (int64_t)f * w.stride);
          const int cap_q = (int)(w.stride >> 4);
          const int nql = min(nq, cap_q);
          for (int i0 = 0; i0 < nql; i0 += 128) { // (two rows per lane per pass, both read first)
            const int ia = i0 + lane, ib = ia + 64;
            const uint4 qa = reinterpret_cast<const uint4 *>(v)[min(ia, nql - 1)];
            const uint4 qb = reinterpret_cast<const uint4 *>(v)[min(ib, nql - 1)];
            auto put = [&](int i, uint4 q) {
              const int keep = store_bytes - 16 * i; // bytes of these 16 that were decoded
              auto msk = [&](uint32_t wd, int k) -> uint32_t {
                const int b = keep - 4 * k;
                return __builtin_bswap32(b >= 4 ? wd : b <= 0 ? 0u : wd & ~(0xFFFFFFFFu >> (8 * b)));
              };
              if (i < nql) dst[i] = make_uint4(msk(q.x, 0), msk(q.y, 1), msk(q.z, 2), msk(q.w, 3));
            };
            put(ia, qa);
            put(ib, qb);
          }
          if (DBG && lane == 0) D->nsym = cur.M;
          // the record: 24 words, one per lane (lane writes, not 24 lane==i masks: those are
          // loop-invariant, get hoisted out of the persistent loop and spill 48 SGPRs)
          const int32_t *const rw = reinterpret_cast<const int32_t *>(&r);
          int32_t val = 0;
#pragma unroll
          for (int i = 0; i < 24; ++i) asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(val) : "s"(__builtin_amdgcn_readfirstlane(rw[i])), "n"(i));
          if (lane < 24) reinterpret_cast<int32_t *>(w.res + f)[lane] = val;
          DSTAMP(26, true);
        }
      }
      __builtin_amdgcn_wave_barrier(); // the stream is read before the next frame clears it
    }
  };
  // the job after (F, k, j): the frame's next, or the next frame's first; false at the end
  auto advance = [&](FrameS &F, int &k, int &j) -> bool {
    if (j + 1 < (F.f == live_f ? fnj : max(frame_jobs(F), 1))) { ++j; return true; }
    FrameS nf;
    const int kc = (!dyn || k + wstride < kstat) ? k + wstride : kstat + __builtin_amdgcn_readfirstlane(pend);
    const int kn = next_frame(kc, nf);
    if (kn >= nfr) return false;
    F = nf; k = kn; j = 0;
    if (dyn && kn + wstride >= kstat) pend = claim(); // (for the frame after this one)
    return true;
  };
  // every load is unconditional (a frame without data symbols reads its CE window, the
  // last job re-reads its own samples), so the in-order vmcnt accounting stays exact
  auto loads = [&](const FrameS &F, int j, f2v (&r)[8]) { job_loads(F, j, r); };
  // the sample registers are refilled with the next job as soon as the FFT input is formed
  FrameS fa, fb;
  int ka = next_frame((int)blockIdx.x * NWAVE + wave, fa), ja = 0, kb, jb;
  if (dyn && ka < nfr && ka + wstride >= kstat) pend = claim();
  if (ka >= nfr) {
    if (w.tl && lane == 0) w.tl[kTlHead + (int)blockIdx.x * NWAVE + wave] = 0ull;
    return;
  }
  const int f_first = fa.f; // diagnostics (AMOD_STAMPS): the wave's lifetime in its first frame's marks
  if (kDemodStamps && w.stamps && lane == 0) w.stamps[(int64_t)f_first * 32 + 28] = __builtin_amdgcn_s_memtime();
  f2v r[8];
  loads(fa, ja, r);
  for (;;) {
    fb = fa; kb = ka; jb = ja;
    const bool hb = advance(fb, kb, jb);
    run_job(fa, ja, r, [&] { if (hb) loads(fb, jb, r); });
    if (!hb) break;
    fa = fb; ka = kb; ja = jb;
  }
  if (kDemodStamps && w.stamps && lane == 0) w.stamps[(int64_t)f_first * 32 + 29] = __builtin_amdgcn_s_memtime();
  if (w.tl && lane == 0) w.tl[kTlHead + (int)blockIdx.x * NWAVE + wave] = (unsigned long long)wall_clock64();
}
template <int MOD, int NS> __global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(AMOD_DEMOD_WPE))) void k_demod(const DevCfg cfg_arg, const DevWork w_arg) {
  (void)cfg_arg;
  (void)w_arg;
  demod_loop<false, MOD, NS>();
}
template <int MOD, int NS> __global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(AMOD_DEMOD_WPE))) void k_demod_soft(const DevCfg cfg_arg, const DevWork w_arg) {
  (void)cfg_arg;
  (void)w_arg;
  demod_loop<false, MOD, NS, true>();
}
template <int MOD, int NS> __global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(AMOD_DEMOD_WPE))) void k_demod_dbg(const DevCfg cfg_arg, const DevWork w_arg) {
  (void)cfg_arg;
  (void)w_arg;
  demod_loop<true, MOD, NS>();
}
typedef void (*demod_fn)(const DevCfg, const DevWork);
template <int MOD> __host__ demod_fn demod_kernel_ns(int ns, bool dbg) {
  switch (ns) {
  case 1: return dbg ? k_demod_dbg<MOD, 1> : k_demod<MOD, 1>;
  case 2: return dbg ? k_demod_dbg<MOD, 2> : k_demod<MOD, 2>;
  case 3: return dbg ? k_demod_dbg<MOD, 3> : k_demod<MOD, 3>;
  default: return dbg ? k_demod_dbg<MOD, 4> : k_demod<MOD, 4>;
  }
}
template <int MOD> __host__ demod_fn demod_kernel_soft(int ns) {
  switch (ns) {
  case 1: return k_demod_soft<MOD, 1>;
  case 2: return k_demod_soft<MOD, 2>;
  case 3: return k_demod_soft<MOD, 3>;
  default: return k_demod_soft<MOD, 4>;
  }
}
__host__ demod_fn demod_kernel(const DevCfg &cfg, bool dbg, bool soft = false) {
  const int ns = (cfg.nband + 63) / 64; // validate(): 1 <= nband <= 255
  if (soft && !dbg) return cfg.mod == AMOD_BPSK ? demod_kernel_soft<AMOD_BPSK>(ns) : demod_kernel_soft<AMOD_QPSK>(ns);
  if (cfg.mod == AMOD_BPSK) return demod_kernel_ns<AMOD_BPSK>(ns, dbg);
  if (cfg.mod == AMOD_QPSK) return demod_kernel_ns<AMOD_QPSK>(ns, dbg);
  return demod_kernel_ns<AMOD_QAM16>(ns, dbg);
}


} // namespace
} // namespace amod

// experiments (AMOD_MALL_FLUSH_MB): stream a scratch buffer through L2 / the Infinity
// Cache, so the next launch finds none of the previous launches' lines there
namespace amod {
__global__ __launch_bounds__(256) void k_flush(const float *__restrict__ p, size_t n, float *sink) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n / 4; i += (size_t)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4 *>(p)[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1.2345e-30f) *sink = acc; // (keeps the loads)
}
} // namespace amod

extern "C" hipError_t amod_launch_flush(const void *buf, size_t bytes, float *sink, hipStream_t s) {
  hipLaunchKernelGGL(amod::k_flush, dim3(4096), dim3(256), 0, s, (const float *)buf, bytes / 4, sink);
  return hipGetLastError();
}

// ------------------------------------------------------------ launchers
// dynamic LDS bytes of a k_detect workgroup with nb_cap moment blocks and fine_cap
// fine-search positions
extern "C" int amod_fast_lds_bytes(int nb_cap, int fine_cap, int sym) {
  using namespace amod;
  const int mom = 12 * nb_cap + 2 * SC_MAXCAND + 4 * SC_MAXCAND + 8 * 32 * SC_CACHE;
  const int fine = 4 * fine_floats(fine_cap, sym);
  return (std::max(mom, fine) + 15) & ~15;
}
// per-wave bit-stream words of k_demod (stream, then the voted stream when rep > 1)
extern "C" void amod_demod_stream_words(const amod::DevCfg &cfg, int mcap, int *stream_words, int *vote_off) {
  const int s = ((mcap * cfg.ndata * cfg.bps + 31) / 32 + 4 + 3) & ~3;
  const int v = cfg.rep > 1 ? ((s / cfg.rep + 4 + 3) & ~3) : 0;
  *vote_off = s;
  *stream_words = s + v;
}

// both launchers take frames [w.f0, w.f1)
extern "C" hipError_t amod_launch_detect(const amod::DevCfg &cfg, const amod::DevWork &w, hipStream_t s) {
  const int n = w.f1 - w.f0;
  if (n <= 0) return hipSuccess;
  if (cfg.mode == AMOD_MODE_CHUNK) {
    hipLaunchKernelGGL(amod::k_chunk_prep, dim3((n + amod::WG - 1) / amod::WG), dim3(amod::WG), 0, s, cfg, w);
    return hipGetLastError();
  }
  auto *k = w.dbg ? amod::k_detect_dbg : (cfg.stop_after == 1 ? amod::k_corr_scan : amod::k_detect);
  hipLaunchKernelGGL(k, dim3(n), dim3(amod::WG), (unsigned)amod_fast_lds_bytes(w.nb_cap, w.fine_cap, cfg.sym), s, cfg, w);
  return hipGetLastError();
}
extern "C" hipError_t amod_launch_demod(const amod::DevCfg &cfg, const amod::DevWork &w, int nblocks, hipStream_t s) {
  if (w.f1 <= w.f0 || nblocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(amod::demod_kernel(cfg, w.dbg != nullptr, amod::soft_fast(w.options, cfg)), dim3(nblocks), dim3(amod::WG),
                     (unsigned)(4 * amod::NWAVE * w.stream_words), s, cfg, w);
  return hipGetLastError();
}
// k_demod blocks resident at once on one CU for a dynamic LDS of lds bytes
extern "C" int amod_demod_blocks_per_cu(const amod::DevCfg &cfg, int lds, bool soft) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, amod::demod_kernel(cfg, false, soft), amod::WG, lds) != hipSuccess ||
      n <= 0)
    n = 4;
  return n;
}
