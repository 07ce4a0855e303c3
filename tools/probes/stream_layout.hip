// Experiments only: does the wave-to-address layout of a per-frame streaming pass matter?
// 10,000 frames of 35,874 floats (C2's batch, 1.435 GB); one 256-thread workgroup per frame
// (as k_detect), float4 buffer loads, 9 in flight per wave; every wave sums its samples
// (a stand-in for the stream pass's moments). Layouts:
//   0: wave w reads a contiguous quarter of the frame (k_detect's stream pass)
//   1: the workgroup reads the frame in 4 KB rounds, wave w the w-th KB of each round
// Also a grid-stride copy-style read of the whole batch (the guide's float4 rate).
// hipcc --offload-arch=gfx950 -O3 -o tools/probes/stream_layout tools/probes/stream_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int F = 10000, SPF = 35874;

template <int LAYOUT>
__global__ __launch_bounds__(256) void k_frames(const float *x, float *out) {
  const int f = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float *X = x + (size_t)f * SPF;
  const int nvec = SPF / 4;  // whole float4s (alignment: frames start at multiples of 2 floats: use raw loads)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)X, (short)0, 16 * nvec, 0x00020000);
  const int nch = (nvec + 63) / 64; // 1 KB chunks
  float acc = 0.f;
  auto ld = [&](int q) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 1024 * q, 0);
    return __uint_as_float(v[0]) + __uint_as_float(v[1]) + __uint_as_float(v[2]) + __uint_as_float(v[3]);
  };
  if (LAYOUT == 0) {
    const int q0 = wave * nch / 4, q1 = (wave + 1) * nch / 4;
    int q = q0;
    for (; q + 9 <= q1; q += 9) {
      float t[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) t[j] = ld(q + j);
#pragma unroll
      for (int j = 0; j < 9; ++j) acc += t[j];
    }
    for (; q < q1; ++q) acc += ld(q);
  } else {
    int q = wave;
    for (; q + 4 * 8 < nch; q += 4 * 9) {
      float t[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) t[j] = ld(q + 4 * j);
#pragma unroll
      for (int j = 0; j < 9; ++j) acc += t[j];
    }
    for (; q < nch; q += 4) acc += ld(q);
  }
  if (acc == 1234.5f) out[f] = acc; // (keep the loads)
}

__global__ __launch_bounds__(256) void k_grid(const float4 *x, size_t n4, float *out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  const size_t n = (size_t)F * SPF + 64;
  float *x, *out;
  hipMalloc(&x, n * 4);
  hipMalloc(&out, F * 4);
  hipMemset(x, 0, n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const double bytes = 4.0 * F * SPF;
  for (int rep = 0; rep < 3; ++rep) {
    for (int l = 0; l < 3; ++l) {
      for (int w = 0; w < 5; ++w) {
        if (l == 0) hipLaunchKernelGGL(k_frames<0>, dim3(F), dim3(256), 0, 0, x, out);
        else if (l == 1) hipLaunchKernelGGL(k_frames<1>, dim3(F), dim3(256), 0, 0, x, out);
        else hipLaunchKernelGGL(k_grid, dim3(256 * 16), dim3(256), 0, 0, (const float4 *)x, (size_t)F * SPF / 4, out);
      }
      hipEventRecord(a);
      const int K = 20;
      for (int k = 0; k < K; ++k) {
        if (l == 0) hipLaunchKernelGGL(k_frames<0>, dim3(F), dim3(256), 0, 0, x, out);
        else if (l == 1) hipLaunchKernelGGL(k_frames<1>, dim3(F), dim3(256), 0, 0, x, out);
        else hipLaunchKernelGGL(k_grid, dim3(256 * 16), dim3(256), 0, 0, (const float4 *)x, (size_t)F * SPF / 4, out);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      ms /= K;
      printf("%s: %.4f ms  %.2f TB/s\n", l == 0 ? "frames, wave quarters" : l == 1 ? "frames, 4 KB rounds  " : "grid-stride float4    ",
             ms, bytes / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
