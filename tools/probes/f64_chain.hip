// Probe (experiments only): cycles per dependent fp64 add on one wave, alone and with LDS
// traffic, to bound the exact replica's Schmidl-Cox chain (tools/probes, not product code).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain(const double *in, double *out, long long *cyc, int n, int lanes) {
  __shared__ double2 buf[4096];
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += blockDim.x) buf[i] = make_double2(in[i & 1023], in[(i + 7) & 1023]);
  __syncthreads();
  double acc = in[tid & 1023];
  long long t0 = clock64();
  if (tid < lanes) {
    // (a) register-only chain
    double x = in[3];
    for (int k = 0; k < n; ++k) { acc += x; x *= 1.0000001; }
  }
  long long t1 = clock64();
  double acc2 = acc;
  if (tid < lanes) {
    // (b) chain fed from LDS pairs, 4 loads in flight (the replica's loop shape)
    double2 t[4];
    for (int j = 0; j < 4; ++j) t[j] = buf[j];
    for (int k = 0; k < n / 2; k += 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double2 c = t[j];
        t[j] = buf[(k + 4 + j) & 4095];
        acc2 += c.x;
        acc2 += c.y;
      }
    }
  }
  long long t2 = clock64();
  if (tid == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; }
  out[tid] = acc + acc2;
}

int main() {
  const int n = 1 << 16;
  double *in, *out; long long *cyc;
  hipMalloc(&in, 1024 * 8); hipMalloc(&out, 1024 * 8); hipMalloc(&cyc, 16);
  double h[1024]; for (int i = 0; i < 1024; ++i) h[i] = 1.0 + i * 1e-3;
  hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
  for (int lanes : {1, 3, 64}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, in, out, cyc, n, lanes);
      long long c[2]; hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
      if (rep) printf("lanes %2d: register chain %.2f clocks/add (clock64 units), LDS-fed chain %.2f\n", lanes,
                      (double)c[0] / n, (double)c[1] / n);
    }
  }
  return 0;
}
