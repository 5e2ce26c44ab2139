// Microbenchmark: FP64 FMA throughput on gfx950 by number of VGPR-pair
// operands (the stencil's FMAs read two: v_fmac_f64 acc, s, v / v_fma_f64 d,
// v, s, v).  16 waves per CU, 8 independent chains per lane.
//   mode 0: x = fma(x, s, 1)       one VGPR pair
//   mode 1: x = fma(y, s, x)       two (y loop-invariant, like a stencil input)
//   mode 2: x = fma(y, z, x)       three
//   mode 3: mode 1 with y[j] in the same register bank parity as x[j] (adjacent pairs)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) k(double *out, int iters, int mode, double s) {
  double x[8], y[8], z[8];
  for (int j = 0; j < 8; ++j) {
    x[j] = s * (threadIdx.x + j);
    y[j] = s + j * threadIdx.x;
    z[j] = 1.0 + 0.5 * j;
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int rep = 0; rep < 8; ++rep) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (mode == 0) x[j] = fma(x[j], s, 1.0);
        else if (mode == 2) x[j] = fma(y[j], z[j], x[j]);
        else x[j] = fma(y[j], s, x[j]);
      }
      asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
    }
  }
  double r = 0.0;
  for (int j = 0; j < 8; ++j) r += x[j] + y[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  double *out;
  const int blocks = 256 * 4, threads = 256;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  const int iters = 4000;
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 10, mode, 0.999);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, iters, mode, 0.999);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double waves = blocks * threads / 64.0;
    const double flop = waves * iters * 64.0 * 64 * 2;
    printf("mode %d: %.3f ms  FP64 FMA %.1f TF\n", mode, best, flop / best / 1e9);
  }
  return 0;
}
