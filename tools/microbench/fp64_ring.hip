// Microbenchmark: FP64 FMA issue rate of the v8 stencil consumer's z-scatter
// pattern on gfx950 -- a register ring acc[2p+1][R] += c_k E_j with the
// coefficients in SGPRs (v_fmac_f64 acc, s, v: two VGPR-pair operands) --
// against the one-operand chain of fp64_pipes.hip, 16 waves per CU.
//   mode 0: x = fma(x, s, 1)  (8 chains, one VGPR pair)
//   mode 1: ring of 11 x 4 accumulators, 44 FMAs per "plane" (+ 4 to move E)
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(256) k(double *out, int iters, const double *cs) {
  double r = 0.0;
  if (MODE == 0) {
    double x[8];
    const double s = cs[0];
    for (int j = 0; j < 8; ++j) x[j] = s * (threadIdx.x + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int rep = 0; rep < 6; ++rep)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], s, 1.0);
    }
    for (int j = 0; j < 8; ++j) r += x[j];
  } else {
    double c[11];
#pragma unroll
    for (int q = 0; q < 11; ++q) c[q] = cs[q];  // uniform: SGPRs
    double acc[11][4], E[4];
#pragma unroll
    for (int s = 0; s < 11; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[s][j] = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) E[j] = 0.001 * (threadIdx.x + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int pl = 0; pl < 11; ++pl) {
#pragma unroll
        for (int q = 0; q < 11; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[(pl + q) % 11][j] = fma(c[q], E[j], acc[(pl + q) % 11][j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) E[j] = fma(E[j], c[0], 1e-3);
      }
    }
#pragma unroll
    for (int s = 0; s < 11; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) r += acc[s][j];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  double *out, *cs;
  const int blocks = 256 * 4, threads = 256;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  hipMalloc(&cs, sizeof(double) * 16);
  double h[16];
  for (int i = 0; i < 16; ++i) h[i] = 0.999 - 0.01 * i;
  hipMemcpy(cs, h, sizeof(h), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    const int iters = mode == 0 ? 4000 : 400;
    auto launch = [&](int it) {
      if (mode == 0)
        hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, out, it, cs);
      else
        hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, out, it, cs);
    };
    launch(10);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      launch(iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double waves = blocks * threads / 64.0;
    const double fma_per_iter = mode == 0 ? 48.0 : 11.0 * 48.0;
    const double flop = waves * iters * fma_per_iter * 64 * 2;
    printf("mode %d: %.3f ms  FP64 %.1f TF\n", mode, best, flop / best / 1e9);
  }
  return 0;
}
