// Microbenchmark: can FP64 MFMA (v_mfma_f64_16x16x4_f64) and FP64 VALU FMA run
// concurrently on gfx950?  mode 0: all waves VALU; 1: all waves MFMA;
// 2: half the waves VALU, half MFMA (same workgroup -> same SIMDs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k(double *out, int iters, int mode, double s) {
  const int wave = threadIdx.x >> 6;
  const bool mf = (mode == 1) || (mode == 2 && (wave & 1));
  double r = 0.0;
  if (mf) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = s * threadIdx.x, b = s + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    r = c0[0] + c1[1] + c2[2] + c3[3];
  } else {
    double x[8];
    for (int j = 0; j < 8; ++j) x[j] = s * (threadIdx.x + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int rep = 0; rep < 8; ++rep)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fma(x[j], s, 1.0);
    }
    for (int j = 0; j < 8; ++j) r += x[j];
  }
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
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, iters, mode, 0.999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // flops: VALU wave: iters*64 fma*64 lanes*2 ; MFMA wave: iters*4*16*16*4*2
    const double waves = blocks * threads / 64.0;
    double vw = 0, mw = 0;
    if (mode == 0) vw = waves;
    if (mode == 1) mw = waves;
    if (mode == 2) { vw = waves / 2; mw = waves / 2; }
    const double vflop = vw * iters * 64.0 * 64 * 2, mflop = mw * iters * 4.0 * 1024 * 2;
    printf("mode %d: %.3f ms  VALU %.1f TF  MFMA %.1f TF  total %.1f TF\n", mode, ms, vflop / ms / 1e9,
           mflop / ms / 1e9, (vflop + mflop) / ms / 1e9);
  }
  return 0;
}
