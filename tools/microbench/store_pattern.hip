// Microbenchmark: write bandwidth of the v8 stencil's output pattern on gfx950.
// A 512^3 fp64 field (1.07 GB) is written by 256 workgroups of 512 threads
// (8 "consumer" waves):
//   mode 0: linear, 16 B per lane (grid-stride float4-style copy target)
//   mode 1: stencil tiles, 8 B per lane: workgroup = 64 x 32 (x, y) column x
//           a z-chunk of 256 planes; wave w stores rows 4w..4w+3 per plane
//           (lane = x, one 512-B row segment per store instruction)
//   mode 2: same tiles, 16 B per lane: lanes 0..31 of a wave cover the 64 x of
//           one row pair (two rows per store instruction)
//   mode 3: 128 x 16 tiles, 8 B per lane, two waves per 128-wide row
// Build: hipcc -O3 --offload-arch=gfx950 store_pattern.hip -o store_pattern
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

constexpr int N = 512;

__global__ void __launch_bounds__(512) k_linear(double2 *out, long n2) {
  for (long i = blockIdx.x * 512L + threadIdx.x; i < n2; i += (long)gridDim.x * 512)
    out[i] = make_double2((double)i, 1.0);
}

// tile 64 x 32, z-chunk 256: 8 x 16 tiles x 2 chunks = 256 workgroups
__global__ void __launch_bounds__(512) k_tile8(double *out) {
  const int b = blockIdx.x, tx = b % 8, ty = (b / 8) % 16, tz = b / 128;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = tx * 64 + lane;
  for (int z = tz * 256; z < tz * 256 + 256; ++z)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int y = ty * 32 + 4 * w + j;
      out[((long)z * N + y) * N + x] = (double)z + j;
    }
}

__global__ void __launch_bounds__(512) k_tile16(double2 *out) {
  const int b = blockIdx.x, tx = b % 8, ty = (b / 8) % 16, tz = b / 128;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x2 = tx * 32 + (lane & 31), dy = lane >> 5;  // 32 lanes cover 64 x
  for (int z = tz * 256; z < tz * 256 + 256; ++z)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int y = ty * 32 + 4 * w + 2 * j + dy;
      out[((long)z * N + y) * (N / 2) + x2] = make_double2((double)z, (double)j);
    }
}

// tile 128 x 16, z-chunk 256: 4 x 32 tiles x 2 chunks
__global__ void __launch_bounds__(512) k_tile8w(double *out) {
  const int b = blockIdx.x, tx = b % 4, ty = (b / 4) % 32, tz = b / 128;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = tx * 128 + (w & 1) * 64 + lane;
  for (int z = tz * 256; z < tz * 256 + 256; ++z)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int y = ty * 16 + 4 * (w >> 1) + j;
      out[((long)z * N + y) * N + x] = (double)z + j;
    }
}

int main() {
  const long n = (long)N * N * N;
  double *d;
  if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 4; ++mode) {
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k_linear, dim3(1024), dim3(512), 0, 0, (double2 *)d, n / 2);
      if (mode == 1) hipLaunchKernelGGL(k_tile8, dim3(256), dim3(512), 0, 0, d);
      if (mode == 2) hipLaunchKernelGGL(k_tile16, dim3(256), dim3(512), 0, 0, (double2 *)d);
      if (mode == 3) hipLaunchKernelGGL(k_tile8w, dim3(256), dim3(512), 0, 0, d);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (it > 0 && ms < best) best = ms;
    }
    printf("mode %d: %.3f ms  %.2f TB/s write\n", mode, best, n * 8.0 / best / 1e9);
  }
  hipFree(d);
  return 0;
}
