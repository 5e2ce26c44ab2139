// rows_probe.hip -- experiment, not product code: the HBM rate of the x-pass
// access pattern of the mass inverse (mass3_rows_kernel) with the compute
// removed.  Each wave owns R consecutive rows of length LEN doubles (x lines)
// and copies them visit by visit, W doubles of every row per visit, through
// registers (dwordx4 per lane, the DMA's lane -> (row, pair) map), one visit
// in flight ahead.  Prints GB/s (read + write) per (R, W).
//   hipcc -O3 --offload-arch=gfx950 tools/rows_probe.hip -o rows_probe && ./rows_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

using d2 = double __attribute__((ext_vector_type(2)));

template <int R, int W>
__global__ void __launch_bounds__(64) probe(const double *src, double *dst, int len, int64_t n_rows) {
  constexpr int PAIRS = W / 2, U = R * PAIRS / 64;  // dpairs per lane per visit
  const int lane = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  if (r0 >= n_rows) return;
  d2 a[U], b[U];
  auto load = [&](d2 (&v)[U], int base) {
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int u = q * 64 + lane, row = u / PAIRS, pair = u % PAIRS;
      v[q] = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(src + (r0 + row) * len + base + 2 * pair));
    }
  };
  auto store = [&](const d2 (&v)[U], int base) {
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int u = q * 64 + lane, row = u / PAIRS, pair = u % PAIRS;
      __builtin_nontemporal_store(v[q], reinterpret_cast<d2 *>(dst + (r0 + row) * len + base + 2 * pair));
    }
  };
  const int nv = len / W;
  load(a, 0);
  for (int v = 1; v < nv; v += 2) {
    load(b, v * W);
    store(a, (v - 1) * W);
    if (v + 1 < nv) load(a, (v + 1) * W);
    store(b, v * W);
  }
  if (nv % 2 == 1) store(a, (nv - 1) * W);
}

template <int R, int W>
void run(const double *src, double *dst, int len, int64_t n_rows) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned grid = (unsigned)((n_rows + R - 1) / R);
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((probe<R, W>), dim3(grid), dim3(64), 0, 0, src, dst, len, n_rows);
  hipEventRecord(e0);
  const int iters = 10;
  for (int it = 0; it < iters; ++it) hipLaunchKernelGGL((probe<R, W>), dim3(grid), dim3(64), 0, 0, src, dst, len, n_rows);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= iters;
  const double bytes = 2.0 * 8.0 * (double)len / W * W * n_rows;
  std::printf("{\"R\": %d, \"W\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", R, W, ms, bytes / (ms * 1e6));
  std::fflush(stdout);
}

int main() {
  const int len = 512;
  const int64_t n_rows = 512 * 512;
  double *src, *dst;
  if (hipMalloc(&src, sizeof(double) * len * n_rows) != hipSuccess) return 1;
  if (hipMalloc(&dst, sizeof(double) * len * n_rows) != hipSuccess) return 1;
  hipMemset(src, 0, sizeof(double) * len * n_rows);
  run<64, 16>(src, dst, len, n_rows);
  run<64, 32>(src, dst, len, n_rows);
  run<64, 64>(src, dst, len, n_rows);
  run<32, 64>(src, dst, len, n_rows);
  run<32, 128>(src, dst, len, n_rows);
  run<16, 128>(src, dst, len, n_rows);
  run<16, 256>(src, dst, len, n_rows);
  run<8, 512>(src, dst, len, n_rows);
  run<4, 512>(src, dst, len, n_rows);
  hipFree(src);
  hipFree(dst);
  return 0;
}
