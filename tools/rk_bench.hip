// rk_bench -- streaming micro-benchmark of the RK stage update at C3 size
// (134 M doubles per vector): acc = acc + b k, Y = y + a k in several forms,
// plus a copy for the achievable bandwidth.  tools/rk_bench.hip, built by
//   hipcc -O3 --offload-arch=gfx950 -o lib/rk_bench tools/rk_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

using d2 = double __attribute__((ext_vector_type(2)));

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void __launch_bounds__(256) copy2(int64_t n2, const d2 *__restrict__ a, d2 *__restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

// MODE 0: plain d2; 1: NT loads of k; 2: NT loads of k + NT stores; 3: all NT
template <int MODE>
__global__ void __launch_bounds__(256) upd2(int64_t n2, double beta, const d2 *__restrict__ k, const d2 *acc_in,
                                            d2 *acc_out, double alpha, const d2 *__restrict__ y, d2 *__restrict__ Y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    const d2 ki = MODE >= 1 ? __builtin_nontemporal_load(k + i) : k[i];
    const d2 ai = MODE >= 3 ? __builtin_nontemporal_load(acc_in + i) : acc_in[i];
    const d2 yi = MODE >= 3 ? __builtin_nontemporal_load(y + i) : y[i];
    const d2 o = ai + beta * ki, q = yi + alpha * ki;
    if (MODE >= 2) {
      __builtin_nontemporal_store(o, acc_out + i);
      __builtin_nontemporal_store(q, Y + i);
    } else {
      acc_out[i] = o;
      Y[i] = q;
    }
  }
}

// 4 pairs per lane per iteration (loads first, then stores)
__global__ void __launch_bounds__(256) upd2_u4(int64_t n2, double beta, const d2 *__restrict__ k, const d2 *acc_in,
                                               d2 *acc_out, double alpha, const d2 *__restrict__ y,
                                               d2 *__restrict__ Y) {
  const int64_t step = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += 4 * step) {
    d2 kk[4], aa[4], yy[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * step;
      if (i < n2) {
        kk[u] = __builtin_nontemporal_load(k + i);
        aa[u] = acc_in[i];
        yy[u] = y[i];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * step;
      if (i < n2) {
        acc_out[i] = aa[u] + beta * kk[u];
        Y[i] = yy[u] + alpha * kk[u];
      }
    }
  }
}

int main() {
  const int64_t n = 512LL * 512 * 512, n2 = n / 2;
  double *k, *acc, *y, *Y, *c;
  for (double **p : {&k, &acc, &y, &Y, &c}) CK(hipMalloc(p, sizeof(double) * n));
  for (double *p : {k, acc, y, Y, c}) CK(hipMemset(p, 0, sizeof(double) * n));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char *name, double bytes, auto launch) -> int {
    for (int w = 0; w < 2; ++w) launch();
    CK(hipEventRecord(e0));
    const int it = 10;
    for (int r = 0; r < it; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    std::printf("%-28s %8.3f ms %7.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    return 0;
  };
  const double B5 = 40.0 * n, B2 = 16.0 * n;
  const d2 *K = (const d2 *)k, *A = (const d2 *)acc, *Yi = (const d2 *)y;
  d2 *Ao = (d2 *)acc, *Yo = (d2 *)Y;
  for (int64_t g : {(int64_t)4096, (int64_t)16384, (n2 + 255) / 256}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "copy g=%lld", (long long)g);
    time(nm, B2, [&] { hipLaunchKernelGGL(copy2, dim3(g), dim3(256), 0, 0, n2, K, (d2 *)c); });
    std::snprintf(nm, sizeof nm, "upd mode0 g=%lld", (long long)g);
    time(nm, B5, [&] { hipLaunchKernelGGL(upd2<0>, dim3(g), dim3(256), 0, 0, n2, 0.1, K, A, Ao, 0.2, Yi, Yo); });
    std::snprintf(nm, sizeof nm, "upd mode1 g=%lld", (long long)g);
    time(nm, B5, [&] { hipLaunchKernelGGL(upd2<1>, dim3(g), dim3(256), 0, 0, n2, 0.1, K, A, Ao, 0.2, Yi, Yo); });
    std::snprintf(nm, sizeof nm, "upd mode2 g=%lld", (long long)g);
    time(nm, B5, [&] { hipLaunchKernelGGL(upd2<2>, dim3(g), dim3(256), 0, 0, n2, 0.1, K, A, Ao, 0.2, Yi, Yo); });
    std::snprintf(nm, sizeof nm, "upd mode3 g=%lld", (long long)g);
    time(nm, B5, [&] { hipLaunchKernelGGL(upd2<3>, dim3(g), dim3(256), 0, 0, n2, 0.1, K, A, Ao, 0.2, Yi, Yo); });
    std::snprintf(nm, sizeof nm, "upd u4 g=%lld", (long long)g);
    time(nm, B5, [&] { hipLaunchKernelGGL(upd2_u4, dim3(g), dim3(256), 0, 0, n2, 0.1, K, A, Ao, 0.2, Yi, Yo); });
  }
  // acc_in != acc_out (stage 0: acc_in = y)
  time("upd mode0 stage0 (acc_in=y)", B5, [&] {
    hipLaunchKernelGGL(upd2<0>, dim3(4096), dim3(256), 0, 0, n2, 0.1, K, Yi, Ao, 0.2, Yi, Yo);
  });
  for (double *p : {k, acc, y, Y, c}) CK(hipFree(p));
  return 0;
}
