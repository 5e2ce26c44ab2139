// gdm_band.hip -- device pieces of the cut-cell advection operator
// (gdm_capi.cpp, "Cut-cell advection"): the sparse correction / inflow
// products next to the fused stencil, and the exact banded Cholesky solve of
// the cut mass matrix (the SolverDirect branch of advection/problem.h:
// 236-267; the factor comes from gdm_cut_advection.cpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gdmk {

// y[i] += sum_k v[k] x[ci[k]] over row i (one thread per row; the cut
// corrections have <= (2p+3)^2 entries per row)
__global__ void __launch_bounds__(256) csr_accum_kernel(int64_t n_rows, const int64_t *__restrict__ rp,
                                                        const uint32_t *__restrict__ ci,
                                                        const double *__restrict__ v,
                                                        const double *__restrict__ x, double *__restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_rows; i += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int64_t k = rp[i]; k < rp[i + 1]; ++k) s = fma(v[k], x[ci[k]], s);
    y[i] += s;
  }
}

// y[rows[k]] = 0
__global__ void __launch_bounds__(256) zero_rows_kernel(int64_t n, const int64_t *__restrict__ rows,
                                                        double *__restrict__ y) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    y[rows[k]] = 0.0;
}

// x <- (L L^T)^-1 x, L banded lower triangular with half-bandwidth bw,
// row form L[i * (bw + 1) + k] = L(i, i - bw + k).  One workgroup: the rows
// are sequential, each row's bw-long dot product is spread over the block
// (wave shuffles + one LDS exchange per row).
constexpr int BAND_NT = 256;

__device__ __forceinline__ double block_sum(double s, double *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // the previous row's readers are done with red
  if ((threadIdx.x & 63) == 0) red[w] = s;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < BAND_NT / 64; ++k) t += red[k];
  return t;
}

__global__ void __launch_bounds__(BAND_NT) band_solve_kernel(int64_t n, int64_t bw, const double *__restrict__ L,
                                                             double *__restrict__ x) {
  __shared__ double red[BAND_NT / 64];
  const int64_t W = bw + 1;
  // forward: L y = x
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k0 = i - bw > 0 ? i - bw : 0;
    double s = 0.0;
    for (int64_t k = k0 + threadIdx.x; k < i; k += BAND_NT) s = fma(L[i * W + (k - i + bw)], x[k], s);
    s = block_sum(s, red);
    if (threadIdx.x == 0) x[i] = (x[i] - s) / L[i * W + bw];
    __syncthreads();
  }
  // backward: L^T z = y, row i of L^T = column i of L: L(k, i), k in (i, i + bw]
  for (int64_t i = n - 1; i >= 0; --i) {
    const int64_t k1 = i + bw < n - 1 ? i + bw : n - 1;
    double s = 0.0;
    for (int64_t k = i + 1 + threadIdx.x; k <= k1; k += BAND_NT) s = fma(L[k * W + (i - k + bw)], x[k], s);
    s = block_sum(s, red);
    if (threadIdx.x == 0) x[i] = (x[i] - s) / L[i * W + bw];
    __syncthreads();
  }
}

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_csr_accum(int64_t n_rows, const int64_t *rp, const uint32_t *ci, const double *v,
                                           const double *x, double *y, hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  const int64_t blocks = (n_rows + 255) / 256 < 4096 ? (n_rows + 255) / 256 : 4096;
  hipLaunchKernelGGL(gdmk::csr_accum_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n_rows, rp, ci, v, x, y);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_zero_rows(int64_t n, const int64_t *rows, double *y, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(gdmk::zero_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, rows, y);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_band_solve(int64_t n, int64_t bw, const double *L, double *x, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gdmk::band_solve_kernel, dim3(1), dim3(gdmk::BAND_NT), 0, st, n, bw, L, x);
  return hipGetLastError();
}
