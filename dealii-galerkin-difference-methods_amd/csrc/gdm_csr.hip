// gdm_csr.hip -- assembled sparse matrices on the device (include/gdm_hip.h,
// "Assembled sparse matrices"): the irregular-stencil CG matvec of the cut-cell
// Poisson prototype (prototypes/cut_poisson_01_gdm.cc:148-335)
// and the triplet files of applications/wave/wave-ev.cc:93-127 (§8 f2).
//
// Layout in HBM: CSR with int64 row pointers, uint32 column indices (the
// reference's unsigned int DoF indices) and fp64 values -- 12 B per stored
// entry, the whole matrix streamed once per vmult.
//
// SpMV: K lanes of a 64-wide wavefront per row (K chosen from the mean row
// length), entries and columns read with non-temporal loads so that the L2
// keeps the gathered source vector, lane sums combined with xor shuffles.
// Blocks are remapped so that each XCD walks one contiguous range of rows: the
// (2p+1)^d-point stencil rows then re-use source-vector lines in their own L2.
//
// CG (SolverCG + ReductionControl, deal.II semantics as restated in
// oracle/gdm_oracle.c:gdmo_cg): the scalars (r.r, r.z, p.Ap, alpha, beta) stay
// in device memory, the dot products are fused into the passes that produce
// their operands (p.Ap into the SpMV, r.r and r.D^-1 r into the x/r update),
// and the host reads one double per iteration for the convergence test.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gdm_hip.h"

int gdm_internal_set_error(int code, const char *msg);  // gdm_capi.cpp

namespace {

constexpr int CSR_BLOCK = 256;
constexpr int RED_BLOCK = 1024;
// device scalar slots of the CG
// r.z of iteration k (k = 0: initial residual) lives in S_GH + (k & 1).  No
// kernel reads a slot it writes: a uniform read may be served by the scalar
// cache and then observe the same wave's later vector store to that address
// (the round-1 CG defect, gh_old == gh after an iteration).
enum { S_RR = 0, S_GH = 1, S_PAP = 3, S_N = 8 };

int fail(int code, const std::string &msg) { return gdm_internal_set_error(code, msg.c_str()); }

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  // hardware dispatches block b to XCD b % 8; give XCD x the contiguous range
  // [x * q, (x + 1) * q) of logical blocks (the tail nb % 8 blocks keep their id)
  const int64_t q = nb / 8;
  if (b >= 8 * q) return b;
  return (b % 8) * q + b / 8;
}

// sum over the block of v (CSR_BLOCK threads) -> returned on thread 0
__device__ __forceinline__ double block_sum(double v, double *sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
  if (l == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x / 64); ++i) s += sh[i];
  return s;
}

// y = A x            (mode 0)
// y = b - A x        (mode 1, residual; b = y_in)
// also partial[blk] = sum x[row] * y[row] over the block's rows when partial != NULL (square A)
template <int K>
__global__ void __launch_bounds__(CSR_BLOCK) csr_spmv_kernel(int64_t n_rows, const int64_t *__restrict__ rp,
                                                             const uint32_t *__restrict__ ci,
                                                             const double *__restrict__ v,
                                                             const double *__restrict__ x,
                                                             const double *__restrict__ b, double *__restrict__ y,
                                                             double *__restrict__ partial) {
  constexpr int RPB = CSR_BLOCK / K;
  __shared__ double sh[CSR_BLOCK / 64];
  const int64_t blk = xcd_block(blockIdx.x, gridDim.x);
  const int g = threadIdx.x / K, l = threadIdx.x % K;
  const int64_t row = blk * RPB + g;
  double s = 0.0;
  if (row < n_rows) {
    const int64_t e = rp[row + 1];
    for (int64_t k = rp[row] + l; k < e; k += K)
      s += __builtin_nontemporal_load(v + k) * x[__builtin_nontemporal_load(ci + k)];
  }
#pragma unroll
  for (int o = K / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, K);
  double d = 0.0;
  if (row < n_rows && l == 0) {
    if (b) s = b[row] - s;
    y[row] = s;
    d = x[row] * s;
  }
  if (partial) {
    const double t = block_sum(d, sh);
    if (threadIdx.x == 0) partial[blk] = t;
  }
}

// Row-block ("CSR-stream") SpMV for matrices whose row lengths vary (the cut
// Poisson system of config 5: rows of (2p+1)^2 entries inside the domain, a
// single diagonal outside): block b owns rows [rb[b], rb[b+1]) holding at most
// CSR_NZB entries (or one longer row).  The block's products v[k] x[ci[k]] are
// computed with coalesced loads over k into LDS, then thread t sums row t's
// products in column order (deterministic); a single long row is reduced by the
// whole block.  Same outputs / partials as csr_spmv_kernel.
constexpr int CSR_NZB = 1024;

__global__ void __launch_bounds__(CSR_BLOCK) csr_rowblock_kernel(const int64_t *__restrict__ rb, int64_t n_blocks,
                                                                 const int64_t *__restrict__ rp,
                                                                 const uint32_t *__restrict__ ci,
                                                                 const double *__restrict__ v,
                                                                 const double *__restrict__ x,
                                                                 const double *__restrict__ b, double *__restrict__ y,
                                                                 double *__restrict__ partial) {
  __shared__ double prod[CSR_NZB];
  __shared__ double sh[CSR_BLOCK / 64];
  const int64_t blk = xcd_block(blockIdx.x, gridDim.x);
  const int64_t r0 = rb[blk], r1 = rb[blk + 1];
  const int64_t k0 = rp[r0], k1 = rp[r1];
  double d = 0.0;
  if (r1 - r0 == 1 && k1 - k0 > CSR_NZB) {
    // one long row: block-strided products + block reduction (thread 0 writes)
    double s = 0.0;
    for (int64_t k = k0 + threadIdx.x; k < k1; k += CSR_BLOCK)
      s += __builtin_nontemporal_load(v + k) * x[__builtin_nontemporal_load(ci + k)];
    s = block_sum(s, sh);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (b) s = b[r0] - s;
      y[r0] = s;
      d = x[r0] * s;
    }
  } else {
    const int nz = (int)(k1 - k0);
    for (int k = threadIdx.x; k < nz; k += CSR_BLOCK)
      prod[k] = __builtin_nontemporal_load(v + k0 + k) * x[__builtin_nontemporal_load(ci + k0 + k)];
    __syncthreads();
    const int64_t row = r0 + threadIdx.x;
    if (row < r1) {
      const int a = (int)(rp[row] - k0), e = (int)(rp[row + 1] - k0);
      double s = 0.0;
      for (int k = a; k < e; ++k) s += prod[k];
      if (b) s = b[row] - s;
      y[row] = s;
      d = x[row] * s;
    }
  }
  if (partial) {
    const double t = block_sum(d, sh);
    if (threadIdx.x == 0) partial[blk] = t;
  }
}

// deterministic sum of nparts partials (stride 1) of `nval` arrays laid out
// back to back (part[j * nparts + i]); results are written, never read:
//   S[slot0] = sum 0, S[slot1] = sum 1 (nval == 2)
__global__ void __launch_bounds__(RED_BLOCK) cg_reduce_kernel(const double *__restrict__ part, int64_t nparts,
                                                              int nval, int slot0, int slot1,
                                                              double *__restrict__ S) {
  __shared__ double sh[RED_BLOCK / 64];
  double r[2] = {0.0, 0.0};
  for (int j = 0; j < nval; ++j) {
    double a = 0.0;
    for (int64_t i = threadIdx.x; i < nparts; i += RED_BLOCK) a += part[j * nparts + i];
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (threadIdx.x % 64 == 0) sh[threadIdx.x / 64] = a;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < RED_BLOCK / 64; ++i) t += sh[i];
    r[j] = t;
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  S[slot0] = r[0];
  if (nval > 1) S[slot1] = r[1];
}

// partials of r.r and r.(dinv r) (dinv NULL = identity)
__global__ void __launch_bounds__(CSR_BLOCK) cg_init_kernel(int64_t n, const double *__restrict__ r,
                                                            const double *__restrict__ dinv,
                                                            double *__restrict__ part, int64_t nparts) {
  __shared__ double sh[CSR_BLOCK / 64];
  const int64_t i = (int64_t)blockIdx.x * CSR_BLOCK + threadIdx.x;
  double rr = 0.0, rz = 0.0;
  if (i < n) {
    const double ri = r[i];
    rr = ri * ri;
    rz = dinv ? ri * dinv[i] * ri : rr;
  }
  const double a = block_sum(rr, sh);
  __syncthreads();
  const double c = block_sum(rz, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[nparts + blockIdx.x] = c;
  }
}

// iteration it: p = z + beta p (it == 1: p = z), z = dinv r,
// beta = gh(it - 1) / gh(it - 2)
__global__ void __launch_bounds__(CSR_BLOCK) cg_dir_kernel(int64_t n, const double *__restrict__ r,
                                                           const double *__restrict__ dinv, double *__restrict__ p,
                                                           const double *__restrict__ S, int it) {
  const int64_t i = (int64_t)blockIdx.x * CSR_BLOCK + threadIdx.x;
  if (i >= n) return;
  const double z = dinv ? dinv[i] * r[i] : r[i];
  p[i] = it == 1 ? z : z + (S[S_GH + ((it - 1) & 1)] / S[S_GH + (it & 1)]) * p[i];
}

// iteration it: x += alpha p ; r -= alpha q with alpha = gh(it - 1) / p.Ap ;
// partials of r.r and r.z.  Grid-stride over a fixed grid (CG_GRID blocks at
// most): few partials for cg_reduce_kernel, a fixed summation order.
constexpr int CG_GRID = 2048;
__global__ void __launch_bounds__(CSR_BLOCK) cg_update_kernel(int64_t n, double *__restrict__ x,
                                                              double *__restrict__ r, const double *__restrict__ p,
                                                              const double *__restrict__ q,
                                                              const double *__restrict__ dinv,
                                                              const double *__restrict__ S, int it,
                                                              double *__restrict__ part, int64_t nparts) {
  __shared__ double sh[CSR_BLOCK / 64];
  double rr = 0.0, rz = 0.0;
  const double alpha = S[S_GH + ((it - 1) & 1)] / S[S_PAP];
  for (int64_t i = (int64_t)blockIdx.x * CSR_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * CSR_BLOCK) {
    x[i] += alpha * p[i];
    const double ri = r[i] - alpha * q[i];
    r[i] = ri;
    rr += ri * ri;
    rz += dinv ? ri * dinv[i] * ri : ri * ri;
  }
  const double a = block_sum(rr, sh);
  __syncthreads();
  const double c = block_sum(rz, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[nparts + blockIdx.x] = c;
  }
}

// partials of p.q (q = A p), grid-stride like cg_update_kernel
__global__ void __launch_bounds__(CSR_BLOCK) cg_pap_kernel(int64_t n, const double *__restrict__ p,
                                                           const double *__restrict__ q, double *__restrict__ part) {
  __shared__ double sh[CSR_BLOCK / 64];
  double d = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * CSR_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * CSR_BLOCK)
    d += p[i] * q[i];
  const double t = block_sum(d, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// structural checks of a device CSR: row_ptr non-decreasing, cols < n_cols;
// any violation stores 1 into *bad (plain stores, all writers store the same value)
__global__ void __launch_bounds__(CSR_BLOCK) csr_validate_kernel(int64_t n_rows, int64_t nnz, int64_t n_cols,
                                                                 const int64_t *__restrict__ rp,
                                                                 const uint32_t *__restrict__ ci,
                                                                 int *__restrict__ bad) {
  const int64_t stride = (int64_t)gridDim.x * CSR_BLOCK, work = n_rows > nnz ? n_rows : nnz;
  for (int64_t i = (int64_t)blockIdx.x * CSR_BLOCK + threadIdx.x; i < work; i += stride) {
    if (i < n_rows && rp[i] > rp[i + 1]) *bad = 1;
    if (i < nnz && (int64_t)ci[i] >= n_cols) *bad = 1;
  }
}

// dinv[row] = 1 / A(row, row) (1 when the diagonal is absent or zero)
__global__ void __launch_bounds__(CSR_BLOCK) csr_diag_inv_kernel(int64_t n, const int64_t *__restrict__ rp,
                                                                 const uint32_t *__restrict__ ci,
                                                                 const double *__restrict__ v,
                                                                 double *__restrict__ dinv) {
  const int64_t i = (int64_t)blockIdx.x * CSR_BLOCK + threadIdx.x;
  if (i >= n) return;
  double d = 1.0;
  for (int64_t k = rp[i]; k < rp[i + 1]; ++k)
    if ((int64_t)ci[k] == i && v[k] != 0.0) d = 1.0 / v[k];
  dinv[i] = d;
}

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace

struct gdm_csr {
  int device = 0;
  hipStream_t own_stream = nullptr, stream = nullptr;
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  int64_t *rp = nullptr;
  uint32_t *ci = nullptr;
  double *v = nullptr;
  int K = 16;
  // row blocks of csr_rowblock_kernel (mode 1): rb[0..n_blocks]
  int mode = 0;
  int64_t *rb = nullptr, n_blocks = 0;
  // CG work space (allocated on first use)
  double *r = nullptr, *p = nullptr, *q = nullptr, *dinv = nullptr, *part = nullptr, *S = nullptr;
  double *S_host = nullptr;  // pinned
  int64_t nparts = 0;
};

namespace {

int pick_lanes(int64_t n_rows, int64_t nnz) {
  const double avg = n_rows > 0 ? double(nnz) / double(n_rows) : 0.0;
  if (avg < 6) return 4;
  if (avg < 12) return 8;
  if (avg < 96) return 16;
  if (avg < 192) return 32;
  return 64;
}

hipError_t launch_spmv(const gdm_csr *A, const double *x, const double *b, double *y, double *partial) {
  if (A->n_rows == 0) return hipSuccess;
  if (A->mode == 1) {
    csr_rowblock_kernel<<<(unsigned)A->n_blocks, CSR_BLOCK, 0, A->stream>>>(A->rb, A->n_blocks, A->rp, A->ci, A->v,
                                                                            x, b, y, partial);
    return hipGetLastError();
  }
  const int64_t rpb = CSR_BLOCK / A->K;
  const dim3 grid((unsigned)cdiv(A->n_rows, rpb));
  switch (A->K) {
#define GDM_SPMV_CASE(KK)                                                                                   \
  case KK:                                                                                                  \
    csr_spmv_kernel<KK><<<grid, CSR_BLOCK, 0, A->stream>>>(A->n_rows, A->rp, A->ci, A->v, x, b, y, partial); \
    break;
    GDM_SPMV_CASE(2)
    GDM_SPMV_CASE(4)
    GDM_SPMV_CASE(8)
    GDM_SPMV_CASE(16)
    GDM_SPMV_CASE(32)
    GDM_SPMV_CASE(64)
#undef GDM_SPMV_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

void free_all(gdm_csr *A) {
  (void)hipSetDevice(A->device);
  for (void *ptr : {(void *)A->rp, (void *)A->ci, (void *)A->v, (void *)A->r, (void *)A->p, (void *)A->q,
                    (void *)A->dinv, (void *)A->part, (void *)A->S, (void *)A->rb})
    if (ptr) (void)hipFree(ptr);
  if (A->S_host) (void)hipHostFree(A->S_host);
  if (A->own_stream) (void)hipStreamDestroy(A->own_stream);
}

void validate_host(int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *rp, const uint32_t *ci) {
  if (rp[0] != 0 || rp[n_rows] != nnz) throw std::invalid_argument("row_ptr[0] != 0 or row_ptr[n_rows] != nnz");
  for (int64_t i = 0; i < n_rows; ++i)
    if (rp[i] > rp[i + 1]) throw std::invalid_argument("row_ptr is not non-decreasing");
  for (int64_t k = 0; k < nnz; ++k)
    if ((int64_t)ci[k] >= n_cols) throw std::invalid_argument("column index >= n_cols");
}

#define GDM_GUARD_BEGIN try {
#define GDM_GUARD_END                                                                 \
  }                                                                                   \
  catch (const HipError &e) { return fail(GDM_ERR_HIP, e.what()); }                   \
  catch (const std::bad_alloc &) { return fail(GDM_ERR_NOMEM, "out of host memory"); } \
  catch (const std::invalid_argument &e) { return fail(GDM_ERR_ARG, e.what()); }      \
  catch (const std::exception &e) { return fail(GDM_ERR_STATE, e.what()); }

// CSR from triplets: rows ascending, columns ascending within a row, duplicates summed
void triplets_to_csr(std::vector<uint32_t> &rows, std::vector<uint32_t> &cols, std::vector<double> &vals,
                     int64_t &n_rows, int64_t &n_cols, std::vector<int64_t> &rp, std::vector<uint32_t> &ci,
                     std::vector<double> &v) {
  n_rows = 0;
  n_cols = 0;
  for (size_t i = 0; i < rows.size(); ++i) {
    n_rows = std::max<int64_t>(n_rows, (int64_t)rows[i] + 1);
    n_cols = std::max<int64_t>(n_cols, (int64_t)cols[i] + 1);
  }
  std::vector<int64_t> cnt(n_rows + 1, 0);
  for (uint32_t r : rows) ++cnt[r + 1];
  for (int64_t i = 0; i < n_rows; ++i) cnt[i + 1] += cnt[i];
  std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
  std::vector<uint32_t> c2(rows.size());
  std::vector<double> v2(rows.size());
  for (size_t i = 0; i < rows.size(); ++i) {
    const int64_t k = pos[rows[i]]++;
    c2[k] = cols[i];
    v2[k] = vals[i];
  }
  rp.assign(n_rows + 1, 0);
  ci.clear();
  v.clear();
  ci.reserve(c2.size());
  v.reserve(c2.size());
  std::vector<std::pair<uint32_t, double>> row;
  for (int64_t r = 0; r < n_rows; ++r) {
    row.clear();
    for (int64_t k = cnt[r]; k < cnt[r + 1]; ++k) row.emplace_back(c2[k], v2[k]);
    std::stable_sort(row.begin(), row.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    for (size_t k = 0; k < row.size(); ++k) {
      if (!ci.empty() && (int64_t)ci.size() > rp[r] && ci.back() == row[k].first)
        v.back() += row[k].second;
      else {
        ci.push_back(row[k].first);
        v.push_back(row[k].second);
      }
    }
    rp[r + 1] = (int64_t)ci.size();
  }
}

int create_impl(int device, int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *rp, const uint32_t *ci,
                const double *v, int src_is_device, gdm_csr **out) {
  gdm_csr *A = new gdm_csr();
  try {
    A->device = device;
    A->n_rows = n_rows;
    A->n_cols = n_cols;
    A->nnz = nnz;
    A->K = pick_lanes(n_rows, nnz);
    hip_check(hipSetDevice(device), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&A->own_stream, hipStreamNonBlocking), "hipStreamCreate");
    A->stream = A->own_stream;
    hip_check(hipMalloc(&A->rp, sizeof(int64_t) * (n_rows + 1)), "hipMalloc row_ptr");
    hip_check(hipMalloc(&A->ci, sizeof(uint32_t) * std::max<int64_t>(nnz, 1)), "hipMalloc cols");
    hip_check(hipMalloc(&A->v, sizeof(double) * std::max<int64_t>(nnz, 1)), "hipMalloc vals");
    const hipMemcpyKind kind = src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (!src_is_device) validate_host(n_rows, n_cols, nnz, rp, ci);
    // device sources may still be written by work queued on other streams (the
    // caller's fills and conversions): this setup call orders after all of it
    if (src_is_device) hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipMemcpyAsync(A->rp, rp, sizeof(int64_t) * (n_rows + 1), kind, A->stream), "copy row_ptr");
    if (nnz > 0) {
      hip_check(hipMemcpyAsync(A->ci, ci, sizeof(uint32_t) * nnz, kind, A->stream), "copy cols");
      hip_check(hipMemcpyAsync(A->v, v, sizeof(double) * nnz, kind, A->stream), "copy vals");
    }
    if (src_is_device) {
      int64_t ends[2];
      hip_check(hipMemcpyAsync(&ends[0], A->rp, sizeof(int64_t), hipMemcpyDeviceToHost, A->stream), "d2h");
      hip_check(hipMemcpyAsync(&ends[1], A->rp + n_rows, sizeof(int64_t), hipMemcpyDeviceToHost, A->stream), "d2h");
      int *bad = nullptr;
      hip_check(hipMalloc(&bad, sizeof(int)), "hipMalloc");
      hip_check(hipMemsetAsync(bad, 0, sizeof(int), A->stream), "memset");
      const int64_t work = std::max(n_rows, nnz);
      const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, CSR_BLOCK), 8192));
      csr_validate_kernel<<<g, CSR_BLOCK, 0, A->stream>>>(n_rows, nnz, n_cols, A->rp, A->ci, bad);
      hip_check(hipGetLastError(), "validate launch");
      int hbad = 0;
      hip_check(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, A->stream), "d2h");
      hip_check(hipStreamSynchronize(A->stream), "sync");
      (void)hipFree(bad);
      if (ends[0] != 0 || ends[1] != nnz) throw std::invalid_argument("row_ptr[0] != 0 or row_ptr[n_rows] != nnz");
      if (hbad) throw std::invalid_argument("row_ptr decreasing or column index >= n_cols");
    }
    // row blocks for the row-block kernel: consecutive rows with at most
    // CSR_NZB entries and CSR_BLOCK rows per block (a longer row alone)
    std::vector<int64_t> hrp, rb;  // host staging: alive until the stream sync below
    if (n_rows > 0) {
      const int64_t *r = rp;
      if (src_is_device) {
        hrp.resize((size_t)n_rows + 1);
        hip_check(hipMemcpyAsync(hrp.data(), A->rp, sizeof(int64_t) * (n_rows + 1), hipMemcpyDeviceToHost, A->stream),
                  "d2h");
        hip_check(hipStreamSynchronize(A->stream), "sync");
        r = hrp.data();
      }
      int64_t row = 0;
      rb.push_back(0);
      while (row < n_rows) {
        int64_t e = row + 1;
        while (e < n_rows && e - row < CSR_BLOCK && r[e + 1] - r[row] <= CSR_NZB) ++e;
        rb.push_back(e);
        row = e;
      }
      A->n_blocks = (int64_t)rb.size() - 1;
      hip_check(hipMalloc(&A->rb, sizeof(int64_t) * rb.size()), "hipMalloc row blocks");
      hip_check(hipMemcpyAsync(A->rb, rb.data(), sizeof(int64_t) * rb.size(), hipMemcpyHostToDevice, A->stream),
                "copy row blocks");
      // the row-block kernel everywhere (measured on config 5: cut matrix with
      // rows of 49 and 1 entries 3.11 -> 1.62 ms, full 49-entry stencil
      // 3.97 -> 2.75 ms per SpMV)
      A->mode = 1;
    }
    hip_check(hipStreamSynchronize(A->stream), "sync");
  } catch (...) {
    free_all(A);
    delete A;
    throw;
  }
  *out = A;
  return GDM_OK;
}

void ensure_cg_space(gdm_csr *A, bool jacobi) {
  const int64_t n = A->n_rows;
  const int64_t nparts =
      std::max<int64_t>(cdiv(n, CSR_BLOCK), A->mode == 1 ? A->n_blocks : cdiv(n, CSR_BLOCK / A->K));
  if (!A->r) {
    hip_check(hipMalloc(&A->r, sizeof(double) * std::max<int64_t>(n, 1)), "hipMalloc r");
    hip_check(hipMalloc(&A->p, sizeof(double) * std::max<int64_t>(n, 1)), "hipMalloc p");
    hip_check(hipMalloc(&A->q, sizeof(double) * std::max<int64_t>(n, 1)), "hipMalloc q");
    hip_check(hipMalloc(&A->part, sizeof(double) * 2 * std::max<int64_t>(nparts, 1)), "hipMalloc partials");
    hip_check(hipMalloc(&A->S, sizeof(double) * S_N), "hipMalloc scalars");
    hip_check(hipHostMalloc(&A->S_host, sizeof(double) * S_N), "hipHostMalloc");
    A->nparts = nparts;
  }
  if (jacobi && !A->dinv) {
    hip_check(hipMalloc(&A->dinv, sizeof(double) * std::max<int64_t>(n, 1)), "hipMalloc dinv");
    if (n > 0) {
      csr_diag_inv_kernel<<<(unsigned)cdiv(n, CSR_BLOCK), CSR_BLOCK, 0, A->stream>>>(n, A->rp, A->ci, A->v,
                                                                                     A->dinv);
      hip_check(hipGetLastError(), "diag launch");
    }
  }
}

double read_scalar(gdm_csr *A, int slot) {
  hip_check(hipMemcpyAsync(A->S_host, A->S + slot, sizeof(double), hipMemcpyDeviceToHost, A->stream), "d2h");
  hip_check(hipStreamSynchronize(A->stream), "sync");
  return A->S_host[0];
}

}  // namespace

extern "C" {

int gdm_csr_create(int device, int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *row_ptr,
                   const uint32_t *cols, const double *vals, int src_is_device, gdm_csr **out) {
  if (!out || !row_ptr || (nnz > 0 && (!cols || !vals))) return fail(GDM_ERR_ARG, "NULL argument");
  if (n_rows < 0 || n_cols < 0 || nnz < 0 || n_cols > (int64_t)UINT32_MAX + 1 || n_rows >= (int64_t)1 << 40)
    return fail(GDM_ERR_ARG, "bad matrix size");
  *out = nullptr;
  GDM_GUARD_BEGIN
  return create_impl(device, n_rows, n_cols, nnz, row_ptr, cols, vals, src_is_device, out);
  GDM_GUARD_END
}

int gdm_csr_destroy(gdm_csr *A) {
  if (!A) return GDM_OK;
  free_all(A);
  delete A;
  return GDM_OK;
}

int gdm_csr_info(const gdm_csr *A, int64_t *n_rows, int64_t *n_cols, int64_t *nnz) {
  if (!A) return fail(GDM_ERR_ARG, "matrix is NULL");
  if (n_rows) *n_rows = A->n_rows;
  if (n_cols) *n_cols = A->n_cols;
  if (nnz) *nnz = A->nnz;
  return GDM_OK;
}

int gdm_csr_set_stream(gdm_csr *A, void *hip_stream) {
  if (!A) return fail(GDM_ERR_ARG, "matrix is NULL");
  A->stream = (hipStream_t)hip_stream;
  return GDM_OK;
}

int gdm_csr_download(const gdm_csr *A, int64_t *row_ptr_host, uint32_t *cols_host, double *vals_host) {
  if (!A || !row_ptr_host || (A->nnz > 0 && (!cols_host || !vals_host))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(A->device), "hipSetDevice");
  hip_check(hipMemcpyAsync(row_ptr_host, A->rp, sizeof(int64_t) * (A->n_rows + 1), hipMemcpyDeviceToHost,
                           A->stream),
            "d2h");
  if (A->nnz > 0) {
    hip_check(hipMemcpyAsync(cols_host, A->ci, sizeof(uint32_t) * A->nnz, hipMemcpyDeviceToHost, A->stream), "d2h");
    hip_check(hipMemcpyAsync(vals_host, A->v, sizeof(double) * A->nnz, hipMemcpyDeviceToHost, A->stream), "d2h");
  }
  hip_check(hipStreamSynchronize(A->stream), "sync");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_csr_vmult(gdm_csr *A, const double *src, double *dst) {
  if (!A || (A->n_rows > 0 && (!src || !dst))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(A->device), "hipSetDevice");
  hip_check(launch_spmv(A, src, nullptr, dst, nullptr), "spmv launch");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_csr_cg(gdm_csr *A, const double *b, double *x, int precond, int max_it, double abs_tol, double rel_tol,
               int *its_host, double *res_host) {
  if (!A || (A->n_rows > 0 && (!b || !x))) return fail(GDM_ERR_ARG, "NULL argument");
  if (A->n_rows != A->n_cols) return fail(GDM_ERR_ARG, "CG needs a square matrix");
  if (precond != 0 && precond != 1) return fail(GDM_ERR_ARG, "precond must be 0 (identity) or 1 (Jacobi)");
  if (max_it < 0) return fail(GDM_ERR_ARG, "max_it < 0");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(A->device), "hipSetDevice");
  const int64_t n = A->n_rows;
  int its = 0;
  double res = 0.0;
  if (n > 0) {
    ensure_cg_space(A, precond == 1);
    const double *dinv = precond == 1 ? A->dinv : nullptr;
    const unsigned gv = (unsigned)cdiv(n, CSR_BLOCK);
    const int64_t ns = A->mode == 1 ? A->n_blocks : cdiv(n, CSR_BLOCK / A->K);  // SpMV partials
    // r = b - A x ; r.r ; r.z
    hip_check(launch_spmv(A, x, b, A->r, nullptr), "spmv launch");
    cg_init_kernel<<<gv, CSR_BLOCK, 0, A->stream>>>(n, A->r, dinv, A->part, gv);
    cg_reduce_kernel<<<1, RED_BLOCK, 0, A->stream>>>(A->part, gv, 2, S_RR, S_GH, A->S);
    hip_check(hipGetLastError(), "cg init");
    res = std::sqrt(read_scalar(A, S_RR));
    const double tol = std::max(abs_tol, rel_tol * res);
    bool converged = res <= tol;
    // p.Ap and r.r / r.z from grid-stride kernels over gs <= CG_GRID blocks
    // (the per-row-block SpMV partials and one partial per 256 rows made the
    // single-block reductions 100 us each at config 5)
    const unsigned gs = (unsigned)std::min<int64_t>(CG_GRID, cdiv(n, CSR_BLOCK));
    (void)ns;
    while (!converged && its < max_it) {
      ++its;
      cg_dir_kernel<<<gv, CSR_BLOCK, 0, A->stream>>>(n, A->r, dinv, A->p, A->S, its);
      hip_check(launch_spmv(A, A->p, nullptr, A->q, nullptr), "spmv launch");
      cg_pap_kernel<<<gs, CSR_BLOCK, 0, A->stream>>>(n, A->p, A->q, A->part);
      cg_reduce_kernel<<<1, RED_BLOCK, 0, A->stream>>>(A->part, gs, 1, S_PAP, S_PAP, A->S);
      cg_update_kernel<<<gs, CSR_BLOCK, 0, A->stream>>>(n, x, A->r, A->p, A->q, dinv, A->S, its, A->part, gs);
      cg_reduce_kernel<<<1, RED_BLOCK, 0, A->stream>>>(A->part, gs, 2, S_RR, S_GH + (its & 1), A->S);
      hip_check(hipGetLastError(), "cg iteration");
      res = std::sqrt(read_scalar(A, S_RR));
      converged = res <= tol;
    }
    if (its_host) *its_host = its;
    if (res_host) *res_host = res;
    if (!converged) return fail(GDM_ERR_STATE, "SolverCG: no convergence within max_it iterations");
    return GDM_OK;
  }
  if (its_host) *its_host = 0;
  if (res_host) *res_host = 0.0;
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_csr_read_triplets(int device, const char *path, int binary, gdm_csr **out) {
  if (!path || !out) return fail(GDM_ERR_ARG, "NULL argument");
  *out = nullptr;
  GDM_GUARD_BEGIN
  FILE *f = std::fopen(path, binary ? "rb" : "r");
  if (!f) return fail(GDM_ERR_ARG, std::string("cannot open ") + path);
  std::vector<uint32_t> rows, cols;
  std::vector<double> vals;
  if (binary) {
    unsigned char rec[16];
    size_t got;
    while ((got = std::fread(rec, 1, 16, f)) == 16) {
      uint32_t r, c;
      double val;
      std::memcpy(&r, rec, 4);
      std::memcpy(&c, rec + 4, 4);
      std::memcpy(&val, rec + 8, 8);
      rows.push_back(r);
      cols.push_back(c);
      vals.push_back(val);
    }
    if (got != 0) {
      std::fclose(f);
      return fail(GDM_ERR_ARG, "truncated triplet record");
    }
  } else {
    unsigned long long r, c;
    double val;
    int k;
    while ((k = std::fscanf(f, "%llu %llu %lf", &r, &c, &val)) == 3) {
      if (r > UINT32_MAX || c > UINT32_MAX) {
        std::fclose(f);
        return fail(GDM_ERR_ARG, "index exceeds 32 bits");
      }
      rows.push_back((uint32_t)r);
      cols.push_back((uint32_t)c);
      vals.push_back(val);
    }
    if (k != EOF) {
      std::fclose(f);
      return fail(GDM_ERR_ARG, "malformed triplet line");
    }
  }
  std::fclose(f);
  int64_t n_rows, n_cols;
  std::vector<int64_t> rp;
  std::vector<uint32_t> ci;
  std::vector<double> v;
  triplets_to_csr(rows, cols, vals, n_rows, n_cols, rp, ci, v);
  // square matrices (every reference writer) keep n = max(rows, cols)
  const int64_t n = std::max(n_rows, n_cols);
  rp.resize(n + 1, rp.empty() ? 0 : rp.back());
  return create_impl(device, n, n, (int64_t)ci.size(), rp.data(), ci.data(), v.data(), 0, out);
  GDM_GUARD_END
}

int gdm_csr_write_triplets(const gdm_csr *A, const char *path, int binary) {
  if (!A || !path) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  std::vector<int64_t> rp(A->n_rows + 1);
  std::vector<uint32_t> ci(std::max<int64_t>(A->nnz, 1));
  std::vector<double> v(std::max<int64_t>(A->nnz, 1));
  int rc = gdm_csr_download(A, rp.data(), ci.data(), v.data());
  if (rc != GDM_OK) return rc;
  FILE *f = std::fopen(path, binary ? "wb" : "w");
  if (!f) return fail(GDM_ERR_ARG, std::string("cannot open ") + path);
  const bool square = A->n_rows == A->n_cols;
  auto put = [&](int64_t r, int64_t k) {
    const uint32_t row = (uint32_t)r, col = ci[k];
    if (binary) {
      std::fwrite(&row, 4, 1, f);
      std::fwrite(&col, 4, 1, f);
      std::fwrite(&v[k], 8, 1, f);
    } else {
      std::fprintf(f, "%u %u %.17g\n", row, col, v[k]);
    }
  };
  for (int64_t r = 0; r < A->n_rows; ++r) {
    // deal.II SparsityPattern order: the diagonal first in a square matrix's row
    if (square)
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
        if ((int64_t)ci[k] == r) put(r, k);
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
      if (!square || (int64_t)ci[k] != r) put(r, k);
  }
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  if (!ok) return fail(GDM_ERR_STATE, std::string("write error on ") + path);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_csr_time_vmult(gdm_csr *A, const double *src, double *dst, int n_iter, double *avg_ms_host) {
  if (!A || !avg_ms_host || n_iter <= 0) return fail(GDM_ERR_ARG, "bad argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(A->device), "hipSetDevice");
  hipEvent_t e0, e1;
  hip_check(hipEventCreate(&e0), "event");
  hip_check(hipEventCreate(&e1), "event");
  hip_check(hipEventRecord(e0, A->stream), "record");
  for (int i = 0; i < n_iter; ++i) hip_check(launch_spmv(A, src, nullptr, dst, nullptr), "spmv launch");
  hip_check(hipEventRecord(e1, A->stream), "record");
  hip_check(hipEventSynchronize(e1), "sync");
  float ms = 0.f;
  hip_check(hipEventElapsedTime(&ms, e0, e1), "elapsed");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *avg_ms_host = ms / n_iter;
  return GDM_OK;
  GDM_GUARD_END
}

}  // extern "C"
