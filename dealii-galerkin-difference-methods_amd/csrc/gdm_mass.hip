// gdm_mass.hip -- exact Kronecker mass inverse, v2 (replaces the CG + ILU/AMG
// solve of applications/advection/include/gdm/advection/problem.h:236-267 and
// applications/wave/include/gdm/wave/problem.h:471-502 on the uncut mesh).
//
// M^-1 = M_z^-1 (x) M_y^-1 (x) M_x^-1 is applied as three passes of batched
// banded-Cholesky line solves (M_d = L L^T, half-bandwidth p):
//   forward  w_i = (r_i - sum_k L(i, i-p+k) w_{i-p+k}) / L(i, i)
//   backward x_i = (w_i - sum_m L(i+m, i) x_{i+m}) / L(i, i)
//
// Strided lines (y, z): lane = one line, consecutive lanes = consecutive x, so
// every load / store instruction moves one contiguous 512-B row; the values
// of a line are fetched U positions ahead of the recurrence (register
// double-buffer), so the dependent FMA chain never waits on HBM latency.
//
// Contiguous lines (x): one wave owns 64 lines and walks them in chunks of U
// positions; a chunk (64 lines x U doubles) is loaded row-coalesced into LDS,
// each lane runs the recurrence over its line's U values in LDS, and the
// chunk is written back row-coalesced.  The next chunk's loads are issued
// before the current chunk is processed.
//
// The first pass reads the right-hand side and writes the result vector (no
// separate copy); the forward sweep stores w into the result, the backward
// sweep reads it back right away (mostly from L2 / the memory-side cache).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "gdm_kernels.h"

namespace gdmk {

namespace {

// factor rows: lrow[i * (P + 1) + k] = L(i, i - P + k), k = P is the diagonal;
// rows >= len are zero (backward sweep reads P rows past the end)
template <int P>
struct Chol {
  const double *__restrict__ lrow;
  const double *__restrict__ invd;
  __device__ __forceinline__ double fwd(int i, const double (&win)[P > 0 ? P : 1], double r) const {
    const double *L = lrow + (size_t)i * (P + 1);
    double s = r;
#pragma unroll
    for (int k = 0; k < P; ++k) s = fma(-L[k], win[k], s);
    return s * invd[i];
  }
  __device__ __forceinline__ double bwd(int i, const double (&win)[P > 0 ? P : 1], double w) const {
    double s = w;
#pragma unroll
    for (int m = 1; m <= P; ++m) s = fma(-lrow[(size_t)(i + m) * (P + 1) + (P - m)], win[m - 1], s);
    return s * invd[i];
  }
};

template <int P>
__device__ __forceinline__ void push_fwd(double (&win)[P], double s) {
#pragma unroll
  for (int k = 0; k < P - 1; ++k) win[k] = win[k + 1];
  win[P - 1] = s;
}
template <int P>
__device__ __forceinline__ void push_bwd(double (&win)[P], double s) {
#pragma unroll
  for (int m = P - 1; m > 0; --m) win[m] = win[m - 1];
  win[0] = s;
}

}  // namespace

// line l -> base = (l / A) * B + (l % A); consecutive l are consecutive addresses
template <int P, int U>
__global__ void __launch_bounds__(64) chol_strided_kernel(const double *src, double *dst, int len,
                                                          int64_t stride, int64_t n_lines, int64_t A, int64_t B,
                                                          const double *__restrict__ lrow,
                                                          const double *__restrict__ invd) {
  const Chol<P> ch{lrow, invd};
  for (int64_t l = (int64_t)blockIdx.x * 64 + threadIdx.x - threadIdx.x % 64; l < n_lines;
       l += (int64_t)gridDim.x * 64) {
    const int64_t line = l + threadIdx.x % 64;
    const bool on = line < n_lines;
    const int64_t base = on ? (line / A) * B + (line % A) : 0;
    double win[P];
    double cur[U], nxt[U];
    // ---- forward: src -> dst (w) ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = (on && u < len) ? src[base + (int64_t)u * stride] : 0.0;
    for (int i0 = 0; i0 < len; i0 += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + U + u;
        nxt[u] = (on && i < len) ? src[base + (int64_t)i * stride] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u;
        if (i < len) {
          const double s = ch.fwd(i, win, cur[u]);
          push_fwd<P>(win, s);
          if (on) dst[base + (int64_t)i * stride] = s;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
    // ---- backward: dst (w) -> dst (x) ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
    const int last = len - 1;
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = (on && last - u >= 0) ? dst[base + (int64_t)(last - u) * stride] : 0.0;
    for (int i0 = last; i0 >= 0; i0 -= U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 - U - u;
        nxt[u] = (on && i >= 0) ? dst[base + (int64_t)i * stride] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 - u;
        if (i >= 0) {
          const double s = ch.bwd(i, win, cur[u]);
          push_bwd<P>(win, s);
          if (on) dst[base + (int64_t)i * stride] = s;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
  }
}

// contiguous lines of length len: line l starts at l * len.  One wave per
// workgroup; chunk = 64 lines x U positions staged in LDS (row pitch U + 2).
template <int P, int U>
__global__ void __launch_bounds__(64) chol_rows_kernel(const double *src, double *dst, int len, int64_t n_lines,
                                                       int vec_ok, const double *__restrict__ lrow,
                                                       const double *__restrict__ invd) {
  static_assert(U % 2 == 0 && (64 * U / 2) % 64 == 0, "chunk geometry");
  constexpr int PITCH = U + 2;      // doubles; keeps 16-B alignment, spreads banks
  constexpr int NV = 64 * U / 2 / 64;  // 16-B vectors per lane per chunk
  __shared__ __attribute__((aligned(16))) double tile[64 * PITCH];
  const Chol<P> ch{lrow, invd};
  const int lane = threadIdx.x;  // vec_ok: every row start is 16-B aligned (host-checked)
  for (int64_t l0 = (int64_t)blockIdx.x * 64; l0 < n_lines; l0 += (int64_t)gridDim.x * 64) {
    const int nl = (int)min<int64_t>(64, n_lines - l0);
    // element e of a chunk: line e / (U/2), vector (e % (U/2)) -> positions 2v, 2v+1
    auto load_chunk = [&](const double *from, int i0, double2 (&r)[NV]) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int e = q * 64 + lane, ln = e / (U / 2), v = e % (U / 2);
        const int i = i0 + 2 * v;
        double2 val = make_double2(0.0, 0.0);
        if (ln < nl && i >= 0 && i < len) {
          const double *p = from + (l0 + ln) * (int64_t)len + i;
          if (vec_ok && i + 1 < len)
            val = *reinterpret_cast<const double2 *>(p);
          else {
            val.x = p[0];
            val.y = i + 1 < len ? p[1] : 0.0;
          }
        }
        r[q] = val;
      }
    };
    auto put_lds = [&](const double2 (&r)[NV]) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int e = q * 64 + lane, ln = e / (U / 2), v = e % (U / 2);
        *reinterpret_cast<double2 *>(&tile[ln * PITCH + 2 * v]) = r[q];
      }
    };
    auto store_chunk = [&](int i0) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int e = q * 64 + lane, ln = e / (U / 2), v = e % (U / 2);
        const int i = i0 + 2 * v;
        if (ln < nl && i >= 0 && i < len) {
          const double2 val = *reinterpret_cast<const double2 *>(&tile[ln * PITCH + 2 * v]);
          double *p = dst + (l0 + ln) * (int64_t)len + i;
          if (vec_ok && i + 1 < len)
            *reinterpret_cast<double2 *>(p) = val;
          else {
            p[0] = val.x;
            if (i + 1 < len) p[1] = val.y;
          }
        }
      }
    };
    double win[P];
    double2 cur[NV], nxt[NV];
    // ---- forward: chunks [i0, i0 + U) ascending ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
    load_chunk(src, 0, cur);
    for (int i0 = 0; i0 < len; i0 += U) {
      load_chunk(src, i0 + U, nxt);
      __syncthreads();  // previous chunk's stores have read the tile
      put_lds(cur);
      __syncthreads();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u;
        if (i < len) {
          const double s = ch.fwd(i, win, tile[lane * PITCH + u]);
          push_fwd<P>(win, s);
          tile[lane * PITCH + u] = s;
        }
      }
      __syncthreads();
      store_chunk(i0);
#pragma unroll
      for (int q = 0; q < NV; ++q) cur[q] = nxt[q];
    }
    // ---- backward: chunks [i0, i0 + U) descending ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
    const int c_last = ((len - 1) / U) * U;
    __syncthreads();
    load_chunk(dst, c_last, cur);
    for (int i0 = c_last; i0 >= 0; i0 -= U) {
      load_chunk(dst, i0 - U, nxt);
      __syncthreads();
      put_lds(cur);
      __syncthreads();
#pragma unroll
      for (int u = U - 1; u >= 0; --u) {
        const int i = i0 + u;
        if (i < len) {
          const double s = ch.bwd(i, win, tile[lane * PITCH + u]);
          push_bwd<P>(win, s);
          tile[lane * PITCH + u] = s;
        }
      }
      __syncthreads();
      store_chunk(i0);
#pragma unroll
      for (int q = 0; q < NV; ++q) cur[q] = nxt[q];
    }
    __syncthreads();
  }
}

namespace {

template <int P>
hipError_t launch_mass_lines_p(int dir_kind, const double *src, double *dst, int len, int64_t stride, int64_t n_lines,
                               int64_t A, int64_t B, const double *lrow, const double *invd, int max_wgs,
                               hipStream_t st) {
  const int64_t groups = (n_lines + 63) / 64;
  const unsigned grid = (unsigned)(max_wgs > 0 ? std::min<int64_t>(groups, max_wgs) : groups);
  const int vec = (len % 2 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(dst) & 15) == 0) ? 1 : 0;
  // x chunk width: 16 positions (one 128-B line per row; measured 1.15 vs 1.30 ms for 8 at 512^3), GDM_MASS_XU=8
  static const int xu = [] { const char *e = std::getenv("GDM_MASS_XU"); return e ? std::atoi(e) : 16; }();
  if (dir_kind == 0 && xu == 16)
    hipLaunchKernelGGL((chol_rows_kernel<P, 16>), dim3(grid), dim3(64), 0, st, src, dst, len, n_lines, vec, lrow,
                       invd);
  else if (dir_kind == 0)
    hipLaunchKernelGGL((chol_rows_kernel<P, 8>), dim3(grid), dim3(64), 0, st, src, dst, len, n_lines, vec, lrow,
                       invd);
  else
    hipLaunchKernelGGL((chol_strided_kernel<P, 8>), dim3(grid), dim3(64), 0, st, src, dst, len, stride, n_lines, A,
                       B, lrow, invd);
  return hipGetLastError();
}

}  // namespace

}  // namespace gdmk

// dir_kind 0: contiguous lines (line l at l * len, stride 1);
// dir_kind 1: strided lines, base = (l / A) * B + (l % A), step `stride`.
// src may equal dst.  max_wgs > 0 caps the grid (lines are walked grid-stride).
extern "C" hipError_t gdmk_launch_mass_lines(int p, int dir_kind, const double *src, double *dst, int len,
                                            int64_t stride, int64_t n_lines, int64_t A, int64_t B,
                                            const double *lrow, const double *inv_diag, int max_wgs,
                                            hipStream_t st) {
  using namespace gdmk;
  if (n_lines <= 0 || len <= 0) return hipSuccess;
  switch (p) {
    case 1: return launch_mass_lines_p<1>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 3: return launch_mass_lines_p<3>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 5: return launch_mass_lines_p<5>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 7: return launch_mass_lines_p<7>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 9: return launch_mass_lines_p<9>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    default: return hipErrorInvalidValue;
  }
}
