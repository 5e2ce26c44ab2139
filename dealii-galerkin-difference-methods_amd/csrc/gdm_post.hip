// gdm_post.hip -- postprocess on the device: error norms
// of a GDM field against a built-in analytic function.
//
// The reference computes, per locally owned cell, the field and the exact
// solution at the QGauss(p+1) points and accumulates
//   Linf = max |e|,  L1 = sum |e| JxW,  L2^2 = sum e^2 JxW
// (applications/advection/include/gdm/advection/problem.h:330-425, reduced
// with Utilities::MPI::max / sum), and integrate_difference stores the per-cell
// L2 error sqrt(sum_q e^2 JxW) (include/gdm/vector_tools.h:25-86).
//
// Device form: one work item = a row of up to CX cells along x at fixed
// (cell_y, cell_z).  The (p+1)^2 x-rows of the row's DoF box are staged in
// LDS, contracted with the y / z shape values into the (qy, qz) rows
// (sum factorisation), then four lanes per cell contract x, evaluate the exact
// function (separable sine tables per row, the cone pointwise) and reduce.
// Work items are grid-strided; per-workgroup partials are reduced by a second
// one-workgroup kernel in a fixed order (deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>

#include "gdm_post.h"

namespace gdmk {

namespace {

constexpr int CX = 64;   // cells per work item along x
constexpr int TPC = 4;   // lanes per cell in the point phase
constexpr int NT = CX * TPC;

__device__ __forceinline__ int category_d(int c, int p, int n) {
  const int half = p / 2;
  if (c < half) return c;
  if (c < n - half) return half;
  return p + c - n;
}

__device__ __forceinline__ int box_offset_d(int c, int p, int n) {
  const int half = p / 2;
  if (c < half) return 0;
  return min(n, c + half + 1) - p;
}

__device__ __forceinline__ double sine_1d(const BcFn &f, int e, double x, double t) {
  return sin(2.0 * M_PI * f.prm[3 + e] * (x - f.prm[e] * t) + f.prm[6 + e]);
}

}  // namespace

// LDS: A = row[NB2][NB1][W] (later w[NQ2][NQ1][W]) | B = tz[NQ2][NB1][W] |
//      S[NCAT][N1][N1] | fx[CX][N1] | fy[N1] | fz[N1] | cacc[TPC][CX] ; W = CX + P
template <int P, int DIM>
__global__ void __launch_bounds__(NT) error_norms_kernel(ErrGeom g, BcFn f, double t, const double *__restrict__ S,
                                                         const double *__restrict__ u, double *__restrict__ cell_err,
                                                         double *__restrict__ partial) {
  constexpr int N1 = P + 1, W = CX + P;
  constexpr int NB1 = DIM > 1 ? N1 : 1, NB2 = DIM > 2 ? N1 : 1;  // = quadrature points per direction
  constexpr int NCAT = P > 1 ? P : 1;
  extern __shared__ double lds[];
  double *A = lds;
  double *B = A + NB2 * NB1 * W;
  double *Sl = B + NB2 * NB1 * W;
  double *fx = Sl + NCAT * N1 * N1;
  double *fy = fx + CX * N1;
  double *fz = fy + N1;
  double *cacc = fz + N1;
  const int tid = threadIdx.x;
  for (int i = tid; i < NCAT * N1 * N1; i += NT) Sl[i] = S[i];
  double wq[N1];
#pragma unroll
  for (int q = 0; q < N1; ++q) wq[q] = g.wq[q];

  const int ncx = g.ce[0] - g.cb[0], ncy = g.ce[1] - g.cb[1], ncz = g.ce[2] - g.cb[2];
  const int chunks = (ncx + CX - 1) / CX;
  const int64_t n_items = (int64_t)chunks * ncy * ncz;
  double a_l1 = 0.0, a_l2 = 0.0, a_inf = 0.0;
  const int cl = tid % CX, grp = tid / CX;  // point phase: cell of the chunk, line group

  for (int64_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int chunk = (int)(item % chunks);
    const int64_t r = item / chunks;
    const int cy = g.cb[1] + (int)(r % ncy), cz = g.cb[2] + (int)(r / ncy);
    const int cx0 = g.cb[0] + chunk * CX, nc = min(CX, g.ce[0] - cx0);
    const int xb = box_offset_d(cx0, P, g.ncell[0]);
    const int wdt = box_offset_d(cx0 + nc - 1, P, g.ncell[0]) + P + 1 - xb;
    const int oy = DIM > 1 ? box_offset_d(cy, P, g.ncell[1]) : 0;
    const int oz = DIM > 2 ? box_offset_d(cz, P, g.ncell[2]) : 0;
    const double *Sy = Sl + (DIM > 1 ? category_d(cy, P, g.ncell[1]) : 0) * N1 * N1;
    const double *Sz = Sl + (DIM > 2 ? category_d(cz, P, g.ncell[2]) : 0) * N1 * N1;
    __syncthreads();  // the previous item's LDS reads are done
    // stage the DoF box rows (x contiguous: coalesced)
    for (int i = tid; i < NB2 * NB1 * wdt; i += NT) {
      const int x = i % wdt, yz = i / wdt, iy = yz % NB1, iz = yz / NB1;
      const int64_t gi = (int64_t)(xb + x) + g.N0 * ((int64_t)(oy + iy) + g.N1 * (int64_t)(oz + iz));
      A[yz * W + x] = u[gi - g.base];
    }
    if (f.kind == 2) {
      for (int i = tid; i < nc * N1; i += NT) {
        const int c = i / N1, q = i % N1;
        fx[c * N1 + q] = sine_1d(f, 0, g.lo[0] + (cx0 + c + g.xq[q]) * g.h[0], t);
      }
      if (tid < N1) fy[tid] = DIM > 1 ? sine_1d(f, 1, g.lo[1] + (cy + g.xq[tid]) * g.h[1], t) : 1.0;
      if (tid >= 64 && tid < 64 + N1) fz[tid - 64] = DIM > 2 ? sine_1d(f, 2, g.lo[2] + (cz + g.xq[tid - 64]) * g.h[2], t) : 1.0;
    }
    __syncthreads();
    const double *w = A;
    if (DIM == 3) {  // B[qz][iy][x] = sum_iz Sz[iz][qz] A[iz][iy][x]
      for (int i = tid; i < NB2 * NB1 * W; i += NT) {
        const int x = i % W, qi = i / W, iy = qi % NB1, qz = qi / NB1;
        double s = 0.0;
#pragma unroll
        for (int iz = 0; iz < NB2; ++iz) s = fma(Sz[iz * N1 + qz], A[(iz * NB1 + iy) * W + x], s);
        B[i] = s;
      }
      __syncthreads();
    }
    if (DIM >= 2) {  // A[qz][qy][x] = sum_iy Sy[iy][qy] src[qz][iy][x]
      const double *src = DIM == 3 ? B : A;
      double *dst = DIM == 3 ? A : B;
      for (int i = tid; i < NB2 * NB1 * W; i += NT) {
        const int x = i % W, qi = i / W, qy = qi % NB1, qz = qi / NB1;
        double s = 0.0;
#pragma unroll
        for (int iy = 0; iy < NB1; ++iy) s = fma(Sy[iy * N1 + qy], src[(qz * NB1 + iy) * W + x], s);
        dst[i] = s;
      }
      __syncthreads();
      w = dst;
    }
    // points: one (qy, qz) line of N1 points per step, TPC line groups per cell
    double c_l2 = 0.0;
    if (cl < nc) {
      const int cx = cx0 + cl;
      const double *Sx = Sl + category_d(cx, P, g.ncell[0]) * N1 * N1;
      const int ox = box_offset_d(cx, P, g.ncell[0]) - xb;
      for (int l = grp; l < NB1 * NB2; l += TPC) {
        const int qy = l % NB1, qz = l / NB1;
        const double *wr = w + l * W + ox;
        double wv[N1];
#pragma unroll
        for (int ix = 0; ix < N1; ++ix) wv[ix] = wr[ix];
        const double wyz = g.jxw * (DIM > 1 ? wq[qy] : 1.0) * (DIM > 2 ? wq[qz] : 1.0);
        const double fyz = f.kind == 2 ? fy[qy] * fz[qz] : 0.0;
#pragma unroll
        for (int qx = 0; qx < N1; ++qx) {
          double v = 0.0;
#pragma unroll
          for (int ix = 0; ix < N1; ++ix) v = fma(Sx[ix * N1 + qx], wv[ix], v);
          double ex;
          if (f.kind == 2) {
            ex = fx[cl * N1 + qx] * fyz;
          } else if (f.kind == 1) {
            const double d0 = g.lo[0] + (cx + g.xq[qx]) * g.h[0] - f.prm[1];
            const double d1 = DIM > 1 ? g.lo[1] + (cy + g.xq[qy]) * g.h[1] - f.prm[2] : 0.0;
            const double d2 = DIM > 2 ? g.lo[2] + (cz + g.xq[qz]) * g.h[2] - f.prm[3] : 0.0;
            ex = fmax(0.0, f.prm[0] - sqrt(d0 * d0 + d1 * d1 + d2 * d2));
          } else {
            ex = f.prm[0];
          }
          const double e = v - ex, ae = fabs(e), jxw = wyz * wq[qx];
          c_l2 = fma(e * e, jxw, c_l2);
          a_l1 = fma(ae, jxw, a_l1);
          a_inf = fmax(a_inf, ae);
        }
      }
    }
    a_l2 += c_l2;
    if (cell_err) {
      cacc[grp * CX + cl] = c_l2;
      __syncthreads();
      if (tid < nc) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < TPC; ++k) s += cacc[k * CX + tid];
        const int64_t ci = (int64_t)(cx0 + tid - g.cb[0]) +
                           (int64_t)ncx * ((int64_t)(cy - g.cb[1]) + (int64_t)ncy * (int64_t)(cz - g.cb[2]));
        cell_err[ci] = sqrt(s);
      }
    }
  }
  // block reduction of (Linf, L1, L2^2)
  __shared__ double red[3][NT / 64];
  for (int m = 32; m >= 1; m >>= 1) {
    a_l1 += __shfl_xor(a_l1, m);
    a_l2 += __shfl_xor(a_l2, m);
    a_inf = fmax(a_inf, __shfl_xor(a_inf, m));
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = a_inf;
    red[1][tid >> 6] = a_l1;
    red[2][tid >> 6] = a_l2;
  }
  __syncthreads();
  if (tid == 0) {
    double r0 = red[0][0], r1 = red[1][0], r2 = red[2][0];
    for (int k = 1; k < NT / 64; ++k) {
      r0 = fmax(r0, red[0][k]);
      r1 += red[1][k];
      r2 += red[2][k];
    }
    partial[3 * blockIdx.x + 0] = r0;
    partial[3 * blockIdx.x + 1] = r1;
    partial[3 * blockIdx.x + 2] = r2;
  }
}

// one workgroup: out = (max, sum, sum) of the n partial triples, fixed order
__global__ void __launch_bounds__(256) error_reduce_kernel(int n, const double *__restrict__ partial,
                                                           double *__restrict__ out) {
  __shared__ double red[3][256];
  const int tid = threadIdx.x;
  double r0 = 0.0, r1 = 0.0, r2 = 0.0;
  for (int i = tid; i < n; i += 256) {
    r0 = fmax(r0, partial[3 * i]);
    r1 += partial[3 * i + 1];
    r2 += partial[3 * i + 2];
  }
  red[0][tid] = r0;
  red[1][tid] = r1;
  red[2][tid] = r2;
  __syncthreads();
  for (int m = 128; m >= 1; m >>= 1) {
    if (tid < m) {
      red[0][tid] = fmax(red[0][tid], red[0][tid + m]);
      red[1][tid] += red[1][tid + m];
      red[2][tid] += red[2][tid + m];
    }
    __syncthreads();
  }
  if (tid == 0) {
    out[0] = red[0][0];
    out[1] = red[1][0];
    out[2] = red[2][0];
  }
}

}  // namespace gdmk

extern "C" size_t gdmk_error_norms_lds_bytes(int p, int dim) {
  const int n1 = p + 1, W = gdmk::CX + p, ncat = std::max(1, p);
  const int nb1 = dim > 1 ? n1 : 1, nb2 = dim > 2 ? n1 : 1;
  return sizeof(double) * ((size_t)2 * nb1 * nb2 * W + (size_t)ncat * n1 * n1 + (size_t)gdmk::CX * n1 + 2 * n1 +
                           (size_t)gdmk::TPC * gdmk::CX);
}

namespace {
template <int P, int DIM>
hipError_t launch_err(const gdmk::ErrGeom &g, const gdmk::BcFn &f, double t, const double *S, const double *u,
                      double *cell_err, double *partial, int n_partial, hipStream_t st) {
  const size_t lds = gdmk_error_norms_lds_bytes(P, DIM);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&gdmk::error_norms_kernel<P, DIM>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((gdmk::error_norms_kernel<P, DIM>), dim3((unsigned)n_partial), dim3(gdmk::NT), lds, st, g, f, t,
                     S, u, cell_err, partial);
  return hipSuccess;
}
template <int P>
hipError_t launch_err_dim(const gdmk::ErrGeom &g, const gdmk::BcFn &f, double t, const double *S, const double *u,
                          double *cell_err, double *partial, int n_partial, hipStream_t st) {
  switch (g.dim) {
    case 1: return launch_err<P, 1>(g, f, t, S, u, cell_err, partial, n_partial, st);
    case 2: return launch_err<P, 2>(g, f, t, S, u, cell_err, partial, n_partial, st);
    default: return launch_err<P, 3>(g, f, t, S, u, cell_err, partial, n_partial, st);
  }
}
}  // namespace

extern "C" hipError_t gdmk_launch_error_norms(const gdmk::ErrGeom &g, const gdmk::BcFn &f, double t,
                                             const double *S, const double *u, double *cell_err, double *partial,
                                             int n_partial, double *out3, hipStream_t st) {
  hipError_t e;
  switch (g.p) {
    case 1: e = launch_err_dim<1>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 2: e = launch_err_dim<2>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 3: e = launch_err_dim<3>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 4: e = launch_err_dim<4>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 5: e = launch_err_dim<5>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 6: e = launch_err_dim<6>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 7: e = launch_err_dim<7>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 8: e = launch_err_dim<8>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    case 9: e = launch_err_dim<9>(g, f, t, S, u, cell_err, partial, n_partial, st); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gdmk::error_reduce_kernel, dim3(1), dim3(256), 0, st, n_partial, partial, out3);
  return hipGetLastError();
}
