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

// LDS: row[nb2][nb1][W] | w[nq2][nq1][W] | S[ncat][n1][n1] | fx[CX][n1] | fy[n1] | fz[n1] ; W = CX + p
__global__ void __launch_bounds__(NT) error_norms_kernel(ErrGeom g, BcFn f, double t, const double *__restrict__ S,
                                                         const double *__restrict__ u, double *__restrict__ cell_err,
                                                         double *__restrict__ partial) {
  extern __shared__ double lds[];
  const int p = g.p, n1 = p + 1, W = CX + p;
  const int nb1 = g.nb[1], nb2 = g.nb[2], nq0 = g.nq[0], nq1 = g.nq[1], nq2 = g.nq[2];
  const int ncat = max(1, p);
  double *row = lds;
  double *w = row + (size_t)nb2 * nb1 * W;
  double *Sl = w + (size_t)nq2 * nq1 * W;
  double *fx = Sl + (size_t)ncat * n1 * n1;
  double *fy = fx + CX * n1;
  double *fz = fy + n1;
  const int tid = threadIdx.x;
  for (int i = tid; i < ncat * n1 * n1; i += NT) Sl[i] = S[i];

  const int ncx = g.ce[0] - g.cb[0], ncy = g.ce[1] - g.cb[1], ncz = g.ce[2] - g.cb[2];
  const int chunks = (ncx + CX - 1) / CX;
  const int64_t n_items = (int64_t)chunks * ncy * ncz;
  const int npts = nq0 * nq1 * nq2;
  double a_l1 = 0.0, a_l2 = 0.0, a_inf = 0.0;

  for (int64_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int chunk = (int)(item % chunks);
    const int64_t r = item / chunks;
    const int cy = g.cb[1] + (int)(r % ncy), cz = g.cb[2] + (int)(r / ncy);
    const int cx0 = g.cb[0] + chunk * CX, nc = min(CX, g.ce[0] - cx0);
    const int xb = box_offset_d(cx0, p, g.ncell[0]);
    const int wdt = box_offset_d(cx0 + nc - 1, p, g.ncell[0]) + p + 1 - xb;
    const int oy = g.dim > 1 ? box_offset_d(cy, p, g.ncell[1]) : 0;
    const int oz = g.dim > 2 ? box_offset_d(cz, p, g.ncell[2]) : 0;
    const int caty = g.dim > 1 ? category_d(cy, p, g.ncell[1]) : 0;
    const int catz = g.dim > 2 ? category_d(cz, p, g.ncell[2]) : 0;
    __syncthreads();  // previous item's LDS reads are done
    // stage the DoF box rows (x contiguous: coalesced)
    for (int i = tid; i < nb2 * nb1 * wdt; i += NT) {
      const int x = i % wdt, yz = i / wdt, iy = yz % nb1, iz = yz / nb1;
      const int64_t gi = (int64_t)(xb + x) + g.N0 * ((int64_t)(oy + iy) + g.N1 * (int64_t)(oz + iz));
      row[(size_t)yz * W + x] = u[gi - g.base];
    }
    if (f.kind == 2) {
      for (int i = tid; i < nc * nq0; i += NT) {
        const int c = i / nq0, q = i % nq0;
        fx[c * n1 + q] = sine_1d(f, 0, g.lo[0] + (cx0 + c + g.xq[q]) * g.h[0], t);
      }
      if (tid < nq1) fy[tid] = g.dim > 1 ? sine_1d(f, 1, g.lo[1] + (cy + g.xq[tid]) * g.h[1], t) : 1.0;
      if (tid >= 64 && tid - 64 < nq2) fz[tid - 64] = g.dim > 2 ? sine_1d(f, 2, g.lo[2] + (cz + g.xq[tid - 64]) * g.h[2], t) : 1.0;
    }
    __syncthreads();
    // contract z and y: w[qz][qy][x] = sum_iz sum_iy Sz[iz][qz] Sy[iy][qy] row[iz][iy][x]
    for (int i = tid; i < nq2 * nq1 * wdt; i += NT) {
      const int x = i % wdt, qq = i / wdt, qy = qq % nq1, qz = qq / nq1;
      double acc = 0.0;
      for (int iz = 0; iz < nb2; ++iz) {
        const double sz = g.dim > 2 ? Sl[(catz * n1 + iz) * n1 + qz] : 1.0;
        double s = 0.0;
        for (int iy = 0; iy < nb1; ++iy) {
          const double sy = g.dim > 1 ? Sl[(caty * n1 + iy) * n1 + qy] : 1.0;
          s = fma(sy, row[(size_t)(iz * nb1 + iy) * W + x], s);
        }
        acc = fma(sz, s, acc);
      }
      w[(size_t)qq * W + x] = acc;
    }
    __syncthreads();
    // points: TPC lanes per cell
    const int cl = tid / TPC, sub = tid % TPC;
    double c_l2 = 0.0;
    if (cl < nc) {
      const int cx = cx0 + cl;
      const int catx = category_d(cx, p, g.ncell[0]);
      const int ox = box_offset_d(cx, p, g.ncell[0]) - xb;
      for (int pt = sub; pt < npts; pt += TPC) {
        const int qx = pt % nq0, qy = (pt / nq0) % nq1, qz = pt / (nq0 * nq1);
        const double *wr = w + (size_t)(qz * nq1 + qy) * W + ox;
        double v = 0.0;
        for (int ix = 0; ix < n1; ++ix) v = fma(Sl[(catx * n1 + ix) * n1 + qx], wr[ix], v);
        double ex;
        if (f.kind == 0) {
          ex = f.prm[0];
        } else if (f.kind == 1) {
          const double xc[3] = {g.lo[0] + (cx + g.xq[qx]) * g.h[0], g.lo[1] + (cy + g.xq[qy]) * g.h[1],
                                g.lo[2] + (cz + g.xq[qz]) * g.h[2]};
          double r2 = 0.0;
          for (int d = 0; d < g.dim; ++d) r2 += (xc[d] - f.prm[1 + d]) * (xc[d] - f.prm[1 + d]);
          ex = fmax(0.0, f.prm[0] - sqrt(r2));
        } else {
          ex = fx[cl * n1 + qx] * fy[qy] * fz[qz];
        }
        const double e = v - ex, ae = fabs(e);
        const double jxw = g.jxw * g.wq[qx] * (g.dim > 1 ? g.wq[qy] : 1.0) * (g.dim > 2 ? g.wq[qz] : 1.0);
        c_l2 = fma(e * e, jxw, c_l2);
        a_l1 = fma(ae, jxw, a_l1);
        a_inf = fmax(a_inf, ae);
      }
    }
    a_l2 += c_l2;
    // the cell's TPC lanes are consecutive in one wave
    double s = c_l2;
    for (int m = 1; m < TPC; m <<= 1) s += __shfl_xor(s, m);
    if (cell_err && cl < nc && sub == 0) {
      const int64_t ci = (int64_t)(cx0 + cl - g.cb[0]) +
                         (int64_t)ncx * ((int64_t)(cy - g.cb[1]) + (int64_t)ncy * (int64_t)(cz - g.cb[2]));
      cell_err[ci] = sqrt(s);
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

extern "C" size_t gdmk_error_norms_lds_bytes(int p) {
  const int n1 = p + 1, W = gdmk::CX + p, ncat = std::max(1, p);
  return sizeof(double) * ((size_t)2 * n1 * n1 * W + (size_t)ncat * n1 * n1 + (size_t)gdmk::CX * n1 + 2 * n1);
}

extern "C" hipError_t gdmk_launch_error_norms(const gdmk::ErrGeom &g, const gdmk::BcFn &f, double t,
                                             const double *S, const double *u, double *cell_err, double *partial,
                                             int n_partial, double *out3, hipStream_t st) {
  const size_t lds = gdmk_error_norms_lds_bytes(g.p);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&gdmk::error_norms_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(gdmk::error_norms_kernel, dim3((unsigned)n_partial), dim3(gdmk::NT), lds, st, g, f, t, S, u,
                     cell_err, partial);
  hipLaunchKernelGGL(gdmk::error_reduce_kernel, dim3(1), dim3(256), 0, st, n_partial, partial, out3);
  return hipGetLastError();
}
