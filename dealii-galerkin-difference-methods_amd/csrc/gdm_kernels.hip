// gdm_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the GDM operator
// engine.  See DESIGN.md for the derivation; in short, on an uncut uniform
// Cartesian mesh every hot-path operator of the reference is a sum of
// Kronecker products of 1D band matrices of half-bandwidth p:
//
//   advection (advection/stiffness.h:345-532, alpha = 0, outflow traces folded
//              into B_d):            K = B_x M_y M_z + M_x B_y M_z + M_x M_y B_z
//   wave      (wave/stiffness.h:171-181):                  same with B_d = -L_d
//   mass      (advection/mass.h:144-156):                  M = M_x M_y M_z
//
// The fused kernel marches each (x, y) tile along z.  Per input plane:
//   1. the (TY + 2p) x (64 + 2p) plane tile is staged in LDS,
//   2. x-sweep  A = M_x u, Bv = B_x u          (LDS -> LDS, lane = x),
//   3. y-sweep  D = M_y A, E = M_y Bv + B_y A  (LDS -> registers, R rows/lane),
//   4. z-scatter: out[z'] += M_z(z', z) E + B_z(z', z) D for the 2p + 1 planes
//      z' around z, kept in a register ring that retires one finished output
//      plane per input plane (coalesced 512-B row stores).
// y- and z-coefficients are wave-uniform (scalar loads); x-coefficients are
// per-lane registers (they differ only near the x faces).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gdm_kernels.h"

namespace gdmk {



template <int P, int R, int NW>
struct StencilGeom {
  static constexpr int W = 2 * P + 1;  // band width = ring size
  static constexpr int TX = 64;        // one wave row
  static constexpr int TY = R * NW;
  static constexpr int UR = TY + 2 * P;  // staged rows
  static constexpr int UP = TX + 2 * P;  // staged row pitch (doubles)
  static constexpr int NT = 64 * NW;
  static constexpr size_t lds_bytes(bool mass) {
    return sizeof(double) * ((size_t)UR * UP + (size_t)UR * TX * (mass ? 1 : 2));
  }
};

template <int P, int R, int NW, bool MASS>
__global__ void __launch_bounds__(64 * NW) stencil3d_kernel(StencilArgs a) {
  using G = StencilGeom<P, R, NW>;
  constexpr int W = G::W, TX = G::TX, TY = G::TY, UR = G::UR, UP = G::UP, NT = G::NT;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double *us = smem;              // UR x UP
  double *as = smem + UR * UP;    // UR x TX
  double *bs = as + UR * TX;      // UR x TX (unused for MASS)

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int x0 = blockIdx.x * TX;
  const int y0 = a.out_y0 + blockIdx.y * TY;
  const int zc0 = a.out_z0 + blockIdx.z * a.zchunk;
  const int zc1 = min(zc0 + a.zchunk, a.out_z1);
  const int x = x0 + lane;
  const int Nx = a.Nx;
  const int ny_in = a.in_y1 - a.in_y0, ny_out = a.out_y1 - a.out_y0;

  double cmx[W], cbx[W];
#pragma unroll
  for (int k = 0; k < W; ++k) {
    cmx[k] = (x < Nx) ? a.rowMx[(size_t)x * W + k] : 0.0;
    cbx[k] = (!MASS && x < Nx) ? a.rowBx[(size_t)x * W + k] : 0.0;
  }

  double acc[W][R];
#pragma unroll
  for (int s = 0; s < W; ++s)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[s][j] = 0.0;

  const int zs = max(zc0 - P, a.in_z0);
  const int ze = min(zc1 + P, a.in_z1);  // input planes with contributions: [zs, ze)
  const int zend = zc1 + P;              // retire up to output plane zc1 - 1
  const int ybase = y0 + wv * R;         // first output row of this wave

  for (int zb = zs - (zs % W); zb < zend; zb += W) {
#pragma unroll
    for (int jp = 0; jp < W; ++jp) {
      const int zz = zb + jp;
      if (zz >= zs && zz < zend) {
        if (zz < ze) {
          // ---- 1. stage the plane tile (zero outside the valid input box) ----
          const double *plane = a.src + (int64_t)(zz - a.in_z0) * ny_in * Nx;
          for (int e = threadIdx.x; e < UR * UP; e += NT) {
            const int r = e / UP, c = e - r * UP;
            const int gx = x0 - P + c, gy = y0 - P + r;
            double v = 0.0;
            if (gx >= 0 && gx < Nx && gy >= a.in_y0 && gy < a.in_y1)
              v = plane[(int64_t)(gy - a.in_y0) * Nx + gx];
            us[e] = v;
          }
          __syncthreads();
          // ---- 2. x-sweep ----
          for (int r = wv; r < UR; r += NW) {
            const double *ur = us + r * UP + lane;
            double am = 0.0, ab = 0.0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
              const double u = ur[k];
              am = fma(cmx[k], u, am);
              if (!MASS) ab = fma(cbx[k], u, ab);
            }
            as[r * TX + lane] = am;
            if (!MASS) bs[r * TX + lane] = ab;
          }
          __syncthreads();
          // ---- 3. y-sweep (scatter into this wave's R rows) ----
          double D[R], E[R];
#pragma unroll
          for (int j = 0; j < R; ++j) D[j] = E[j] = 0.0;
#pragma unroll
          for (int t = 0; t < R + 2 * P; ++t) {
            const int trow = wv * R + t;        // tile row
            const int s = ybase - P + t;        // global row, in [-P, Ny + P)
            const double av = as[trow * TX + lane];
            const double bv = MASS ? 0.0 : bs[trow * TX + lane];
            const double *cm = a.colMy + (size_t)(s + P) * W;
            const double *cb = a.colBy + (size_t)(s + P) * W;
#pragma unroll
            for (int j = 0; j < R; ++j) {
              const int k = j + 2 * P - t;
              if (k >= 0 && k < W) {
                const double m = cm[k];
                D[j] = fma(m, av, D[j]);
                if (!MASS) E[j] = fma(m, bv, fma(cb[k], av, E[j]));
              }
            }
          }
          // ---- 4. z-scatter into the register ring ----
          const double *cmz = a.colMz + (size_t)zz * W;
          const double *cbz = a.colBz + (size_t)zz * W;
#pragma unroll
          for (int k = 0; k < W; ++k) {
            const int slot = ((jp - P + k) % W + W) % W;
            const double m = cmz[k];
            if (MASS) {
#pragma unroll
              for (int j = 0; j < R; ++j) acc[slot][j] = fma(m, D[j], acc[slot][j]);
            } else {
              const double b = cbz[k];
#pragma unroll
              for (int j = 0; j < R; ++j) acc[slot][j] = fma(m, E[j], fma(b, D[j], acc[slot][j]));
            }
          }
        }
        // ---- retire output plane zz - P ----
        {
          const int slot = ((jp - P) % W + W) % W;
          const int zo = zz - P;
          if (zo >= zc0 && zo < zc1) {
            double *orow = a.dst + ((int64_t)(zo - a.out_z0) * ny_out + (ybase - a.out_y0)) * Nx + x;
#pragma unroll
            for (int j = 0; j < R; ++j)
              if (x < Nx && ybase + j < a.out_y1) orow[(int64_t)j * Nx] = acc[slot][j];
          }
#pragma unroll
          for (int j = 0; j < R; ++j) acc[slot][j] = 0.0;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Exact Kronecker mass inverse: banded Cholesky solves along one direction.
// One thread per line; the position along the line is wave-uniform, so the
// factor entries are scalar loads.  line l -> base = (l / A) * B + (l % A) * C.
// lrow: (len + P) x (P + 1), rows >= len zero-padded.
// ---------------------------------------------------------------------------
template <int P>
__global__ void __launch_bounds__(256) chol_lines_kernel(double *__restrict__ v, int len, int64_t stride,
                                                          int64_t n_lines, int64_t A, int64_t B, int64_t C,
                                                          const double *__restrict__ lrow,
                                                          const double *__restrict__ inv_diag) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_lines) return;
  double *line = v + (l / A) * B + (l % A) * C;
  double win[P];
#pragma unroll
  for (int k = 0; k < P; ++k) win[k] = 0.0;
  // forward: w_i = (r_i - sum_k L(i, i-P+k) w_{i-P+k}) / L(i,i)
  for (int i = 0; i < len; ++i) {
    const double *L = lrow + (size_t)i * (P + 1);
    double s = line[(int64_t)i * stride];
#pragma unroll
    for (int k = 0; k < P; ++k) s = fma(-L[k], win[k], s);
    s *= inv_diag[i];
    line[(int64_t)i * stride] = s;
#pragma unroll
    for (int k = 0; k < P - 1; ++k) win[k] = win[k + 1];
    win[P - 1] = s;
  }
#pragma unroll
  for (int k = 0; k < P; ++k) win[k] = 0.0;
  // backward: x_i = (w_i - sum_m L(i+m, i) x_{i+m}) / L(i,i)
  for (int i = len - 1; i >= 0; --i) {
    double s = line[(int64_t)i * stride];
#pragma unroll
    for (int m = 1; m <= P; ++m) s = fma(-lrow[(size_t)(i + m) * (P + 1) + (P - m)], win[m - 1], s);
    s *= inv_diag[i];
    line[(int64_t)i * stride] = s;
#pragma unroll
    for (int m = P - 1; m > 0; --m) win[m] = win[m - 1];
    win[0] = s;
  }
}

// ---------------------------------------------------------------------------
// Inflow boundary-data term (advection/stiffness.h:473-532 with a.n < 0):
//   rhs(node) += |a.n| sum_{q on face} u+_q phi_node(x_q) JxW_q
// factorised over the two tangential directions of the face:
//   step 1: T[q1][i0] = sum_m U[q1][qs0(i0) + m] w0[i0][m]
//   step 2: dst(i0, i1) += scale * sum_m w1[i1][m] T[qs1(i1) + m][i0]
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) face_step1_kernel(const double *__restrict__ U, int Q0, int Q1, int i0_begin,
                                                          int n0, const int *__restrict__ qs0,
                                                          const int *__restrict__ qc0,
                                                          const double *__restrict__ w0, int wmax0,
                                                          double *__restrict__ T) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int q1 = blockIdx.y;
  if (t >= n0 || q1 >= Q1) return;
  const int i0 = i0_begin + t;
  const double *u = U + (int64_t)q1 * Q0 + qs0[i0];
  const double *w = w0 + (int64_t)i0 * wmax0;
  const int n = qc0[i0];
  double s = 0.0;
  for (int m = 0; m < n; ++m) s = fma(u[m], w[m], s);
  T[(int64_t)q1 * n0 + t] = s;
}

__global__ void __launch_bounds__(256) face_step2_kernel(const double *__restrict__ T, int n0, int i1_begin,
                                                          int i1_end, const int *__restrict__ qs1,
                                                          const int *__restrict__ qc1,
                                                          const double *__restrict__ w1, int wmax1,
                                                          double *__restrict__ dst, int64_t base,
                                                          int64_t stride0, int64_t stride1, double scale) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i1 = i1_begin + (int)blockIdx.y;
  if (t >= n0 || i1 >= i1_end) return;
  const double *w = w1 + (int64_t)i1 * wmax1;
  const int n = qc1[i1], q = qs1[i1];
  double s = 0.0;
  for (int m = 0; m < n; ++m) s = fma(w[m], T[(int64_t)(q + m) * n0 + t], s);
  double *d = dst + base + (int64_t)t * stride0 + (int64_t)(i1 - i1_begin) * stride1;
  *d += scale * s;
}

// ---------------------------------------------------------------------------
// BLAS-1
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) axpby_kernel(int64_t n, double a, const double *__restrict__ x, double b,
                                                     double *__restrict__ y) {
  const int64_t n2 = n / 2;
  const double2 *x2 = reinterpret_cast<const double2 *>(x);
  double2 *y2 = reinterpret_cast<double2 *>(y);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 xv = x2[i];
    double2 yv = y2[i];
    yv.x = fma(a, xv.x, b * yv.x);
    yv.y = fma(a, xv.y, b * yv.y);
    y2[i] = yv;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) y[n - 1] = fma(a, x[n - 1], b * y[n - 1]);
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) dot_partial_kernel(int64_t n, const double *__restrict__ x,
                                                           const double *__restrict__ y,
                                                           double *__restrict__ partial) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s = fma(x[i], y[i], s);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) dot_final_kernel(int n, const double *__restrict__ partial,
                                                         double *__restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) zero_kernel(int64_t n, double *__restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = 0.0;
}

// ---------------------------------------------------------------------------
// host-side launchers (called from gdm_capi.cpp)
// ---------------------------------------------------------------------------
template <int P, int R, int NW, bool MASS>
static hipError_t launch_stencil_t(const StencilArgs &a, hipStream_t st) {
  using G = StencilGeom<P, R, NW>;
  const size_t lds = G::lds_bytes(MASS);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)stencil3d_kernel<P, R, NW, MASS>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  dim3 grid((a.Nx + G::TX - 1) / G::TX, (a.out_y1 - a.out_y0 + G::TY - 1) / G::TY,
            (a.out_z1 - a.out_z0 + a.zchunk - 1) / a.zchunk);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  hipLaunchKernelGGL((stencil3d_kernel<P, R, NW, MASS>), grid, dim3(G::NT), lds, st, a);
  return hipGetLastError();
}

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_stencil(int p, bool mass, const gdmk::StencilArgs &a, hipStream_t st) {
  using namespace gdmk;
  switch (p) {
    case 1: return mass ? launch_stencil_t<1, 4, 8, true>(a, st) : launch_stencil_t<1, 4, 8, false>(a, st);
    case 3: return mass ? launch_stencil_t<3, 4, 8, true>(a, st) : launch_stencil_t<3, 4, 8, false>(a, st);
    case 5: return mass ? launch_stencil_t<5, 4, 8, true>(a, st) : launch_stencil_t<5, 4, 8, false>(a, st);
    case 7: return mass ? launch_stencil_t<7, 4, 8, true>(a, st) : launch_stencil_t<7, 4, 8, false>(a, st);
    case 9: return mass ? launch_stencil_t<9, 2, 8, true>(a, st) : launch_stencil_t<9, 2, 8, false>(a, st);
    default: return hipErrorInvalidValue;
  }
}

extern "C" int gdmk_stencil_tile_rows(int p) { return p == 9 ? 16 : 32; }

extern "C" hipError_t gdmk_launch_chol_lines(int p, double *v, int len, int64_t stride, int64_t n_lines, int64_t A,
                                             int64_t B, int64_t C, const double *lrow, const double *inv_diag,
                                             hipStream_t st) {
  using namespace gdmk;
  if (n_lines <= 0) return hipSuccess;
  dim3 grid((unsigned)((n_lines + 255) / 256)), block(256);
  switch (p) {
    case 1: hipLaunchKernelGGL(chol_lines_kernel<1>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 3: hipLaunchKernelGGL(chol_lines_kernel<3>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 5: hipLaunchKernelGGL(chol_lines_kernel<5>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 7: hipLaunchKernelGGL(chol_lines_kernel<7>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 9: hipLaunchKernelGGL(chol_lines_kernel<9>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_face(const gdmk::FaceArgs &f, hipStream_t st) {
  using namespace gdmk;
  const int n0 = f.i0_end - f.i0_begin;
  if (n0 <= 0 || f.Q1 <= 0 || f.i1_end <= f.i1_begin) return hipSuccess;
  dim3 g1((n0 + 255) / 256, f.Q1), b(256);
  hipLaunchKernelGGL(face_step1_kernel, g1, b, 0, st, f.U, f.Q0, f.Q1, f.i0_begin, n0, f.qs0, f.qc0, f.w0, f.wmax0,
                     f.T);
  dim3 g2((n0 + 255) / 256, f.i1_end - f.i1_begin);
  hipLaunchKernelGGL(face_step2_kernel, g2, b, 0, st, f.T, n0, f.i1_begin, f.i1_end, f.qs1, f.qc1, f.w1, f.wmax1,
                     f.dst, f.base, f.stride0, f.stride1, f.scale);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_axpby(int64_t n, double a, const double *x, double b, double *y, hipStream_t st) {
  using namespace gdmk;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n / 2 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, a, x, b, y);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_dot(int64_t n, const double *x, const double *y, double *partial, int n_partial,
                                     double *out, hipStream_t st) {
  using namespace gdmk;
  hipLaunchKernelGGL(dot_partial_kernel, dim3(n_partial), dim3(256), 0, st, n, x, y, partial);
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(256), 0, st, n_partial, partial, out);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_zero(int64_t n, double *y, hipStream_t st) {
  using namespace gdmk;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, y);
  return hipGetLastError();
}
