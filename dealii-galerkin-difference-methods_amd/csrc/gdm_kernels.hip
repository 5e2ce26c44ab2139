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
#include <cstdlib>

#include "gdm_kernels.h"

namespace gdmk {



template <int P, int R, int NW, int NBUF_ = 3, int WPC_ = 2>
struct StencilGeom {
  static constexpr int W = 2 * P + 1;      // band width = ring size
  static constexpr int TX = 64;            // one wave row
  static constexpr int TY = R * NW;        // output rows per tile
  static constexpr int UR = TY + 2 * P;    // staged rows
  static constexpr int XH = (P + 1) & ~1;  // x halo, even -> 16-B aligned row start
  static constexpr int RL = TX + 2 * XH;   // staged row length (doubles)
  static constexpr int NT = 64 * NW;
  static constexpr int NBUF = NBUF_;       // plane ring: current + NBUF-1 in flight
  static constexpr int WPC = WPC_;         // resident workgroups per CU (register budget)
  static constexpr int NCORR = 2 * (P + 1);  // x columns whose band row differs from the Toeplitz row
  static constexpr int USZ = UR * RL;      // doubles per staged plane
  static constexpr size_t lds_bytes(bool mass) {
    return sizeof(double) * ((size_t)NBUF * USZ + (size_t)UR * TX * (mass ? 1 : 2) + (size_t)NCORR * 2 * W);
  }
};

// Stage one plane tile (rows y0-P .. y0+TY+P-1, columns x0-XH .. x0+TX+XH-1)
// into LDS with LDS-DMA (buffer_load ... lds).  Chunks outside the valid
// input box get an out-of-range voffset, which the buffer range check turns
// into zeros.  CH = 16 (2 doubles per lane; rows 16-B aligned: Nx even) or
// CH = 4 (any Nx).
template <int P, int R, int NW, int CH>
struct StageCount {
  using G = StencilGeom<P, R, NW>;
  static constexpr int DPC = CH / 4;                 // dwords per chunk
  static constexpr int CPR = G::RL * 2 / DPC;        // chunks per row
  static constexpr int NCH = G::UR * CPR;            // chunks per plane
  static constexpr int NI = (NCH + 63) / 64;         // wave-instructions per plane
  static constexpr int MIN_PER_WAVE = NI / NW;       // issued by every wave
};

template <int P, int R, int NW, int CH>
__device__ __forceinline__ void stage_plane(const StencilArgs &a, int zz, int x0, int y0, double *ubuf, int wv,
                                            int lane) {
  using G = StencilGeom<P, R, NW>;
  using SC = StageCount<P, R, NW, CH>;
  const int ny_in = a.in_y1 - a.in_y0;
  const double *plane = a.src + (int64_t)(zz - a.in_z0) * ny_in * a.Nx;
  const int nbytes = (int)((int64_t)ny_in * a.Nx * 8);
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)plane, 0, nbytes, 0x00020000);
  for (int j = wv; j < SC::NI; j += NW) {
    const int e = j * 64 + lane;
    const int r = e / SC::CPR, c = e - r * SC::CPR;
    const int gy = y0 - P + r;
    const int gx2 = (x0 - G::XH) * 2 + c * SC::DPC;  // dword column
    uint32_t voff = 0x80000000u;                      // out of range -> zeros
    if (e < SC::NCH && gy >= a.in_y0 && gy < a.in_y1 && gx2 >= 0 && gx2 < 2 * a.Nx)
      voff = (uint32_t)(((int64_t)(gy - a.in_y0) * a.Nx * 2 + gx2) * 4);
    if (e < SC::NCH) {
      auto *dst = (__attribute__((address_space(3))) void *)((char *)ubuf + (size_t)j * 64 * CH);
      if constexpr (CH == 16)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 16, voff, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 4, voff, 0, 0, 0);
    }
  }
}

#define GDM_WAIT_VMCNT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")
#define GDM_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Coefficient tables are read-only for the whole launch and indexed by
// wave-uniform positions: read them through the constant address space so
// they become scalar (s_load) loads instead of vector loads.
typedef __attribute__((address_space(4))) const double cdouble;
__device__ __forceinline__ cdouble *cptr(const double *p) { return (cdouble *)(p); }

// Per-workgroup state of the z-march (all wave-uniform except lane/x).
struct MarchCtx {
  double *ubase, *as, *bs, *corr;
  int lane, wv, x0, y0, x, zc0, zc1, zs, ze, zend, ybase, cslot, ny_out;
  bool need_corr;
};

// One input plane zz at ring phase JP (= zz mod W): stage/sweep/scatter, then
// retire output plane zz - p.  JP is a template parameter so every ring slot
// index is a compile-time constant and the ring stays in registers.
template <int JP, int P, int R, int NW, int NBUF, int WPC, bool MASS, int CH>
__device__ __forceinline__ void march_plane(const StencilArgs &a, const MarchCtx &c, double (&acc)[2 * P + 1][R],
                                            int zz) {
  using G = StencilGeom<P, R, NW, NBUF, WPC>;
  using SC = StageCount<P, R, NW, CH>;
  constexpr int W = G::W, TX = G::TX, UR = G::UR, RL = G::RL, XH = G::XH, USZ = G::USZ;
  if (zz < c.ze) {
    // ---- 1. this wave's DMA of plane zz landed; barrier: every wave's did
    //         and every wave finished plane zz-1 ----
    if (zz + 1 < c.ze)
      GDM_WAIT_VMCNT(SC::MIN_PER_WAVE);
    else
      GDM_WAIT_VMCNT(0);
    GDM_LDS_BARRIER();
    // buffer (zz+NBUF-1) % NBUF == (zz-1) % NBUF was last read by the x-sweep of zz-1
    if (zz + NBUF - 1 < c.ze)
      stage_plane<P, R, NW, CH>(a, zz + NBUF - 1, c.x0, c.y0, c.ubase + ((zz + NBUF - 1) % NBUF) * USZ, c.wv,
                                c.lane);
    const double *us = c.ubase + (zz % NBUF) * USZ;
    // ---- 2. x-sweep: A = M_x u, Bv = B_x u on the UR staged rows ----
    // (the Toeplitz row is re-read from the scalar cache every plane instead
    //  of pinning 4(2p+1) SGPRs for the whole kernel)
    cdouble *tM = cptr(a.tMx), *tB = cptr(a.tBx);
    asm volatile("" : "+s"(tM), "+s"(tB));
    for (int r = c.wv; r < UR; r += NW) {
      const double *ur = us + r * RL + c.lane + (XH - P);
      double uk[W];
#pragma unroll
      for (int k = 0; k < W; ++k) uk[k] = ur[k];
      double am = 0.0, ab = 0.0;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        am = fma(tM[k], uk[k], am);
        if (!MASS) ab = fma(tB[k], uk[k], ab);
      }
      if (c.need_corr && c.cslot >= 0) {
        const double *cm = c.corr + c.cslot * 2 * W;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          am = fma(cm[k], uk[k], am);
          if (!MASS) ab = fma(cm[W + k], uk[k], ab);
        }
      }
      c.as[r * TX + c.lane] = am;
      if (!MASS) c.bs[r * TX + c.lane] = ab;
    }
    GDM_LDS_BARRIER();
    // ---- 3. y-sweep: scatter the R + 2p staged rows into this wave's R rows ----
    double D[R], E[R];
#pragma unroll
    for (int j = 0; j < R; ++j) D[j] = E[j] = 0.0;
#pragma unroll
    for (int t = 0; t < R + 2 * P; ++t) {
      const int trow = c.wv * R + t;  // tile row
      const int s = c.ybase - P + t;  // global row, in [-P, Ny + P + TY)
      const double av = c.as[trow * TX + c.lane];
      const double bv = MASS ? 0.0 : c.bs[trow * TX + c.lane];
      cdouble *cm = cptr(a.colMy) + (size_t)(s + P) * W;
      cdouble *cb = cptr(a.colBy) + (size_t)(s + P) * W;
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
    cdouble *cmz = cptr(a.colMz) + (size_t)zz * W;
    cdouble *cbz = cptr(a.colBz) + (size_t)zz * W;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      constexpr int base = JP - P + 2 * W;
      const int slot = (base + k) % W;
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
  // ---- retire output plane zz - p (complete: every contributing plane done) ----
  constexpr int rslot = (JP - P + 2 * W) % W;
  const int zo = zz - P;
  if (zo >= c.zc0 && zo < c.zc1) {
    const int Nx = a.Nx;
    double *orow = a.dst + ((int64_t)(zo - a.out_z0) * c.ny_out + (c.ybase - a.out_y0)) * Nx + c.x;
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (c.x < Nx && c.ybase + j < a.out_y1) orow[(int64_t)j * Nx] = acc[rslot][j];
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc[rslot][j] = 0.0;
}

template <int JP, int P, int R, int NW, int NBUF, int WPC, bool MASS, int CH>
__device__ __forceinline__ void march_phases(const StencilArgs &a, const MarchCtx &c, double (&acc)[2 * P + 1][R],
                                             int zb) {
  if constexpr (JP < 2 * P + 1) {
    const int zz = zb + JP;
    if (zz >= c.zs && zz < c.zend) march_plane<JP, P, R, NW, NBUF, WPC, MASS, CH>(a, c, acc, zz);
    march_phases<JP + 1, P, R, NW, NBUF, WPC, MASS, CH>(a, c, acc, zb);
  }
}

template <int P, int R, int NW, int NBUF, int WPC, bool MASS, int CH>
__global__ void __launch_bounds__(64 * NW, (64 * NW * WPC) / 256) stencil3d_kernel(StencilArgs a) {
  using G = StencilGeom<P, R, NW, NBUF, WPC>;
  constexpr int W = G::W, TX = G::TX, UR = G::UR, USZ = G::USZ;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  MarchCtx c;
  c.ubase = smem;                                // NBUF x UR x RL
  c.as = smem + NBUF * USZ;                      // UR x TX
  c.bs = c.as + UR * TX;                         // UR x TX (unused for MASS)
  c.corr = c.as + UR * TX * (MASS ? 1 : 2);      // NCORR x 2W wall-row corrections
  c.lane = threadIdx.x & 63;
  c.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.x0 = blockIdx.x * TX;
  c.y0 = a.out_y0 + blockIdx.y * G::TY;
  c.zc0 = a.out_z0 + blockIdx.z * a.zchunk;
  c.zc1 = min(c.zc0 + a.zchunk, a.out_z1);
  c.x = c.x0 + c.lane;
  c.ny_out = a.out_y1 - a.out_y0;
  c.zs = max(c.zc0 - P, a.in_z0);
  c.ze = min(c.zc1 + P, a.in_z1);  // input planes with contributions: [zs, ze)
  c.zend = c.zc1 + P;              // retire up to output plane zc1 - 1
  c.ybase = c.y0 + c.wv * R;       // first output row of this wave

  // x rows: wave-uniform Toeplitz row; the p+1 columns next to each wall
  // (every column of a domain narrower than 2p + 3) add row(x) - T from a
  // per-tile LDS table
  c.need_corr = (c.x0 < a.x_corr_left) || (c.x0 + TX > a.Nx - a.x_corr_right);
  c.cslot = -1;
  if (c.need_corr) {
    if (c.x < a.x_corr_left)
      c.cslot = c.x;
    else if (c.x < a.Nx && c.x >= a.Nx - a.x_corr_right)
      c.cslot = (P + 1) + (c.x - (a.Nx - a.x_corr_right));
    for (int e = threadIdx.x; e < G::NCORR * 2 * W; e += G::NT) c.corr[e] = a.corrX[e];
  }

  double acc[W][R];
#pragma unroll
  for (int s = 0; s < W; ++s)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[s][j] = 0.0;

  // prologue: NBUF-1 planes in flight
#pragma unroll
  for (int d = 0; d < NBUF - 1; ++d)
    if (c.zs + d < c.ze)
      stage_plane<P, R, NW, CH>(a, c.zs + d, c.x0, c.y0, c.ubase + ((c.zs + d) % NBUF) * USZ, c.wv, c.lane);

  for (int zb = c.zs - (c.zs % W); zb < c.zend; zb += W)
    march_phases<0, P, R, NW, NBUF, WPC, MASS, CH>(a, c, acc, zb);
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
template <int P, int R, int NW, int NBUF, int WPC, bool MASS, int CH>
static hipError_t launch_stencil_t(const StencilArgs &a, hipStream_t st) {
  using G = StencilGeom<P, R, NW, NBUF, WPC>;
  const size_t lds = G::lds_bytes(MASS);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void *)stencil3d_kernel<P, R, NW, NBUF, WPC, MASS, CH>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  dim3 grid((a.Nx + G::TX - 1) / G::TX, (a.out_y1 - a.out_y0 + G::TY - 1) / G::TY,
            (a.out_z1 - a.out_z0 + a.zchunk - 1) / a.zchunk);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  hipLaunchKernelGGL((stencil3d_kernel<P, R, NW, NBUF, WPC, MASS, CH>), grid, dim3(G::NT), lds, st, a);
  return hipGetLastError();
}

template <int P, int R, int NW, int NBUF, int WPC>
static hipError_t launch_stencil_p(bool mass, const StencilArgs &a, hipStream_t st) {
  // 16-B LDS-DMA chunks need every staged row to start 16-B aligned
  const bool vec = (a.Nx % 2 == 0) && ((reinterpret_cast<uintptr_t>(a.src) & 15) == 0);
  if (vec)
    return mass ? launch_stencil_t<P, R, NW, NBUF, WPC, true, 16>(a, st)
                : launch_stencil_t<P, R, NW, NBUF, WPC, false, 16>(a, st);
  return mass ? launch_stencil_t<P, R, NW, NBUF, WPC, true, 4>(a, st)
              : launch_stencil_t<P, R, NW, NBUF, WPC, false, 4>(a, st);
}

}  // namespace gdmk


extern "C" int gdmk_stencil_tile_rows(int p) { return 16; }

extern "C" hipError_t gdmk_launch_stencil(int p, bool mass, const gdmk::StencilArgs &a, hipStream_t st) {
  using namespace gdmk;
  switch (p) {  // <P, R, NW, NBUF, WG per CU>
    case 1: return launch_stencil_p<1, 2, 8, 3, 2>(mass, a, st);
    case 3: return launch_stencil_p<3, 2, 8, 3, 2>(mass, a, st);
    case 5: return launch_stencil_p<5, 2, 8, 3, 2>(mass, a, st);
    case 7: return launch_stencil_p<7, 2, 8, 2, 2>(mass, a, st);
    case 9: return launch_stencil_p<9, 2, 8, 2, 1>(mass, a, st);
    default: return hipErrorInvalidValue;
  }
}

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
