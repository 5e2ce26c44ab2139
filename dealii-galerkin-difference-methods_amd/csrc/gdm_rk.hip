// gdm_rk.hip -- device-resident explicit Runge-Kutta stages.
//
// The reference evolves y = (block(0), block(1)) with
// TimeStepping::ExplicitRungeKutta (applications/advection/include/gdm/
// advection/problem.h:40-102, applications/wave/include/gdm/wave/problem.h:
// 280-346): per stage a new BlockVector (problem.h:64-65), k_i = f(t + c_i h,
// y + h sum_j a_ij k_j), then y += h sum_i b_i k_i, and block(0) (the boundary
// values at the face quadrature points) is reset to g(t_n) every step by
// initialize_time_step and evolved with dg/dt in the stages
// (advection/stiffness.h:181-194, 286-289).
//
// Here the RK state never leaves HBM:
//   * rk_update: acc_out = acc_in + beta k and (optionally) Y = y + alpha k in
//     one pass -- the low-storage form of a Butcher table with one nonzero
//     a_ij per stage (classic RK4): the b-sum is accumulated as the stages
//     are produced, in the same order as deal.II's final sadd loop;
//   * boundary functions: g(t) and dg/dt(t) of built-in analytic functions
//     evaluated at the boundary points straight from the face geometry
//     (coordinates computed from the point index, no coordinate array), so
//     no host evaluation and no H2D copy happen inside the RK loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>

#include "gdm_bcfn.h"
#include "gdm_kernels.h"
#include "gdm_rk.h"

namespace gdmk {

// RK stage update, 16 B per lane and array (double2): acc_out = acc_in +
// beta k and, with Y, Y = y + alpha k.  acc_in may alias acc_out (in-place
// accumulator).  Every access non-temporal (1 GB vectors at C3 only stream
// through the caches) and one pair per lane (grid = n / 512): 0.88 ms for the
// 5.4 GB of a C3 stage update against 1.11 ms with cached accesses and a
// 4096-block grid-stride loop (tools/rk_bench.hip, profiles/r3u).  The odd
// tail element, if any, is done by the first lane.  Host-checked: every
// pointer 16-B aligned.
// AY: acc_in == y (the first RK stage): one load serves both (8 B per entry less)
template <bool WITH_Y, bool AY = false>
__global__ void __launch_bounds__(256) rk_update2_kernel(int64_t n, double beta, const double *__restrict__ k,
                                                         const double *acc_in, double *acc_out, double alpha,
                                                         const double *y, double *__restrict__ Y) {
  using d2 = double __attribute__((ext_vector_type(2)));
  const int64_t n2 = n / 2, stride = (int64_t)gridDim.x * blockDim.x;
  const d2 *k2 = reinterpret_cast<const d2 *>(k), *a2 = reinterpret_cast<const d2 *>(acc_in);
  d2 *o2 = reinterpret_cast<d2 *>(acc_out);
  const d2 av = {alpha, alpha}, bv = {beta, beta};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
    const d2 ki = __builtin_nontemporal_load(k2 + i);
    const d2 ai = __builtin_nontemporal_load(a2 + i);
    // one FMA per update (the arithmetic of the x pass with the update fused, gdm_mass.hip)
    if (WITH_Y) {
      const d2 yi = AY ? ai : __builtin_nontemporal_load(reinterpret_cast<const d2 *>(y) + i);
      __builtin_nontemporal_store(__builtin_elementwise_fma(av, ki, yi), reinterpret_cast<d2 *>(Y) + i);
    }
    __builtin_nontemporal_store(__builtin_elementwise_fma(bv, ki, ai), o2 + i);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const double ki = k[n - 1];
    if (WITH_Y) Y[n - 1] = fma(alpha, ki, y[n - 1]);
    acc_out[n - 1] = fma(beta, ki, acc_in[n - 1]);
  }
}

// scalar form for unaligned vectors
__global__ void __launch_bounds__(256) rk_update_kernel(int64_t n, double beta, const double *__restrict__ k,
                                                        const double *acc_in, double *acc_out, double alpha,
                                                        const double *__restrict__ y, double *__restrict__ Y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (Y) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const double ki = k[i];
      acc_out[i] = fma(beta, ki, acc_in[i]);
      Y[i] = fma(alpha, ki, y[i]);
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
      acc_out[i] = fma(beta, k[i], acc_in[i]);
  }
}

// Separable functions: per face, the 1D factors along t0 / t1 / the normal
// are tabulated once (tab[slot][q] = (s, c); slot 2 = the normal coordinate),
// so a boundary point costs two table reads and a few multiplies instead of
// 2 * dim transcendental evaluations.
// all faces in one launch: grid (x, 3 slots, faces)
__global__ void __launch_bounds__(256) bc_table_kernel(BcGeom g, BcFace F, BcFn f, double t, double *tab, int ld) {
  const int slot = blockIdx.y;  // 0: t0, 1: t1, 2: normal
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < (slot < 2 ? F.Q[slot] : 1); q += gridDim.x * blockDim.x) {
    double s, c;
    bc_table_entry(g, F, f, t, slot, q, s, c);
    tab[((size_t)slot * ld + q) * 2] = s;
    tab[((size_t)slot * ld + q) * 2 + 1] = c;
  }
}

// every face's tables at t_g (blockIdx.z < n_faces) and t_k (the rest) in
// one launch: grid (x, 3 slots, n_faces or 2 n_faces); layout of BcStage::tab
__global__ void __launch_bounds__(256) bc_tables_kernel(BcGeom g, BcFn f, double t_g, double t_k, double *tab,
                                                        int ld) {
  const int slot = blockIdx.y, z = blockIdx.z;
  const int fi = z % g.n_faces, which = z / g.n_faces;
  const BcFace &F = g.face[fi];
  const double t = which ? t_k : t_g;
  double *tb = tab + (size_t)(which * BcStage::kMaxFaces + fi) * 3 * ld * 2;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < (slot < 2 ? F.Q[slot] : 1); q += gridDim.x * blockDim.x) {
    double s, c;
    bc_table_entry(g, F, f, t, slot, q, s, c);
    tb[((size_t)slot * ld + q) * 2] = s;
    tb[((size_t)slot * ld + q) * 2 + 1] = c;
  }
}

// one face: grid (ceil(Q0 / 256), Q1); i1 = blockIdx.y, i0 = lane index
__global__ void __launch_bounds__(256) bc_face_kernel(BcGeom g, BcFace F, BcFn f, BcSine w, double t,
                                                      int derivative, const double *__restrict__ tab, int ld,
                                                      double *out) {
  const int i1 = blockIdx.y;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= F.Q[0]) return;
  out[F.offset + (int64_t)i1 * F.Q[0] + i0] =
      f.kind == 2 ? bc_sine_point(tab, ld, w, i0, i1, derivative) : bc_point(g, F, f, tab, ld, i0, i1, derivative);
}

// Periodicity constraints of System::make_periodicity_constraints
// (include/gdm/system.h:427-463): vertex N_d - 1 of direction d is
// constrained to vertex 0.  mode 0 = distribute (v[i1] = v[i0]), mode 1 =
// condense a residual (v[i0] += v[i1], v[i1] = 0).  One thread per vertex of
// the face x_d = 0; global lexicographic layout (x fastest).
__global__ void __launch_bounds__(256) periodic_kernel(double *v, int64_t N0, int64_t N1, int64_t N2, int d,
                                                       int mode) {
  const int64_t N[3] = {N0, N1, N2};
  const int64_t stride[3] = {1, N0, N0 * N1};
  const int a = d == 0 ? 1 : 0, b = d == 2 ? 1 : 2;  // the two other directions
  const int64_t nf = N[a] * N[b];
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < nf; f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ia = f % N[a], ib = f / N[a];
    const int64_t i0 = ia * stride[a] + ib * stride[b];
    const int64_t i1 = i0 + (N[d] - 1) * stride[d];
    if (mode == 0) {
      v[i1] = v[i0];
    } else {
      v[i0] += v[i1];
      v[i1] = 0.0;
    }
  }
}

// x *= w elementwise (Jacobi preconditioner application, w = 1 / diag)
__global__ void __launch_bounds__(256) vmul_kernel(int64_t n, const double *__restrict__ w,
                                                   const double *__restrict__ x, double *__restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = w[i] * x[i];
}

// Interface correction of the distributed mass inverse (truncated SPIKE, see
// gdm_capi.cpp build_spike): one thread per line of the plane, the 2p
// interface unknowns of both slab edges in registers, then a rank-2p update
// of the line's planes.  The edge planes are read before any plane is written
// (one thread owns its line), so the update is in place.
//
// mode 1 (refinement round, thin slabs): instead of the update, the slab's
// edge planes g_first / g_last (saved to G0 [2p][ps] at round 0) are replaced
// by the right-hand sides of the next interface systems with the dropped
// far-spike couplings evaluated at the current interface values:
//   first p planes: g_first - V[0:p] t,  last p planes: g_last - W[n-p:n] b;
// the caller then exchanges ghost planes again.  mode 0 with G0 != NULL
// restores the saved edge planes before the update.  mode 2 = mode 0 and the
// interface unknowns b / t (the lower neighbour's last p planes, the upper
// neighbour's first p planes of x) also replace the ghost planes: x_local is
// then a valid local vector of x without another exchange (the one-exchange
// RK stage, gdm_mass_solve_interface_ghosts).
template <int P>
__global__ void __launch_bounds__(256) spike_kernel(double *x_local, int64_t ps, int64_t own_off, int n, int has_lo,
                                                    int has_hi, const double *__restrict__ VW,
                                                    const double *__restrict__ S, int k_begin, int k_end, int mode,
                                                    int round, double *__restrict__ G0) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ps; i += (int64_t)gridDim.x * blockDim.x) {
    double *xo = x_local + own_off + i;
    double b[P], t[P], in[2 * P];
#pragma unroll
    for (int j = 0; j < P; ++j) b[j] = t[j] = 0.0;
    if (has_lo) {
#pragma unroll
      for (int a = 0; a < P; ++a) {
        in[a] = xo[(int64_t)(a - P) * ps];
        in[P + a] = xo[(int64_t)a * ps];
      }
#pragma unroll
      for (int j = 0; j < P; ++j) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < 2 * P; ++c) s = fma(S[j * 2 * P + c], in[c], s);
        b[j] = s;
      }
    }
    if (has_hi) {
#pragma unroll
      for (int a = 0; a < P; ++a) {
        in[a] = xo[(int64_t)(n - P + a) * ps];
        in[P + a] = xo[(int64_t)(n + a) * ps];
      }
#pragma unroll
      for (int j = 0; j < P; ++j) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < 2 * P; ++c) s = fma(S[2 * P * P + j * 2 * P + c], in[c], s);
        t[j] = s;
      }
    }
    if (mode == 1) {
      // every load of the line's edge planes first, then the stores: one
      // memory latency per line instead of one per plane (the compiler keeps
      // loads behind stores to the same array)
      double gf[P], gl[P];
#pragma unroll
      for (int a = 0; a < P; ++a) {
        if (round == 0) {
          gf[a] = xo[(int64_t)a * ps];
          gl[a] = xo[(int64_t)(n - P + a) * ps];
        } else {
          gf[a] = G0[(int64_t)a * ps + i];
          gl[a] = G0[(int64_t)(P + a) * ps + i];
        }
      }
      if (round == 0) {
#pragma unroll
        for (int a = 0; a < P; ++a) {
          G0[(int64_t)a * ps + i] = gf[a];
          G0[(int64_t)(P + a) * ps + i] = gl[a];
        }
      }
#pragma unroll
      for (int a = 0; a < P; ++a) {
        const double *vf = VW + (size_t)a * 2 * P, *wl = VW + (size_t)(n - P + a) * 2 * P + P;
        double f = gf[a], l = gl[a];
#pragma unroll
        for (int j = 0; j < P; ++j) {
          f = fma(-vf[j], t[j], f);
          l = fma(-wl[j], b[j], l);
        }
        xo[(int64_t)a * ps] = f;
        xo[(int64_t)(n - P + a) * ps] = l;
      }
      continue;
    }
    if (G0) {
#pragma unroll
      for (int a = 0; a < P; ++a) {
        xo[(int64_t)a * ps] = G0[(int64_t)a * ps + i];
        xo[(int64_t)(n - P + a) * ps] = G0[(int64_t)(P + a) * ps + i];
      }
    }
    if (mode == 2) {
#pragma unroll
      for (int a = 0; a < P; ++a) {
        if (has_lo) xo[(int64_t)(a - P) * ps] = b[a];
        if (has_hi) xo[(int64_t)(n + a) * ps] = t[a];
      }
    }
    // the correction in blocks of KB planes: the block's loads are issued
    // together (one memory latency per block, not per plane)
    constexpr int KB = 8;
    for (int k0 = k_begin; k0 < k_end; k0 += KB) {
      double xv[KB];
#pragma unroll
      for (int u = 0; u < KB; ++u)
        if (k0 + u < k_end) xv[u] = xo[(int64_t)(k0 + u) * ps];
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        if (k0 + u < k_end) {
          const double *vw = VW + (size_t)(k0 + u) * 2 * P;
          double c = 0.0;
#pragma unroll
          for (int j = 0; j < P; ++j) c = fma(vw[j], t[j], c);
#pragma unroll
          for (int j = 0; j < P; ++j) c = fma(vw[P + j], b[j], c);
          xo[(int64_t)(k0 + u) * ps] = xv[u] - c;
        }
      }
    }
  }
}

// The interface correction fused with the RK stage update of the one-exchange
// stage (gdm_mass_solve_interface_rk): for every plane of the local layout the
// stage derivative k -- b / t (spike_kernel mode 2) on the ghost planes below /
// above, g_k - V[k] t - W[k] b on the owned ones (g_k from G0 on the edge
// planes after refinement rounds) -- goes straight into acc_out = acc_in +
// beta k and Y = y + alpha k (local vectors, one FMA each as in
// rk_update2_kernel); k itself is not stored.  Grid: (line block, chunk of
// SRK_CH planes), laid out so that the chunks of a line block are 8 block ids
// apart: consecutive ids go to the 8 XCDs in turn, so all chunks of a line
// block run on one XCD, close in time, and their re-reads of the 2 x 2p edge
// planes behind b / t hit that XCD's L2 (chunk-fastest ids spread them over
// all eight L2s: 1.4x the kernel's algorithmic fetch, profiles/r6r).  A chunk
// computes b / t only when it needs them.  Planes in blocks of KB: one memory
// latency per block.
constexpr int SRK_CH = 16;
template <int P, bool WITH_Y>
__global__ void __launch_bounds__(256) spike_rk_kernel(const double *__restrict__ x_local, int64_t ps, int gb, int ga,
                                                       int n, int has_lo, int has_hi, const double *__restrict__ VW,
                                                       const double *__restrict__ S, int k_begin, int k_end,
                                                       const double *__restrict__ G0, const RkOut rk, int nch) {
  // block id = (lb / 8) * 8 nch + chunk * 8 + lb % 8
  const unsigned bid = blockIdx.x, g = bid / (8u * (unsigned)nch), rem = bid - g * 8u * (unsigned)nch;
  const int chunk = (int)(rem / 8u);
  const int64_t lb = (int64_t)g * 8 + (rem % 8u);
  const int64_t i = lb * blockDim.x + threadIdx.x;
  if (i >= ps) return;
  const int kb = -gb + chunk * SRK_CH, ke = min(n + ga, kb + SRK_CH);  // planes relative to the first owned one
  const bool corr = kb < k_end && k_begin < ke;
  const double *xo = x_local + (int64_t)gb * ps + i;
  double b[P], t[P], in[2 * P];
#pragma unroll
  for (int j = 0; j < P; ++j) b[j] = t[j] = 0.0;
  if (has_lo && (kb < 0 || corr)) {
#pragma unroll
    for (int a = 0; a < P; ++a) {
      in[a] = xo[(int64_t)(a - P) * ps];
      in[P + a] = xo[(int64_t)a * ps];
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < 2 * P; ++c) s = fma(S[j * 2 * P + c], in[c], s);
      b[j] = s;
    }
  }
  if (has_hi && (ke > n || corr)) {
#pragma unroll
    for (int a = 0; a < P; ++a) {
      in[a] = xo[(int64_t)(n - P + a) * ps];
      in[P + a] = xo[(int64_t)(n + a) * ps];
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < 2 * P; ++c) s = fma(S[2 * P * P + j * 2 * P + c], in[c], s);
      t[j] = s;
    }
  }
  constexpr int KB = 8;
  for (int k0 = kb; k0 < ke; k0 += KB) {
    double kv[KB], av[KB], yv[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int k = k0 + u;
      if (k < ke) {
        const int64_t e = (int64_t)(gb + k) * ps + i;
        av[u] = __builtin_nontemporal_load(rk.acc_in + e);
        if (WITH_Y) yv[u] = __builtin_nontemporal_load(rk.y + e);
        if ((k < 0 && !has_lo) || (k >= n && !has_hi)) {
          kv[u] = xo[(int64_t)k * ps];  // a ghost plane the interface leaves alone
        } else if (k >= 0 && k < n) {
          if (G0 && k < P)
            kv[u] = G0[(int64_t)k * ps + i];
          else if (G0 && k >= n - P)
            kv[u] = G0[(int64_t)(P + k - (n - P)) * ps + i];
          else
            kv[u] = xo[(int64_t)k * ps];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int k = k0 + u;
      if (k < ke) {
        double kval;
        if (k < 0 && has_lo) {
          kval = b[k + P];
        } else if (k >= n && has_hi) {
          kval = t[k - n];
        } else if (k < 0 || k >= n) {
          kval = kv[u];
        } else {
          kval = kv[u];
          if (k >= k_begin && k < k_end) {
            const double *vw = VW + (size_t)k * 2 * P;
            double c = 0.0;
#pragma unroll
            for (int j = 0; j < P; ++j) c = fma(vw[j], t[j], c);
#pragma unroll
            for (int j = 0; j < P; ++j) c = fma(vw[P + j], b[j], c);
            kval = kval - c;
          }
        }
        const int64_t e = (int64_t)(gb + k) * ps + i;
        if (WITH_Y) __builtin_nontemporal_store(fma(rk.alpha, kval, yv[u]), rk.Y + e);
        __builtin_nontemporal_store(fma(rk.beta, kval, av[u]), rk.acc_out + e);
      }
    }
  }
}

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_spike_rk(int p, const double *x_local, int64_t ps, int gb, int ga, int n,
                                          int has_lo, int has_hi, const double *VW, const double *S, int k_begin,
                                          int k_end, const double *G0, const gdmk::RkOut &rk, hipStream_t st) {
  if (ps <= 0 || n + gb + ga <= 0) return hipSuccess;
  const int nch = (n + gb + ga + gdmk::SRK_CH - 1) / gdmk::SRK_CH;
  const int64_t nb = ((ps + 255) / 256 + 7) / 8 * 8 * nch;  // line blocks padded to a multiple of 8
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)nb;
#define GDM_SPIKE_RK(PP)                                                                                        \
  case PP:                                                                                                      \
    if (rk.Y)                                                                                                   \
      hipLaunchKernelGGL((gdmk::spike_rk_kernel<PP, true>), dim3(blocks), dim3(256), 0, st, x_local, ps, gb, ga, \
                         n, has_lo, has_hi, VW, S, k_begin, k_end, G0, rk, nch);                                \
    else                                                                                                        \
      hipLaunchKernelGGL((gdmk::spike_rk_kernel<PP, false>), dim3(blocks), dim3(256), 0, st, x_local, ps, gb,   \
                         ga, n, has_lo, has_hi, VW, S, k_begin, k_end, G0, rk, nch);                            \
    break;
  switch (p) {
    GDM_SPIKE_RK(1)
    GDM_SPIKE_RK(2)
    GDM_SPIKE_RK(3)
    GDM_SPIKE_RK(4)
    GDM_SPIKE_RK(5)
    GDM_SPIKE_RK(6)
    GDM_SPIKE_RK(7)
    GDM_SPIKE_RK(8)
    GDM_SPIKE_RK(9)
    default: return hipErrorInvalidValue;
  }
#undef GDM_SPIKE_RK
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_spike(int p, double *x_local, int64_t ps, int64_t own_off, int n, int has_lo,
                                       int has_hi, const double *VW, const double *S, int k_begin, int k_end,
                                       int mode, int round, double *G0, hipStream_t st) {
  if (ps <= 0 || (mode == 0 && !G0 && k_end <= k_begin)) return hipSuccess;
  if (mode == 2 && !has_lo && !has_hi && !G0 && k_end <= k_begin) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<int64_t>((ps + 255) / 256, 4096);
#define GDM_SPIKE(PP)                                                                                           \
  case PP:                                                                                                      \
    hipLaunchKernelGGL(gdmk::spike_kernel<PP>, dim3(blocks), dim3(256), 0, st, x_local, ps, own_off, n, has_lo, \
                       has_hi, VW, S, k_begin, k_end, mode, round, G0);                                         \
    break;
  switch (p) {
    GDM_SPIKE(1)
    GDM_SPIKE(2)
    GDM_SPIKE(3)
    GDM_SPIKE(4)
    GDM_SPIKE(5)
    GDM_SPIKE(6)
    GDM_SPIKE(7)
    GDM_SPIKE(8)
    GDM_SPIKE(9)
    default: return hipErrorInvalidValue;
  }
#undef GDM_SPIKE
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_rk_update(int64_t n, double beta, const double *k, const double *acc_in,
                                           double *acc_out, double alpha, const double *y, double *Y,
                                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  auto al16 = [](const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (al16(k) && al16(acc_in) && al16(acc_out) && (!Y || (al16(y) && al16(Y)))) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n / 2 + 255) / 256, (int64_t)1 << 30));
    if (Y && y == acc_in)
      hipLaunchKernelGGL((gdmk::rk_update2_kernel<true, true>), dim3((unsigned)blocks), dim3(256), 0, st, n, beta, k,
                         acc_in, acc_out, alpha, y, Y);
    else if (Y)
      hipLaunchKernelGGL(gdmk::rk_update2_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, n, beta, k, acc_in,
                         acc_out, alpha, y, Y);
    else
      hipLaunchKernelGGL(gdmk::rk_update2_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, n, beta, k, acc_in,
                         acc_out, alpha, y, Y);
    return hipGetLastError();
  }
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(gdmk::rk_update_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, beta, k, acc_in, acc_out,
                     alpha, y, Y);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_bc_eval(const gdmk::BcGeom &g, const gdmk::BcFn &f, double t, int derivative,
                                         double *out, double *tab, int ld, hipStream_t st) {
  for (int fi = 0; fi < g.n_faces; ++fi) {
    const gdmk::BcFace &F = g.face[fi];
    if ((int64_t)F.Q[0] * F.Q[1] <= 0) continue;
    if (f.kind == 2) {
      hipLaunchKernelGGL(gdmk::bc_table_kernel, dim3((unsigned)((ld + 255) / 256), 3), dim3(256), 0, st, g, F, f, t,
                         tab + (size_t)fi * 3 * ld * 2, ld);
    }
    hipLaunchKernelGGL(gdmk::bc_face_kernel, dim3((unsigned)((F.Q[0] + 255) / 256), (unsigned)F.Q[1]), dim3(256), 0,
                       st, g, F, f, gdmk::bc_sine_weights(f, F), t, derivative, tab + (size_t)fi * 3 * ld * 2, ld, out);
  }
  return hipGetLastError();
}

namespace gdmk {
// the faces to fill (kinds 2 and 0), compact per-face sources resolved on the
// host: the kernel reads them from the argument block by blockIdx.z (scalar
// loads, no private copy)
struct BcFillSet {
  BcStageFace fc[BcStage::kMaxFaces];
  int64_t offset[BcStage::kMaxFaces];
  int Q0[BcStage::kMaxFaces], Q1[BcStage::kMaxFaces];
};
// one face per blockIdx.z, lane = t0 point (coalesced table reads and writes)
__global__ void __launch_bounds__(256) bc_stage_fill_kernel(const BcFillSet set, double *out) {
  const int f = blockIdx.z, i1 = blockIdx.y, i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int q0 = set.Q0[f];
  if (i0 >= q0 || i1 >= set.Q1[f]) return;
  out[set.offset[f] + (int64_t)i1 * q0 + i0] = bc_stage_face_value(set.fc[f], i0, i1);
}
// GDM_FN_CONE (any geometry; small meshes): the generic evaluation, one face
__global__ void __launch_bounds__(256) bc_stage_fill_generic_kernel(BcStage s, double *out) {
  const BcFace &F = s.g.face[s.face];
  const int i1 = blockIdx.y, i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= F.Q[0]) return;
  out[F.offset + (int64_t)i1 * F.Q[0] + i0] = bc_stage_value(s, i0, i1);
}
}  // namespace gdmk

extern "C" hipError_t gdmk_launch_bc_stage_fill(const gdmk::BcStage &s, const int *faces, int n, double *out,
                                               hipStream_t st) {
  using namespace gdmk;
  if (n <= 0) return hipSuccess;
  if (n > BcStage::kMaxFaces) return hipErrorInvalidValue;
  if (s.f.kind == 1) {
    for (int i = 0; i < n; ++i) {
      BcStage one = s;
      one.face = faces[i];
      const BcFace &F = s.g.face[faces[i]];
      if ((int64_t)F.Q[0] * F.Q[1] <= 0) continue;
      hipLaunchKernelGGL(bc_stage_fill_generic_kernel, dim3((unsigned)((F.Q[0] + 255) / 256), (unsigned)F.Q[1]),
                         dim3(256), 0, st, one, out);
    }
    return hipGetLastError();
  }
  BcFillSet set{};
  int q0 = 0, q1 = 0;
  for (int i = 0; i < n; ++i) {
    const int fi = faces[i];
    const BcFace &F = s.g.face[fi];
    BcStageFace &c = set.fc[i];
    c.tg = s.tab + (size_t)fi * 3 * s.ld * 2;
    c.tk = s.tab + (size_t)(BcStage::kMaxFaces + fi) * 3 * s.ld * 2;
    c.ld = s.ld;
    c.kind = s.f.kind;
    c.w = bc_sine_weights(s.f, F);
    c.alpha = s.alpha;
    c.c = s.f.prm[0];
    set.offset[i] = F.offset;
    set.Q0[i] = F.Q[0];
    set.Q1[i] = F.Q[1];
    q0 = std::max(q0, F.Q[0]);
    q1 = std::max(q1, F.Q[1]);
  }
  if (q0 <= 0 || q1 <= 0) return hipSuccess;
  hipLaunchKernelGGL(bc_stage_fill_kernel, dim3((unsigned)((q0 + 255) / 256), (unsigned)q1, (unsigned)n), dim3(256), 0,
                     st, set, out);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_bc_tables(const gdmk::BcGeom &g, const gdmk::BcFn &f, double t_g, double t_k,
                                            int with_k, double *tab, int ld, hipStream_t st) {
  if (f.kind != 2 || g.n_faces <= 0) return hipSuccess;
  if (g.n_faces > gdmk::BcStage::kMaxFaces) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gdmk::bc_tables_kernel, dim3((unsigned)((ld + 255) / 256), 3, (unsigned)(g.n_faces * (with_k ? 2 : 1))),
                     dim3(256), 0, st, g, f, t_g, t_k, tab, ld);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_periodic(double *v, const int64_t N[3], int d, int mode, hipStream_t st) {
  const int a = d == 0 ? 1 : 0, b = d == 2 ? 1 : 2;
  const int64_t nf = N[a] * N[b];
  const int64_t blocks = std::min<int64_t>((nf + 255) / 256, 4096);
  hipLaunchKernelGGL(gdmk::periodic_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, v, N[0],
                     N[1], N[2], d, mode);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_vmul(int64_t n, const double *w, const double *x, double *y, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(gdmk::vmul_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, w, x, y);
  return hipGetLastError();
}
