// gdm_rk.h -- device-side argument blocks and launchers of gdm_rk.hip
// (device-resident RK stage updates, boundary-function evaluation,
// periodicity constraints and the vector kernels of the matrix-free CG).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

namespace gdmk {

// Boundary-point geometry for device evaluation of boundary functions
// (gdm_rk.hip): the device block(0) order, face by face, [q_t1][q_t0].
struct BcFace {
  int64_t offset;     // first point of the face in the bc array
  int Q[2];           // points along t0, t1
  int dim_index[2];   // reference directions of t0, t1 (-1 = trivial)
  int cell_begin[2];  // first local cell along t0, t1
  int d, side;        // normal direction, 0 = lo / 1 = hi
};
struct BcGeom {
  int dim, p, n_faces;
  int64_t n_points;
  int n_sub[3];
  double lo[3], hi[3];
  double xq[10];  // QGauss(p+1) points on [0, 1]
  BcFace face[6];
};
// built-in boundary functions (include/gdm_hip.h gdm_fn_kind)
struct BcFn {
  int kind, dim;
  double prm[12];
};
// GDM_FN_SINE_PRODUCT's d/dt weights of one face: P = -2 pi k_e a_e of its t0,
// t1 and normal directions (has0 / has1: t0 / t1 non-trivial); the same host
// arithmetic feeds the stored (bc_face_kernel) and the in-kernel evaluation
struct BcSine {
  double P0, P1, Pn;
  int has0, has1;
};
__host__ __device__ inline BcSine bc_sine_weights(const BcFn &f, const BcFace &F) {
  auto P = [&](int e) { return -2.0 * M_PI * f.prm[3 + e] * f.prm[e]; };
  BcSine w{};
  w.has0 = F.dim_index[0] >= 0;
  w.has1 = F.dim_index[1] >= 0;
  w.P0 = w.has0 ? P(F.dim_index[0]) : 0.0;
  w.P1 = w.has1 ? P(F.dim_index[1]) : 0.0;
  w.Pn = P(F.d);
  return w;
}
// the compact stage source of one face for GDM_FN_SINE_PRODUCT / GDM_FN_CONSTANT
// (no geometry: the per-point work is four table reads and a few multiplies)
struct BcStageFace {
  const double *tg, *tk;  // the face's [3][ld][2] factor tables at t_g, t_k
  int ld, kind;
  BcSine w;
  double alpha, c;  // c: GDM_FN_CONSTANT's value
};
// the RK stage boundary values of one face, evaluated where they are read
// (gdm_apply_bc_fn): y + alpha k with y = g(t_g), k = dg/dt(t_k); tab =
// [2][kMaxFaces][3][ld][2] factor tables at t_g, then at t_k (bc_tables_kernel)
struct BcStage {
  static constexpr int kMaxFaces = 6;
  BcGeom g;
  BcFn f;
  const double *tab;
  int ld, face;
  double alpha;
};

}  // namespace gdmk

namespace gdmk {
struct RkOut;  // gdm_kernels.h
}

extern "C" {
// gdm_rk.hip: acc_out = acc_in + beta k; Y = y + alpha k (Y may be NULL)
hipError_t gdmk_launch_rk_update(int64_t n, double beta, const double *k, const double *acc_in, double *acc_out,
                                 double alpha, const double *y, double *Y, hipStream_t st);
// periodicity constraints along direction d (global layout): mode 0
// distribute v[last] = v[first], mode 1 condense v[first] += v[last], v[last] = 0
hipError_t gdmk_launch_periodic(double *v, const int64_t N[3], int d, int mode, hipStream_t st);
// distributed mass inverse, interface correction (gdm_mass_solve_interface):
// per line i of the plane, b = S_lo [ghost below (p planes); owned bottom p],
// t = S_hi [owned top p; ghost above (p planes)], then for owned planes k in
// [k_begin, k_end): x_k -= VW[k][0:p] . t + VW[k][p:2p] . b (mode 0; G0 != NULL:
// the saved edge planes are restored first).  mode 1 (refinement round):
// the owned first / last p planes become g_first - V[0:p] t / g_last - W[n-p:n] b
// with g saved to G0 [2p][plane_size] at round 0.  mode 2: mode 0, and b / t
// overwrite the ghost planes below / above (the neighbours' edge planes of x)
// the interface correction fused with the one-exchange RK stage update
// (gdm_mass_solve_interface_rk): k of every local plane -> acc_out = acc_in +
// beta k, Y = y + alpha k (rk.Y may be NULL); x_local is only read
hipError_t gdmk_launch_spike_rk(int p, const double *x_local, int64_t plane_size, int ghost_below, int ghost_above,
                                int n_planes, int has_lo, int has_hi, const double *VW, const double *S, int k_begin,
                                int k_end, const double *G0, const gdmk::RkOut &rk, hipStream_t st);
hipError_t gdmk_launch_spike(int p, double *x_local, int64_t plane_size, int64_t own_off, int n_planes, int has_lo,
                             int has_hi, const double *VW, const double *S, int k_begin, int k_end, int mode,
                             int round, double *G0, hipStream_t st);
// y = w .* x
hipError_t gdmk_launch_vmul(int64_t n, const double *w, const double *x, double *y, hipStream_t st);
// tab: scratch of n_faces * 3 * ld * 2 doubles, ld >= max(Q0, Q1)
hipError_t gdmk_launch_bc_eval(const gdmk::BcGeom &g, const gdmk::BcFn &f, double t, int derivative, double *out,
                               double *tab, int ld, hipStream_t st);
// the stage boundary values of BcStage into out (device block(0) order) for
// the n faces faces[0..n): out = g(t_g) + alpha dg/dt(t_k), tables ready
hipError_t gdmk_launch_bc_stage_fill(const gdmk::BcStage &s, const int *faces, int n, double *out, hipStream_t st);
// the factor tables of BcStage (kind 2; nothing to do otherwise): every face
// at t_g and, with_k, at t_k, one launch; tab holds 2 * 6 * 3 * ld * 2 doubles
hipError_t gdmk_launch_bc_tables(const gdmk::BcGeom &g, const gdmk::BcFn &f, double t_g, double t_k, int with_k,
                                 double *tab, int ld, hipStream_t st);
}
