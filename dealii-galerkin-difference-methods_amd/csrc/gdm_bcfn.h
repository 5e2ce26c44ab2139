// gdm_bcfn.h -- device evaluation of the built-in boundary functions
// (include/gdm_hip.h gdm_fn_kind) at the boundary points of one face, shared
// by the bc evaluation kernels (gdm_rk.hip, gdm_eval_boundary) and the face
// kernels of the inflow term (gdm_kernels.hip, gdm_apply_bc_fn), so both
// produce the same bits for the same point and time.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gdm_rk.h"

namespace gdmk {

// coordinate of quadrature point qi along face direction slot k (0 = t0, 1 = t1)
__device__ __forceinline__ double bc_slot_coord(const BcFace &F, const BcGeom &g, int k, int qi) {
  const int e = F.dim_index[k];
  const int n1 = g.p + 1;
  const int c = F.cell_begin[k] + qi / n1, qq = qi - (qi / n1) * n1;
  const double h = (g.hi[e] - g.lo[e]) / g.n_sub[e];
  return g.lo[e] + (c + g.xq[qq]) * h;
}

// separable factor of GDM_FN_SINE_PRODUCT in direction e at coordinate x:
// (s, c) = (sin, cos) of 2 pi k_e (x - a_e t) + phi_e
__device__ __forceinline__ void bc_sine_factor(const BcFn &f, int e, double x, double t, double &s, double &c) {
  const double arg = 2.0 * M_PI * f.prm[3 + e] * (x - f.prm[e] * t) + f.prm[6 + e];
  sincos(arg, &s, &c);
}

// entry q of table slot (0: t0, 1: t1, 2: the normal coordinate) of face F at time t
__device__ __forceinline__ void bc_table_entry(const BcGeom &g, const BcFace &F, const BcFn &f, double t, int slot,
                                               int q, double &s, double &c) {
  s = 1.0;
  c = 0.0;
  if (slot < 2 && F.dim_index[slot] >= 0)
    bc_sine_factor(f, F.dim_index[slot], bc_slot_coord(F, g, slot, q), t, s, c);
  else if (slot == 2)
    bc_sine_factor(f, F.d, F.side ? g.hi[F.d] : g.lo[F.d], t, s, c);
}

// g (derivative 0) or dg/dt (1) at point (i0, i1) of face F; tab = the face's
// [3][ld][2] factor table at the same time (kind 2 only)
__device__ __forceinline__ double bc_point(const BcGeom &g, const BcFace &F, const BcFn &f,
                                           const double *__restrict__ tab, int ld, int i0, int i1, int derivative) {
  if (f.kind == 0) return derivative ? 0.0 : f.prm[0];
  if (f.kind == 1) {  // cone max(0, r0 - |x - c|) (applications/advection/advection-app.cc:51-79), dg/dt = 0
    if (derivative) return 0.0;
    double x[3] = {0.0, 0.0, 0.0};
    x[F.d] = F.side ? g.hi[F.d] : g.lo[F.d];
    if (F.dim_index[0] >= 0) x[F.dim_index[0]] = bc_slot_coord(F, g, 0, i0);
    if (F.dim_index[1] >= 0) x[F.dim_index[1]] = bc_slot_coord(F, g, 1, i1);
    double r2 = 0.0;
    for (int d = 0; d < g.dim; ++d) r2 += (x[d] - f.prm[1 + d]) * (x[d] - f.prm[1 + d]);
    return fmax(0.0, f.prm[0] - sqrt(r2));
  }
  return 0.0;  // kind 2: bc_sine_point
}

// GDM_FN_SINE_PRODUCT at point (i0, i1) of a face from its factor table at the
// same time: prod_d sin(.) (trivial slots hold (1, 0)); d/dt = sum over the
// directions of P_e cos(.) * the other sines, added without contraction so the
// stored and the in-kernel evaluations round alike
__device__ __forceinline__ double bc_sine_point(const double *__restrict__ tab, int ld, const BcSine &w, int i0,
                                                int i1, int derivative) {
  const double s0 = tab[2 * i0], c0 = tab[2 * i0 + 1];
  const double s1 = tab[2 * ((size_t)ld + i1)], c1 = tab[2 * ((size_t)ld + i1) + 1];
  const double sn = tab[2 * (size_t)2 * ld], cn = tab[2 * (size_t)2 * ld + 1];
  if (!derivative) return s0 * s1 * sn;
  double r = 0.0;
  {
#pragma clang fp contract(off)
    if (w.has0) r = r + w.P0 * c0 * s1 * sn;
    if (w.has1) r = r + w.P1 * s0 * c1 * sn;
    r = r + w.Pn * s0 * s1 * cn;
  }
  asm volatile("" : "+v"(r));
  return r;
}

// the compact stage value (kinds 2 and 0): y + alpha k with y = g(t_g), k =
// dg/dt(t_k), as rk_update2_kernel forms Y (GDM_FN_CONSTANT: dg/dt = 0)
__device__ __forceinline__ double bc_stage_face_value(const BcStageFace &s, int i0, int i1) {
  if (s.kind == 0) return s.c;
  const double y = bc_sine_point(s.tg, s.ld, s.w, i0, i1, 0);
  if (s.alpha == 0.0) return y;
  return fma(s.alpha, bc_sine_point(s.tk, s.ld, s.w, i0, i1, 1), y);
}

// the stage boundary value Y = y + alpha k of the RK stages with y = g(t_g)
// and k = dg/dt(t_k) (alpha = 0: y), written as rk_update2_kernel writes Y
// (generic form, any kind; the face kernels use it for GDM_FN_CONE)
__device__ __forceinline__ double bc_stage_value(const BcStage &s, int i0, int i1) {
  const BcFace &F = s.g.face[s.face];
  const double *tg = s.tab + (size_t)s.face * 3 * s.ld * 2;
  const double *tk = s.tab + (size_t)(BcStage::kMaxFaces + s.face) * 3 * s.ld * 2;
  const BcSine w = bc_sine_weights(s.f, F);
  const double y = s.f.kind == 2 ? bc_sine_point(tg, s.ld, w, i0, i1, 0) : bc_point(s.g, F, s.f, tg, s.ld, i0, i1, 0);
  if (s.alpha == 0.0) return y;
  const double k = s.f.kind == 2 ? bc_sine_point(tk, s.ld, w, i0, i1, 1) : bc_point(s.g, F, s.f, tk, s.ld, i0, i1, 1);
  return fma(s.alpha, k, y);
}

}  // namespace gdmk
