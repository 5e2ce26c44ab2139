// gdm_post.h -- argument block and launcher of gdm_post.hip (device error norms)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gdm_rk.h"  // BcFn: the built-in analytic functions

namespace gdmk {

// Owned cell box and the local-vector addressing of the DoF boxes.  Absent
// directions (d >= dim): ncell = 1, cb = 0, ce = 1, nb = nq = 1.
struct ErrGeom {
  int dim, p;
  int ncell[3];       // cells per direction (global)
  int cb[3], ce[3];   // owned cell range per direction
  int nb[3], nq[3];   // DoF box width / quadrature points per direction
  int64_t N0, N1;     // vertices along x, y (global lexicographic index)
  int64_t base;       // global index of local entry 0
  double lo[3], h[3];
  double jxw;         // prod_d h_d
  double xq[10], wq[10];  // QGauss(p+1) on [0, 1]
};

}  // namespace gdmk

extern "C" {
size_t gdmk_error_norms_lds_bytes(int p, int dim);
// S: [max(1, p)][p+1][p+1] shape values phi^cat_i(xq_q); out3 (device) =
// (Linf, L1, L2^2) of the owned cells; partial: 3 * n_partial doubles
hipError_t gdmk_launch_error_norms(const gdmk::ErrGeom &g, const gdmk::BcFn &f, double t, const double *S,
                                   const double *u, double *cell_err, double *partial, int n_partial, double *out3,
                                   hipStream_t st);
}
