// gdm_cut.h -- shared host pieces of the 2D cut-cell assembly (gdm_cut.cpp:
// cut Poisson, gdm_cut_advection.cpp: cut advection): the FE_Q(1) cell level
// set, deal.II's QuadratureGenerator (Saye) on the unit cell, 1D shapes.
#pragma once

#include <vector>

#include "gdm_setup.h"

namespace gdm {

enum { INSIDE = -1, INTERSECTED = 0, OUTSIDE = 1 };

struct Bilinear {
  double a, b, c, d;  // f(s, t) = a + b s + c t + d s t on the unit square
  double operator()(double s, double t) const { return a + b * s + c * t + d * s * t; }
  double gs(double t) const { return b + d * t; }
  double gt(double s) const { return c + d * s; }
};

struct QPoint {
  double s, t, w;
};
struct SPoint {
  double s, t, w, nx, ny;
};

// root in (0, 1) of the linear function with values f0 at 0 and f1 at 1, or -1
inline double linear_root(double f0, double f1) {
  if ((f0 < 0.0 && 0.0 < f1) || (f1 < 0.0 && 0.0 < f0)) return f0 / (f0 - f1);
  return -1.0;
}

// inside (f < 0) and surface quadrature of the unit cell for one bilinear
// level set (reference measure; surface normal = grad f / |grad f|)
void saye_unit(const Bilinear &f, const std::vector<double> &qx, const std::vector<double> &qw,
               std::vector<QPoint> &inside, std::vector<SPoint> &surface);

struct Shapes {
  // values / reference derivatives of the p+1 1D shapes at a point
  double v[16], d[16];
};

inline void shapes_1d(int p, int cat, double x, Shapes &out) {
  for (int i = 0; i <= p; ++i) {
    out.v[i] = shape_1d(p, cat, i, x, 0);
    out.d[i] = shape_1d(p, cat, i, x, 1);
  }
}

}  // namespace gdm
