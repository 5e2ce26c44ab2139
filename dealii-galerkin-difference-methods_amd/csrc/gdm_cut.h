// gdm_cut.h -- shared host pieces of the cut-cell assembly (gdm_cut.cpp:
// cut Poisson, gdm_cut_advection.cpp: cut advection, gdm_cut_wave.cpp: cut
// wave / heat): the FE_Q(1) and FE_Q(k) cell level sets, deal.II's
// QuadratureGenerator (Saye) on the unit cell, 1D shapes.
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

// FE_Q(k) level set of one cell in reference coordinates (k <= 9):
// f(s, t) = sum_ij C[i][j] s^i t^j, the tensor-product Lagrange interpolant
// of the values at the cell's Gauss-Lobatto support points
struct TensorPoly {
  int k = 1;
  double C[10][10] = {};
  // vals[a + (k + 1) b] = f(x_a, x_b) on the support points x (a along s)
  void interpolate(int k_, const double *vals, const std::vector<double> &support);
  double value(double s, double t) const;
  void derivatives(double s, double t, double &v, double g[2], double H[2][2]) const;
};

// Gauss-Lobatto points of n >= 2 points on [0, 1] (FE_Q support points)
std::vector<double> gauss_lobatto(int n);

// NonMatching::MeshClassifier of one cell: the Lagrange values mapped to the
// Bernstein basis of degree k (tensor product in 2D); all < 0 INSIDE, all > 0
// OUTSIDE, else INTERSECTED
int bernstein_location(int dim, int k, const double *vals, const std::vector<double> &support);

// QuadratureGenerator<2> (Saye) for a FE_Q(k) cell level set on the unit box,
// with deal.II's box splits / midpoint fallback; *n_splits counts splits;
// outside (when given) receives the f > 0 region's quadrature of the same pass
void saye_poly(const TensorPoly &f, const std::vector<double> &qx, const std::vector<double> &qw,
               std::vector<QPoint> &inside, std::vector<SPoint> &surface, int *n_splits,
               std::vector<QPoint> *outside = nullptr);

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
