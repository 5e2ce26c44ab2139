// gdm_setup.cpp -- host-side setup of the GDM operator engine (see gdm_setup.h).
#include "gdm_setup.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <utility>

namespace gdm {

void gauss_unit(int n, std::vector<double> &x, std::vector<double> &w) {
  // Newton iteration on the Legendre polynomial P_n, started from the
  // asymptotic root estimate; deal.II's QGauss gives the same rule.
  x.assign(n, 0.0);
  w.assign(n, 0.0);
  const double pi = 3.14159265358979323846;
  for (int r = 0; r < n; ++r) {
    double t = std::cos(pi * (r + 0.75) / (n + 0.5));
    double dp = 1.0;
    for (int it = 0; it < 200; ++it) {
      double p0 = 1.0, p1 = t;
      for (int k = 2; k <= n; ++k) {
        const double pk = ((2 * k - 1) * t * p1 - (k - 1) * p0) / k;
        p0 = p1;
        p1 = pk;
      }
      if (n == 1) { p1 = t; p0 = 1.0; }
      dp = n * (t * p1 - p0) / (t * t - 1.0);
      const double dt = p1 / dp;
      t -= dt;
      if (std::abs(dt) < 1e-17) break;
    }
    double p0 = 1.0, p1 = t;
    for (int k = 2; k <= n; ++k) {
      const double pk = ((2 * k - 1) * t * p1 - (k - 1) * p0) / k;
      p0 = p1;
      p1 = pk;
    }
    if (n == 1) { p1 = t; p0 = 1.0; }
    dp = n * (t * p1 - p0) / (t * t - 1.0);
    x[r] = 0.5 * (1.0 - t);  // r = 0 is the largest root -> smallest x
    w[r] = 1.0 / ((1.0 - t * t) * dp * dp);
  }
}

double shape_1d(int p, int cat, int i, double x, int d) {
  // Expand prod_{j != i} (x - t_j) / (t_i - t_j) into monomials, then
  // differentiate d times and evaluate with Horner (the reference stores the
  // same polynomials as monomial coefficient tables, fe.h:323-333).
  std::vector<double> c(p + 2, 0.0);
  c[0] = 1.0;
  int deg = 0;
  double denom = 1.0;
  for (int j = 0; j <= p; ++j) {
    if (j == i) continue;
    const double tj = double(j - cat);
    for (int k = deg + 1; k >= 1; --k) c[k] = c[k - 1] - tj * c[k];
    c[0] *= -tj;
    ++deg;
    denom *= double(i - j);
  }
  for (int k = 0; k <= deg; ++k) c[k] /= denom;
  for (int o = 0; o < d; ++o) {
    for (int k = 0; k < deg; ++k) c[k] = c[k + 1] * double(k + 1);
    --deg;
  }
  if (deg < 0) return 0.0;
  double r = c[deg];
  for (int k = deg - 1; k >= 0; --k) r = r * x + c[k];
  return r;
}

unsigned category(unsigned cell, unsigned p, unsigned n_cells) {
  const unsigned half = p / 2;
  if (cell < half) return cell;
  if (cell < n_cells - half) return half;
  return p + cell - n_cells;
}

unsigned box_offset(unsigned cell, unsigned p, unsigned n_cells) {
  const unsigned half = p / 2;
  if (cell < half) return 0;
  return std::min(n_cells, cell + half + 1) - p;
}

Matrices1D assemble_1d(int p, unsigned n_cells, double h) {
  if (n_cells < (unsigned)p) throw std::invalid_argument("n_subdivisions must be >= fe_degree");
  const int n1 = p + 1, N = int(n_cells) + 1;
  Matrices1D m{Band(N, p), Band(N, p), Band(N, p)};
  std::vector<double> xq, wq;
  gauss_unit(n1, xq, wq);
  const int ncat = std::max(1, p);
  // per category: values and derivatives at the quadrature points
  std::vector<double> val((size_t)ncat * n1 * n1), der((size_t)ncat * n1 * n1);
  for (int cat = 0; cat < ncat; ++cat)
    for (int i = 0; i < n1; ++i)
      for (int q = 0; q < n1; ++q) {
        val[((size_t)cat * n1 + i) * n1 + q] = shape_1d(p, cat, i, xq[q], 0);
        der[((size_t)cat * n1 + i) * n1 + q] = shape_1d(p, cat, i, xq[q], 1) / h;
      }
  for (unsigned c = 0; c < n_cells; ++c) {
    const int cat = int(category(c, p, n_cells));
    const int off = int(box_offset(c, p, n_cells));
    const double *v = &val[(size_t)cat * n1 * n1];
    const double *g = &der[(size_t)cat * n1 * n1];
    for (int i = 0; i < n1; ++i)
      for (int j = 0; j < n1; ++j) {
        double mm = 0, cc = 0, ll = 0;
        for (int q = 0; q < n1; ++q) {
          const double jxw = wq[q] * h;
          mm += v[i * n1 + q] * v[j * n1 + q] * jxw;
          cc += g[i * n1 + q] * v[j * n1 + q] * jxw;
          ll += g[i * n1 + q] * g[j * n1 + q] * jxw;
        }
        m.M(off + i, off + j) += mm;
        m.C(off + i, off + j) += cc;
        m.L(off + i, off + j) += ll;
      }
  }
  return m;
}

void cholesky_band(const Band &M, std::vector<double> &lrow, std::vector<double> &inv_diag) {
  const int n = M.n, hb = M.hb, wl = hb + 1;
  lrow.assign((size_t)n * wl, 0.0);
  inv_diag.assign(n, 0.0);
  auto Lij = [&](int i, int j) -> double & { return lrow[(size_t)i * wl + (j - i + hb)]; };
  for (int i = 0; i < n; ++i) {
    for (int j = std::max(0, i - hb); j <= i; ++j) {
      double s = M(i, j);
      for (int k = std::max(0, i - hb); k < j; ++k) s -= Lij(i, k) * Lij(j, k);
      if (j == i) {
        if (s <= 0.0) throw std::runtime_error("mass matrix not positive definite");
        Lij(i, i) = std::sqrt(s);
        inv_diag[i] = 1.0 / Lij(i, i);
      } else {
        Lij(i, j) = s / Lij(j, j);
      }
    }
  }
}

FaceTable face_table_1d(int p, unsigned n_cells, double h, unsigned cell_begin, unsigned cell_end) {
  FaceTable t;
  const int n1 = p + 1;
  const unsigned N = n_cells + 1;
  t.n_nodes = int(N);
  t.qstart.assign(N, 0);
  t.qcount.assign(N, 0);
  // A node near a wall lies in the boxes of up to p + p/2 + 1 cells (the
  // first p/2 + 1 cells all use the box [0, p], system.h:228-233), so the row
  // width is the largest count, not (p + 1)^2.
  std::vector<std::pair<unsigned, unsigned>> range(N, {1u, 0u});
  int maxc = 1;
  for (unsigned i = 0; i < N; ++i) {
    unsigned first = ~0u, last = 0;
    for (unsigned c = cell_begin; c < cell_end; ++c) {
      const unsigned off = box_offset(c, p, n_cells);
      if (i < off || i > off + unsigned(p)) continue;
      first = std::min(first, c);
      last = std::max(last, c);
    }
    if (first != ~0u) {
      range[i] = {first, last};
      maxc = std::max(maxc, int(last - first + 1));
    }
  }
  t.wmax = maxc * n1;
  t.w.assign((size_t)N * t.wmax, 0.0);
  std::vector<double> xq, wq;
  gauss_unit(n1, xq, wq);
  for (unsigned i = 0; i < N; ++i) {
    if (range[i].first > range[i].second) continue;
    int m = 0;
    for (unsigned c = range[i].first; c <= range[i].second; ++c) {
      const unsigned off = box_offset(c, p, n_cells);
      const int cat = int(category(c, p, n_cells));
      for (int q = 0; q < n1; ++q)
        t.w[(size_t)i * t.wmax + m++] = shape_1d(p, cat, int(i - off), xq[q], 0) * wq[q] * h;
    }
    t.qstart[i] = int(range[i].first - cell_begin) * n1;
    t.qcount[i] = m;
  }
  return t;
}

Slab slab_partition(unsigned n_cells_last, unsigned n_ranks, unsigned rank) {
  const unsigned stride = (n_cells_last + n_ranks - 1) / n_ranks;
  Slab s;
  s.plane_begin = std::min(rank == 0 ? 0u : stride * rank + 1, n_cells_last + 1);
  s.plane_end = std::min(stride * (rank + 1) + 1, n_cells_last + 1);
  s.cell_begin = std::min(stride * rank, n_cells_last);
  s.cell_end = std::min(stride * (rank + 1), n_cells_last);
  return s;
}

}  // namespace gdm
