// gdm_cut.cpp -- host assembly of the 2D cut-cell Poisson system of
// prototypes/cut_poisson_01_gdm.cc:148-323 (GDM degree p on a uniform
// n_sub x n_sub mesh, level set = FE_Q(1) interpolant of the signed distance
// to a circle, Nitsche boundary condition on the zero contour, optional ghost
// penalty), handed to the device SpMV / SolverCG (gdm_csr.hip) through the
// C ABI (include/gdm_hip.h, "Cut-cell systems").
//
// What it restates (reference paths; the same algorithm as the test oracle
// oracle/cut2d.py, which is pinned to prototypes/cut_poisson_01_gdm.output):
//   * NonMatching::MeshClassifier on the vertex values of the level set
//     (all < 0 inside, all > 0 outside, else intersected), :100-120
//   * NonMatching::FEValues quadrature: QGauss(p+1)^2 on inside cells; on
//     intersected cells deal.II's QuadratureGenerator (Saye) on the bilinear
//     cell level set: Taylor bounds over the box, the height direction with
//     the largest lower bound of |df/dx_i|, the cross-section split at the
//     roots of the bottom / top face restrictions, QGauss(p+1) per
//     sub-interval lifted along the height direction (inside segments get
//     QGauss(p+1), the root a surface point with weight w |grad f| / |f_h|)
//   * the local stiffness (grad v, grad u), Nitsche terms with
//     gamma = 5 (p+1) p and h = minimum_vertex_distance, rhs f v + Nitsche
//     data, ghost penalty 0.5 * gamma_g * h [d_n v][d_n u] on interior faces
//     with an intersected cell and a non-outside neighbour (visited from both
//     cells), zero diagonals -> 1, :148-323
//   * integrate_difference-style L2 error against the manufactured solution
//     u = g + f / (2 dim) (r^2 - |x - c|^2) over the inside quadrature, :349-405
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "gdm_cut.h"
#include "gdm_setup.h"

namespace gdm {

// deal.II QuadratureGenerator on the unit box for one bilinear level set
void saye_unit(const Bilinear &f, const std::vector<double> &qx, const std::vector<double> &qw,
               std::vector<QPoint> &inside, std::vector<SPoint> &surface) {
  inside.clear();
  surface.clear();
  // Taylor bounds at the centre (Hessian [[0, d], [d, 0]])
  const double val = f(0.5, 0.5), g0 = f.gs(0.5), g1 = f.gt(0.5), hd = std::fabs(f.d);
  const double spread = std::fabs(g0) * 0.5 + std::fabs(g1) * 0.5 + 0.5 * (2.0 * hd * 0.25);
  if (val - spread > 1e-11) return;  // definitely outside
  const int nq = (int)qx.size();
  if (val + spread < -1e-11) {       // definitely inside
    for (int b = 0; b < nq; ++b)
      for (int a = 0; a < nq; ++a) inside.push_back({qx[a], qx[b], qw[a] * qw[b]});
    return;
  }
  const double gb[2][2] = {{g0 - hd * 0.5, g0 + hd * 0.5}, {g1 - hd * 0.5, g1 + hd * 0.5}};
  double low[2];
  for (int i = 0; i < 2; ++i)
    low[i] = (gb[i][0] > 0.0 || gb[i][1] < 0.0) ? std::min(std::fabs(gb[i][0]), std::fabs(gb[i][1])) : 0.0;
  const int hdir = low[1] > low[0] ? 1 : 0;  // first of equal ones
  if (!(low[hdir] > 1e-11))
    throw std::runtime_error("cut quadrature: no height direction (box split / midpoint fallback not implemented)");
  auto fval = [&](double c, double h) { return hdir == 1 ? f(c, h) : f(h, c); };
  auto point = [&](double c, double h, double &s, double &t) {
    if (hdir == 1) {
      s = c;
      t = h;
    } else {
      s = h;
      t = c;
    }
  };
  double roots[2];
  int nr = 0;
  for (double hh : {0.0, 1.0}) {
    const double r = linear_root(fval(0.0, hh), fval(1.0, hh));
    if (r >= 0.0) roots[nr++] = r;
  }
  if (nr == 2 && roots[1] < roots[0]) std::swap(roots[0], roots[1]);
  double edges[4];
  int ne = 0;
  edges[ne++] = 0.0;
  for (int i = 0; i < nr; ++i) edges[ne++] = roots[i];
  edges[ne++] = 1.0;
  for (int e = 0; e + 1 < ne; ++e) {
    const double a = edges[e], L = edges[e + 1] - a;
    if (!(L > 0.0)) continue;
    for (int k = 0; k < nq; ++k) {
      const double c = a + L * qx[k], w = qw[k] * L;
      const double r = linear_root(fval(c, 0.0), fval(c, 1.0));
      double hs[3];
      int nh = 0;
      hs[nh++] = 0.0;
      if (r >= 0.0) hs[nh++] = r;
      hs[nh++] = 1.0;
      for (int g = 0; g + 1 < nh; ++g) {
        const double ha = hs[g], Lh = hs[g + 1] - ha;
        if (!(Lh > 0.0)) continue;
        if (fval(c, ha + 0.5 * Lh) < 0.0)
          for (int m = 0; m < nq; ++m) {
            double s, t;
            point(c, ha + Lh * qx[m], s, t);
            inside.push_back({s, t, w * qw[m] * Lh});
          }
      }
      if (r >= 0.0) {
        double s, t;
        point(c, r, s, t);
        const double gx = f.gs(t), gy = f.gt(s), ng = std::hypot(gx, gy);
        const double gh = hdir == 0 ? gx : gy;
        surface.push_back({s, t, w * ng / std::fabs(gh), gx / ng, gy / ng});
      }
    }
  }
}

std::vector<double> gauss_lobatto(int n) {
  // the roots of P'_{n-1} by Newton from the Chebyshev-Gauss-Lobatto guesses
  std::vector<double> x(n);
  x[0] = 0.0;
  x[n - 1] = 1.0;
  const int m = n - 1;
  for (int i = 1; i < m; ++i) {
    double t = -std::cos(M_PI * i / m);  // on [-1, 1]
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = t;
      for (int j = 2; j <= m; ++j) {
        const double p2 = ((2 * j - 1) * t * p1 - (j - 1) * p0) / j;
        p0 = p1;
        p1 = p2;
      }
      const double dp = m * (t * p1 - p0) / (t * t - 1.0);                  // P'_m
      const double d2p = (2.0 * t * dp - m * (m + 1) * p1) / (1.0 - t * t);  // P''_m
      const double dt = dp / d2p;
      t -= dt;
      if (std::fabs(dt) < 1e-16) break;
    }
    x[i] = 0.5 * (t + 1.0);
  }
  std::sort(x.begin(), x.end());
  return x;
}

namespace {

// monomial coefficients A[a][i] of the 1D Lagrange polynomials through x
void lagrange_monomials(const std::vector<double> &x, double A[10][10]) {
  const int n = (int)x.size();
  for (int a = 0; a < n; ++a) {
    double c[10] = {1.0};
    int deg = 0;
    double den = 1.0;
    for (int b = 0; b < n; ++b) {
      if (b == a) continue;
      // c *= (s - x_b)
      for (int i = deg + 1; i >= 0; --i) c[i] = (i > 0 ? c[i - 1] : 0.0) - x[b] * c[i];
      ++deg;
      den *= x[a] - x[b];
    }
    for (int i = 0; i < n; ++i) A[a][i] = c[i] / den;
  }
}

// inverse of a small dense matrix (Gauss-Jordan, partial pivoting)
void invert(int n, double M[10][10], double R[10][10]) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) R[i][j] = i == j ? 1.0 : 0.0;
  for (int c = 0; c < n; ++c) {
    int piv = c;
    for (int r = c + 1; r < n; ++r)
      if (std::fabs(M[r][c]) > std::fabs(M[piv][c])) piv = r;
    for (int j = 0; j < n; ++j) {
      std::swap(M[c][j], M[piv][j]);
      std::swap(R[c][j], R[piv][j]);
    }
    const double d = M[c][c];
    for (int j = 0; j < n; ++j) {
      M[c][j] /= d;
      R[c][j] /= d;
    }
    for (int r = 0; r < n; ++r) {
      if (r == c || M[r][c] == 0.0) continue;
      const double f = M[r][c];
      for (int j = 0; j < n; ++j) {
        M[r][j] -= f * M[c][j];
        R[r][j] -= f * R[c][j];
      }
    }
  }
}

void powers(int k, double x, double *p, double *d, double *d2) {
  for (int i = 0; i <= k; ++i) {
    p[i] = i == 0 ? 1.0 : p[i - 1] * x;
    d[i] = i == 0 ? 0.0 : i * (i == 1 ? 1.0 : p[i - 2] * x);
    d2[i] = i < 2 ? 0.0 : i * (i - 1) * (i == 2 ? 1.0 : p[i - 3] * x);
  }
}

constexpr double kLimit = 1e-11;  // limit_to_be_definite, lower_bound_implicit_function
constexpr int kMaxBoxSplits = 4, kMaxRootSplits = 2;
constexpr double kRootTol = 1e-12;

bool indefinite(double lo, double hi) { return !(lo > 0.0 || hi < 0.0); }
double lower_abs(double lo, double hi) { return (lo > 0.0 || hi < 0.0) ? std::min(std::fabs(lo), std::fabs(hi)) : 0.0; }
int sgn(double x) { return (x > 0.0) - (x < 0.0); }

// RootFinder::find_roots of the 1D function L(x) -> (value, first, second
// derivative) on [a, b]: a sign change at the ends gives a root (bisected to
// machine precision); otherwise Taylor bounds at the centre and up to two
// halvings
template <class Line>
void find_roots(const Line &L, double a, double b, int depth, std::vector<double> &roots) {
  double fa, fb, d1, d2;
  L(a, fa, d1, d2);
  L(b, fb, d1, d2);
  if (sgn(fa) != sgn(fb)) {
    if (fa == 0.0) {
      roots.push_back(a);
      return;
    }
    double lo = a, hi = b, flo = fa;
    for (int it = 0; it < 200; ++it) {
      const double m = 0.5 * (lo + hi);
      if (m == lo || m == hi) break;
      double fm;
      L(m, fm, d1, d2);
      if (fm == 0.0) {
        roots.push_back(m);
        return;
      }
      if ((fm < 0.0) == (flo < 0.0)) {
        lo = m;
        flo = fm;
      } else {
        hi = m;
      }
    }
    roots.push_back(0.5 * (lo + hi));
    return;
  }
  const double c = 0.5 * (a + b), dx = 0.5 * (b - a);
  double v;
  L(c, v, d1, d2);
  const double spread = std::fabs(d1) * dx + 0.5 * std::fabs(d2) * dx * dx;
  if (!indefinite(v - spread, v + spread)) return;
  if (depth < kMaxRootSplits) {
    find_roots(L, a, c, depth + 1, roots);
    find_roots(L, c, b, depth + 1, roots);
  }
}

void unique_sorted(std::vector<double> &r) {
  std::sort(r.begin(), r.end());
  std::vector<double> out;
  for (double x : r)
    if (out.empty() || std::fabs(x - out.back()) >= kRootTol) out.push_back(x);
  r.swap(out);
}

struct PolyGen {
  const TensorPoly &f;
  const std::vector<double> &qx, &qw;
  std::vector<QPoint> &inside;
  std::vector<SPoint> &surface;
  std::vector<QPoint> *outside;  // f > 0 (q_partitioning.positive), NULL: not collected
  int n_splits = 0;

  void tensor(const double lo[2], const double hi[2], std::vector<QPoint> *dst) {
    if (!dst) return;
    const double L0 = hi[0] - lo[0], L1 = hi[1] - lo[1];
    for (size_t b = 0; b < qx.size(); ++b)
      for (size_t a = 0; a < qx.size(); ++a)
        dst->push_back({lo[0] + L0 * qx[a], lo[1] + L1 * qx[b], qw[a] * qw[b] * L0 * L1});
  }
  // the region a point of level-set value fv belongs to (exact zeros: neither)
  std::vector<QPoint> *region(double fv) { return fv < 0.0 ? &inside : (fv > 0.0 ? outside : nullptr); }

  void generate(const double lo[2], const double hi[2], int n_box_splits) {
    const double c[2] = {0.5 * (lo[0] + hi[0]), 0.5 * (lo[1] + hi[1])};
    const double dx[2] = {0.5 * (hi[0] - lo[0]), 0.5 * (hi[1] - lo[1])};
    double val, g[2], H[2][2];
    f.derivatives(c[0], c[1], val, g, H);
    double spread = std::fabs(g[0]) * dx[0] + std::fabs(g[1]) * dx[1];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) spread += 0.5 * std::fabs(H[i][j]) * dx[i] * dx[j];
    double vmin = val - spread, vmax = val + spread;
    for (double vs : {lo[0], hi[0]})
      for (double vt : {lo[1], hi[1]}) {
        const double fv = f.value(vs, vt);
        vmin = std::min(vmin, fv);
        vmax = std::max(vmax, fv);
      }
    if (vmin > kLimit) {
      tensor(lo, hi, outside);
      return;
    }
    if (vmax < -kLimit) {
      tensor(lo, hi, &inside);
      return;
    }
    double low[2];
    for (int i = 0; i < 2; ++i) {
      const double dg = std::fabs(H[i][0]) * dx[0] + std::fabs(H[i][1]) * dx[1];
      low[i] = lower_abs(g[i] - dg, g[i] + dg);
    }
    // first of equal ones (within 1e-12 relative: symmetric cells tie up to round-off)
    const int hdir = low[1] > low[0] + 1e-12 * std::max(low[0], low[1]) ? 1 : 0;
    if (low[hdir] > kLimit) {
      height(hdir, lo, hi);
    } else if (n_box_splits < kMaxBoxSplits) {
      ++n_splits;
      const int d = (hi[0] - lo[0]) >= (hi[1] - lo[1]) ? 0 : 1;
      const double mid = 0.5 * (lo[d] + hi[d]);
      double hl[2] = {hi[0], hi[1]}, lr[2] = {lo[0], lo[1]};
      hl[d] = mid;
      lr[d] = mid;
      generate(lo, hl, n_box_splits + 1);
      generate(lr, hi, n_box_splits + 1);
    } else if (auto *dst = region(f.value(c[0], c[1]))) {  // midpoint rule
      dst->push_back({c[0], c[1], 4.0 * dx[0] * dx[1]});
    }
  }

  void height(int hdir, const double lo[2], const double hi[2]) {
    const int cdir = 1 - hdir;
    const double c_lo = lo[cdir], c_hi = hi[cdir], h_lo = lo[hdir], h_hi = hi[hdir];
    auto at = [&](double cc, double hh, double &s, double &t) {
      s = cdir == 0 ? cc : hh;
      t = cdir == 0 ? hh : cc;
    };
    // the level set along direction dir through the point (cc, hh) with the other coordinate fixed
    auto line = [&](int dir, double fixed_c, double fixed_h) {
      return [&, dir, fixed_c, fixed_h](double x, double &v, double &d1, double &d2) {
        double s, t, g[2], H[2][2];
        if (dir == cdir)
          at(x, fixed_h, s, t);
        else
          at(fixed_c, x, s, t);
        f.derivatives(s, t, v, g, H);
        d1 = g[dir];
        d2 = H[dir][dir];
      };
    };
    std::vector<double> roots;
    find_roots(line(cdir, 0.0, h_lo), c_lo, c_hi, 0, roots);
    find_roots(line(cdir, 0.0, h_hi), c_lo, c_hi, 0, roots);
    unique_sorted(roots);
    std::vector<double> edges;
    edges.push_back(c_lo);
    edges.insert(edges.end(), roots.begin(), roots.end());
    edges.push_back(c_hi);
    const double Lh = h_hi - h_lo;
    const int nq = (int)qx.size();
    std::vector<double> hr;
    for (size_t e = 0; e + 1 < edges.size(); ++e) {
      const double a = edges[e], L = edges[e + 1] - a;
      if (!(L > 0.0)) continue;
      double s, t;
      at(a + 0.5 * L, h_lo, s, t);
      const double sb = f.value(s, t);
      at(a + 0.5 * L, h_hi, s, t);
      const double st = f.value(s, t);
      const bool definite = (sb < 0.0 && st < 0.0) || (sb > 0.0 && st > 0.0);
      if (definite && sb > 0.0 && !outside) continue;
      for (int k = 0; k < nq; ++k) {
        const double cc = a + L * qx[k], wc = qw[k] * L;
        if (definite) {
          std::vector<QPoint> &dst = sb < 0.0 ? inside : *outside;
          for (int m = 0; m < nq; ++m) {
            at(cc, h_lo + Lh * qx[m], s, t);
            dst.push_back({s, t, wc * qw[m] * Lh});
          }
          continue;
        }
        hr.clear();
        find_roots(line(hdir, cc, 0.0), h_lo, h_hi, 0, hr);
        unique_sorted(hr);
        double prev = h_lo;
        for (size_t r = 0; r <= hr.size(); ++r) {
          const double nxt = r < hr.size() ? hr[r] : h_hi, Ls = nxt - prev;
          if (Ls > 0.0) {
            at(cc, prev + 0.5 * Ls, s, t);
            if (auto *dst = region(f.value(s, t)))
              for (int m = 0; m < nq; ++m) {
                at(cc, prev + Ls * qx[m], s, t);
                dst->push_back({s, t, wc * qw[m] * Ls});
              }
          }
          prev = nxt;
        }
        if (hr.size() == 1) {
          double v, g[2], H[2][2];
          at(cc, hr[0], s, t);
          f.derivatives(s, t, v, g, H);
          const double ng = std::hypot(g[0], g[1]);
          surface.push_back({s, t, wc * ng / std::fabs(g[hdir]), g[0] / ng, g[1] / ng});
        }
      }
    }
  }
};

}  // namespace

void TensorPoly::interpolate(int k_, const double *vals, const std::vector<double> &support) {
  k = k_;
  double A[10][10] = {};
  lagrange_monomials(support, A);
  const int n = k + 1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double c = 0.0;
      for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) c += A[a][i] * vals[a + n * b] * A[b][j];
      C[i][j] = c;
    }
}

double TensorPoly::value(double s, double t) const {
  double r = 0.0;
  for (int i = k; i >= 0; --i) {
    double row = 0.0;
    for (int j = k; j >= 0; --j) row = row * t + C[i][j];
    r = r * s + row;
  }
  return r;
}

void TensorPoly::derivatives(double s, double t, double &v, double g[2], double H[2][2]) const {
  double ps[10], ds[10], d2s[10], pt[10], dt[10], d2t[10];
  powers(k, s, ps, ds, d2s);
  powers(k, t, pt, dt, d2t);
  double r[6] = {0, 0, 0, 0, 0, 0};  // v, fs, ft, fss, fst, ftt
  for (int i = 0; i <= k; ++i) {
    double c0 = 0.0, c1 = 0.0, c2 = 0.0;  // sum_j C_ij t^j, d/dt, d2/dt2
    for (int j = 0; j <= k; ++j) {
      c0 += C[i][j] * pt[j];
      c1 += C[i][j] * dt[j];
      c2 += C[i][j] * d2t[j];
    }
    r[0] += ps[i] * c0;
    r[1] += ds[i] * c0;
    r[2] += ps[i] * c1;
    r[3] += d2s[i] * c0;
    r[4] += ds[i] * c1;
    r[5] += ps[i] * c2;
  }
  v = r[0];
  g[0] = r[1];
  g[1] = r[2];
  H[0][0] = r[3];
  H[0][1] = H[1][0] = r[4];
  H[1][1] = r[5];
}

int bernstein_location(int dim, int k, const double *vals, const std::vector<double> &support) {
  const int n = k + 1;
  double B[10][10], T[10][10];
  for (int a = 0; a < n; ++a)
    for (int i = 0; i < n; ++i) {
      double binom = 1.0;
      for (int q = 1; q <= i; ++q) binom = binom * (k - i + q) / q;
      B[a][i] = binom * std::pow(support[a], i) * std::pow(1.0 - support[a], k - i);
    }
  invert(n, B, T);
  double lo = INFINITY, hi = -INFINITY;
  if (dim == 1) {
    for (int i = 0; i < n; ++i) {
      double c = 0.0;
      for (int a = 0; a < n; ++a) c += T[i][a] * vals[a];
      lo = std::min(lo, c);
      hi = std::max(hi, c);
    }
  } else {
    // T V T^T with V[a][b] = vals[a + n b]
    double TV[10][10];
    for (int i = 0; i < n; ++i)
      for (int b = 0; b < n; ++b) {
        double c = 0.0;
        for (int a = 0; a < n; ++a) c += T[i][a] * vals[a + n * b];
        TV[i][b] = c;
      }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double c = 0.0;
        for (int b = 0; b < n; ++b) c += TV[i][b] * T[j][b];
        lo = std::min(lo, c);
        hi = std::max(hi, c);
      }
  }
  if (hi < 0.0) return INSIDE;
  if (lo > 0.0) return OUTSIDE;
  return INTERSECTED;
}

void saye_poly(const TensorPoly &f, const std::vector<double> &qx, const std::vector<double> &qw,
               std::vector<QPoint> &inside, std::vector<SPoint> &surface, int *n_splits,
               std::vector<QPoint> *outside) {
  inside.clear();
  surface.clear();
  if (outside) outside->clear();
  PolyGen gen{f, qx, qw, inside, surface, outside};
  const double lo[2] = {0.0, 0.0}, hi[2] = {1.0, 1.0};
  gen.generate(lo, hi, 0);
  if (n_splits) *n_splits += gen.n_splits;
}

}  // namespace gdm

struct gdm_cut_system {
  int p = 0, n = 0;
  double lo = 0.0, h = 0.0, cx = 0.0, cy = 0.0, r = 1.0, f = 0.0, g = 0.0;
  std::vector<int8_t> loc;  // [cy][cx]
  std::vector<double> ls;   // vertex level set [iy][ix]
  std::vector<int64_t> row_ptr;
  std::vector<uint32_t> cols;
  std::vector<double> vals, rhs;
  int64_t n_inside = 0, n_intersected = 0;
};

namespace {

using namespace gdm;

// inside / surface quadrature of cell (cx, cy) in reference coordinates (weights in reference measure)
void cell_quadrature(const gdm_cut_system &S, int cx, int cy, const std::vector<double> &qx,
                     const std::vector<double> &qw, std::vector<QPoint> &ins, std::vector<SPoint> &sur) {
  ins.clear();
  sur.clear();
  const int loc = S.loc[(size_t)cy * S.n + cx];
  const int nq = (int)qx.size();
  if (loc == OUTSIDE) return;
  if (loc == INSIDE) {
    for (int b = 0; b < nq; ++b)
      for (int a = 0; a < nq; ++a) ins.push_back({qx[a], qx[b], qw[a] * qw[b]});
    return;
  }
  const int N = S.n + 1;
  const double v00 = S.ls[(size_t)cy * N + cx], v10 = S.ls[(size_t)cy * N + cx + 1];
  const double v01 = S.ls[(size_t)(cy + 1) * N + cx], v11 = S.ls[(size_t)(cy + 1) * N + cx + 1];
  Bilinear f{v00, v10 - v00, v01 - v00, v11 - v10 - v01 + v00};
  saye_unit(f, qx, qw, ins, sur);
}

void assemble(gdm_cut_system &S, bool gp) {
  const int p = S.p, n = S.n, N = n + 1, n1 = p + 1, nd = n1 * n1;
  const double h = S.h, gamma = 5.0 * (p + 1) * p, gpar = 0.5;
  std::vector<double> qx, qw;
  gauss_unit(n1, qx, qw);
  // dense per-row slots: columns j = i + dy N + dx, |dx|, |dy| <= p + 1
  const int R = p + 1, SW = 2 * R + 1, SL = SW * SW;
  const int64_t nd_tot = (int64_t)N * N;
  std::vector<double> slot((size_t)nd_tot * SL, 0.0);
  std::vector<uint8_t> touched((size_t)nd_tot * SL, 0);
  S.rhs.assign((size_t)nd_tot, 0.0);
  auto add = [&](int64_t row, int64_t col, double v) {
    const int64_t ry = row / N, rx = row % N, cyy = col / N, cxx = col % N;
    const int64_t k = (cyy - ry + R) * SW + (cxx - rx + R);
    slot[(size_t)row * SL + k] += v;
    touched[(size_t)row * SL + k] = 1;
  };
  auto dofs = [&](int cx, int cy, int64_t *d) {
    const int ox = (int)box_offset((unsigned)cx, (unsigned)p, (unsigned)n);
    const int oy = (int)box_offset((unsigned)cy, (unsigned)p, (unsigned)n);
    for (int iy = 0; iy < n1; ++iy)
      for (int ix = 0; ix < n1; ++ix) d[iy * n1 + ix] = (int64_t)(oy + iy) * N + (ox + ix);
  };
  // per-category tables of fully inside cells (interior-cell local matrix and rhs)
  std::vector<std::vector<double>> catK((size_t)p * p), catF((size_t)p * p);
  std::vector<QPoint> ins;
  std::vector<SPoint> sur;
  std::vector<double> K((size_t)nd * nd), F(nd), val(nd), gx(nd), gy(nd);
  auto eval = [&](int catx, int caty, double s, double t) {
    Shapes sx, sy;
    shapes_1d(p, catx, s, sx);
    shapes_1d(p, caty, t, sy);
    for (int iy = 0; iy < n1; ++iy)
      for (int ix = 0; ix < n1; ++ix) {
        const int i = iy * n1 + ix;
        val[i] = sx.v[ix] * sy.v[iy];
        gx[i] = sx.d[ix] * sy.v[iy] / h;
        gy[i] = sx.v[ix] * sy.d[iy] / h;
      }
  };
  auto local = [&](int cx, int cy, bool cut) {
    std::fill(K.begin(), K.end(), 0.0);
    std::fill(F.begin(), F.end(), 0.0);
    const int catx = (int)category((unsigned)cx, (unsigned)p, (unsigned)n);
    const int caty = (int)category((unsigned)cy, (unsigned)p, (unsigned)n);
    cell_quadrature(S, cx, cy, qx, qw, ins, sur);
    (void)cut;
    for (const QPoint &q : ins) {
      eval(catx, caty, q.s, q.t);
      const double w = q.w * h * h;
      for (int i = 0; i < nd; ++i) {
        for (int j = 0; j < nd; ++j) K[(size_t)i * nd + j] += (gx[i] * gx[j] + gy[i] * gy[j]) * w;
        F[i] += S.f * val[i] * w;
      }
    }
    for (const SPoint &q : sur) {
      eval(catx, caty, q.s, q.t);
      const double w = q.w * h;
      for (int i = 0; i < nd; ++i) {
        const double dni = q.nx * gx[i] + q.ny * gy[i];
        for (int j = 0; j < nd; ++j) {
          const double dnj = q.nx * gx[j] + q.ny * gy[j];
          K[(size_t)i * nd + j] += (-dni * val[j] - dnj * val[i] + gamma / h * val[i] * val[j]) * w;
        }
        F[i] += S.g * (gamma / h * val[i] - dni) * w;
      }
    }
  };
  int64_t d[64], e[64];
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx) {
      const int loc = S.loc[(size_t)cy * n + cx];
      if (loc == OUTSIDE) continue;
      dofs(cx, cy, d);
      if (gp) {
        const int nb[4][2] = {{cx - 1, cy}, {cx + 1, cy}, {cx, cy - 1}, {cx, cy + 1}};
        for (int fi = 0; fi < 4; ++fi) {
          const int nx = nb[fi][0], ny = nb[fi][1];
          if (nx < 0 || ny < 0 || nx >= n || ny >= n) continue;
          const int lb = S.loc[(size_t)ny * n + nx];
          if (!((loc == INTERSECTED && lb != OUTSIDE) || (lb == INTERSECTED && loc != OUTSIDE))) continue;
          const int axis = fi < 2 ? 0 : 1, side = fi % 2;
          dofs(nx, ny, e);
          const int c0x = (int)category((unsigned)cx, (unsigned)p, (unsigned)n);
          const int c0y = (int)category((unsigned)cy, (unsigned)p, (unsigned)n);
          const int c1x = (int)category((unsigned)nx, (unsigned)p, (unsigned)n);
          const int c1y = (int)category((unsigned)ny, (unsigned)p, (unsigned)n);
          std::vector<double> S2((size_t)4 * nd * nd, 0.0);
          std::vector<double> jump(2 * nd);
          for (int q = 0; q < n1; ++q) {
            double s0, t0, s1, t1;
            if (axis == 0) {
              s0 = side;
              t0 = qx[q];
              s1 = 1 - side;
              t1 = qx[q];
            } else {
              s0 = qx[q];
              t0 = side;
              s1 = qx[q];
              t1 = 1 - side;
            }
            eval(c0x, c0y, s0, t0);
            for (int i = 0; i < nd; ++i) jump[i] = axis == 0 ? gx[i] : gy[i];
            eval(c1x, c1y, s1, t1);
            for (int i = 0; i < nd; ++i) jump[nd + i] = -(axis == 0 ? gx[i] : gy[i]);
            const double w = 0.5 * gpar * h * qw[q] * h;
            for (int i = 0; i < 2 * nd; ++i)
              for (int j = 0; j < 2 * nd; ++j) S2[(size_t)i * 2 * nd + j] += jump[i] * jump[j] * w;
          }
          for (int i = 0; i < 2 * nd; ++i)
            for (int j = 0; j < 2 * nd; ++j)
              add(i < nd ? d[i] : e[i - nd], j < nd ? d[j] : e[j - nd], S2[(size_t)i * 2 * nd + j]);
        }
      }
      const double *Kc;
      const double *Fc;
      if (loc == INSIDE) {
        const int catx = (int)category((unsigned)cx, (unsigned)p, (unsigned)n);
        const int caty = (int)category((unsigned)cy, (unsigned)p, (unsigned)n);
        std::vector<double> &ck = catK[(size_t)caty * p + catx];
        if (ck.empty()) {
          local(cx, cy, false);
          ck = K;
          catF[(size_t)caty * p + catx] = F;
        }
        Kc = ck.data();
        Fc = catF[(size_t)caty * p + catx].data();
        ++S.n_inside;
      } else {
        local(cx, cy, true);
        Kc = K.data();
        Fc = F.data();
        ++S.n_intersected;
      }
      // cell-local (i, j) -> slot of row d[i]: the offsets of a cell's DoF box
      // are the local index differences (no division per entry)
      for (int iy = 0; iy < n1; ++iy)
        for (int ix = 0; ix < n1; ++ix) {
          const int i = iy * n1 + ix;
          double *srow = slot.data() + (size_t)d[i] * SL;
          uint8_t *trow = touched.data() + (size_t)d[i] * SL;
          for (int jy = 0; jy < n1; ++jy)
            for (int jx = 0; jx < n1; ++jx) {
              const int k = (jy - iy + R) * SW + (jx - ix + R);
              srow[k] += Kc[(size_t)i * nd + jy * n1 + jx];
              trow[k] = 1;
            }
          S.rhs[(size_t)d[i]] += Fc[i];
        }
    }
  // CSR: touched entries (ascending columns) + every diagonal; zero diagonals -> 1
  S.row_ptr.assign((size_t)nd_tot + 1, 0);
  S.cols.clear();
  S.vals.clear();
  for (int64_t row = 0; row < nd_tot; ++row) {
    const int64_t ry = row / N, rx = row % N;
    for (int k = 0; k < SL; ++k) {
      const int dy = k / SW - R, dx = k % SW - R;
      const bool diag = dx == 0 && dy == 0;
      if (!touched[(size_t)row * SL + k] && !diag) continue;
      const int64_t cyy = ry + dy, cxx = rx + dx;
      if (cyy < 0 || cyy >= N || cxx < 0 || cxx >= N) continue;
      double v = slot[(size_t)row * SL + k];
      if (diag && v == 0.0) v = 1.0;
      S.cols.push_back((uint32_t)(cyy * N + cxx));
      S.vals.push_back(v);
    }
    S.row_ptr[(size_t)row + 1] = (int64_t)S.cols.size();
  }
}

}  // namespace

extern "C" {

int gdmh_cut_poisson_create(int p, int n_sub, double lo, double hi, const double *center, double radius,
                            int ghost_penalty, double rhs_value, double bc_value, gdm_cut_system **out,
                            char *err, size_t err_len) {
  try {
    if (!out || p < 1 || p > 9 || p % 2 == 0 || n_sub < p || !(hi > lo) || !(radius > 0.0))
      throw std::invalid_argument("cut_poisson: invalid arguments (p odd in [1, 9], n_sub >= p, hi > lo, radius > 0)");
    if ((int64_t)(n_sub + 1) * (n_sub + 1) >= (int64_t)1 << 32) throw std::invalid_argument("cut_poisson: mesh too large");
    auto *S = new gdm_cut_system();
    S->p = p;
    S->n = n_sub;
    S->lo = lo;
    S->h = (hi - lo) / n_sub;
    S->cx = center ? center[0] : 0.0;
    S->cy = center ? center[1] : 0.0;
    S->r = radius;
    S->f = rhs_value;
    S->g = bc_value;
    const int N = n_sub + 1;
    S->ls.resize((size_t)N * N);
    for (int iy = 0; iy < N; ++iy)
      for (int ix = 0; ix < N; ++ix) {
        const double x = lo + ix * S->h - S->cx, y = lo + iy * S->h - S->cy;
        S->ls[(size_t)iy * N + ix] = std::sqrt(x * x + y * y) - radius;  // SignedDistance::Sphere
      }
    S->loc.resize((size_t)n_sub * n_sub);
    for (int cy = 0; cy < n_sub; ++cy)
      for (int cx = 0; cx < n_sub; ++cx) {
        const double v[4] = {S->ls[(size_t)cy * N + cx], S->ls[(size_t)cy * N + cx + 1],
                             S->ls[(size_t)(cy + 1) * N + cx], S->ls[(size_t)(cy + 1) * N + cx + 1]};
        bool neg = true, pos = true;
        for (double w : v) {
          neg = neg && w < 0.0;
          pos = pos && w > 0.0;
        }
        S->loc[(size_t)cy * n_sub + cx] = neg ? gdm::INSIDE : (pos ? gdm::OUTSIDE : gdm::INTERSECTED);
      }
    try {
      assemble(*S, ghost_penalty != 0);
    } catch (...) {
      delete S;
      throw;
    }
    *out = S;
    return 0;
  } catch (const std::exception &e) {
    if (err && err_len) std::snprintf(err, err_len, "%s", e.what());
    return -1;
  }
}

void gdmh_cut_info(const gdm_cut_system *S, int64_t *n_rows, int64_t *nnz, int64_t *n_inside,
                   int64_t *n_intersected) {
  *n_rows = (int64_t)S->rhs.size();
  *nnz = (int64_t)S->vals.size();
  *n_inside = S->n_inside;
  *n_intersected = S->n_intersected;
}

void gdmh_cut_arrays(const gdm_cut_system *S, const int64_t **row_ptr, const uint32_t **cols, const double **vals,
                     const double **rhs) {
  *row_ptr = S->row_ptr.data();
  *cols = S->cols.data();
  *vals = S->vals.data();
  *rhs = S->rhs.data();
}

// L2 error of u (host, n_rows values) against u = g + f / 4 (r^2 - |x - c|^2)
// over the inside quadrature (cut_poisson_01_gdm.cc:349-405 with its
// manufactured solution)
double gdmh_cut_l2_error(const gdm_cut_system *S, const double *u) {
  using namespace gdm;
  const int p = S->p, n = S->n, N = n + 1, n1 = p + 1;
  std::vector<double> qx, qw;
  gauss_unit(n1, qx, qw);
  std::vector<QPoint> ins;
  std::vector<SPoint> sur;
  double err2 = 0.0;
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx) {
      if (S->loc[(size_t)cy * n + cx] == OUTSIDE) continue;
      cell_quadrature(*S, cx, cy, qx, qw, ins, sur);
      const int catx = (int)category((unsigned)cx, (unsigned)p, (unsigned)n);
      const int caty = (int)category((unsigned)cy, (unsigned)p, (unsigned)n);
      const int ox = (int)box_offset((unsigned)cx, (unsigned)p, (unsigned)n);
      const int oy = (int)box_offset((unsigned)cy, (unsigned)p, (unsigned)n);
      for (const QPoint &q : ins) {
        Shapes sx, sy;
        shapes_1d(p, catx, q.s, sx);
        shapes_1d(p, caty, q.t, sy);
        double uh = 0.0;
        for (int iy = 0; iy < n1; ++iy)
          for (int ix = 0; ix < n1; ++ix) uh += u[(size_t)(oy + iy) * N + ox + ix] * sx.v[ix] * sy.v[iy];
        const double x = S->lo + (cx + q.s) * S->h - S->cx, y = S->lo + (cy + q.t) * S->h - S->cy;
        const double ex = S->g + S->f / 4.0 * (S->r * S->r - (x * x + y * y));
        err2 += (uh - ex) * (uh - ex) * q.w * S->h * S->h;
      }
    }
  return std::sqrt(err2);
}

void gdmh_cut_destroy(gdm_cut_system *S) { delete S; }

}  // extern "C"
