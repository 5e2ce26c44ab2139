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
