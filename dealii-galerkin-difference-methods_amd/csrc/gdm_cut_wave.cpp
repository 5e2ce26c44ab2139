// gdm_cut_wave.cpp -- host assembly of the cut-cell parts of the wave /
// heat / poisson application (applications/wave: wave-app.cc presets "wave",
// "heat-rk", "heat-impl" (inside field, interface data), "heat-composite",
// "wave-composite" (inside + outside fields, domain data, interface coupling)
// at dim = 1 and 2, "step85" at dim = 2) for the device operator of
// gdm_capi.cpp ("Cut-cell wave" in include/gdm_hip.h).
//
// The mesh is a GDM line [left, right] or square [left, right]^2 cut by the
// FE_Q(k) interpolant of a level set (wave/discretization.h:78-93:
// SignedDistance::Sphere into FE_Q(k), MeshClassifier): the caller gives the
// interpolant's values at the (k + 1)^dim Gauss-Lobatto support points of
// every cell.  Per cell: inside / outside / intersected by the signs of the
// interpolant's Bernstein coefficients (MeshClassifier).  1D: an intersected
// cell's inside part comes from the roots of its interpolant (sign changes on
// a 64-interval grid refined by bisection to machine precision), QGauss(p+1)
// on each inside sub-interval and one surface point per root (weight 1,
// normal = sign of the slope).  2D: deal.II's QuadratureGenerator on the
// cell's tensor-product polynomial (saye_poly, gdm_cut.cpp) -- NonMatching::
// FEValues.
//
// The device evaluates StiffnessMatrixOperator::compute_rhs
// (wave/stiffness.h:42-407) as
//   rhs = impl ? (Z S u + C u) : 0  +  Ff f(x_q, t)  +  Fg g(x_s, t)
// with S the uncut 1D wave stencil of the box (-(v', u'), gdm_op kind wave),
// Z zeroing the rows of DoFs in the box of a cell that is not fully inside,
// and the sparse parts assembled here:
//   C   those rows of -(grad v, grad u)_inside in full, the surface Nitsche
//       terms -(-d_n v u - d_n u v + gamma_D / h v u) (stiffness.h:205-259)
//       of the cut cells, and the ghost penalty -0.5 gamma_A h [d_n v][d_n u]
//       (h^1 in the right-hand side, stiffness.h:386-392; QGauss(p+1) on 2D
//       faces) on the faces of intersected cells with a non-outside
//       neighbour, visited from both cells;
//   Ff  (v, f): column q = the inside quadrature point q (JxW folded in);
//   Fg  the Nitsche data g (gamma_D / h v - n v'): column s = surface point s.
// Mass (wave/mass.h:47-249): (v, u)_inside + 0.5 gamma_M h^3 [d_n v][d_n u],
// zero diagonals -> 1 (none when gamma_M < 0); stiffness matrix
// (stiffness.h:602-800): (grad v, grad u)_inside + surface Nitsche +
// 0.5 gamma_A h^3 [d_n v][d_n u], zero diagonals -> 1.  Both are band
// matrices (half-bandwidth (p+1)(N+1) in 2D): the mass solve, the (M + dt K)
// solve of heat-impl and the K solve of poisson are exact banded Cholesky
// solves (factor here, triangular solves on the device); the reference's
// solves converge in 2-3 AMG-preconditioned CG steps to 1e-14.
// E (n_quad x N): shape values at the inside quadrature points, for the
// postprocess (problem.h:504-615).  Test oracles: oracle/cut1d.py and
// oracle/cut_wave2d.py, pinned by applications/wave/tests/{wave_0,heat_0,
// heat_1,wave_1,step85_0}.output.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <map>
#include <stdexcept>
#include <vector>

#include "gdm_cut.h"
#include "gdm_setup.h"

struct gdm_cut_wave_system {
  int dim = 1, p = 0, n = 0, k = 0, n_splits = 0;
  int location = -1, dirichlet = 1;  // the field's region (INSIDE -1 / OUTSIDE 1); Nitsche data: bit 0 interface, bit 1 domain
  bool coupled = false;                  // composite: interface coupling to the other region's field
  double lo = 0.0, h = 0.0, gM = 0.0, gA = 0.0, nitsche = 0.0;
  std::vector<int8_t> loc;
  std::vector<double> qx, qw;  // inside quadrature: global coordinates [n][dim], JxW
  std::vector<double> sx, sn;  // surface points: global coordinates [n][dim], normal [n][dim]
  std::vector<int64_t> zero_rows;
  // CSR: C [N][N], Ff [N][nq], Fg [N][ns], E [nq][N], M [N][N], K [N][N], X [N][N]
  std::vector<int64_t> c_rp, ff_rp, fg_rp, e_rp, m_rp, s_rp, x_rp;
  std::vector<uint32_t> c_ci, ff_ci, fg_ci, e_ci, m_ci, s_ci, x_ci;
  std::vector<double> c_v, ff_v, fg_v, e_v, m_v, s_v, x_v;
  int64_t cells[3] = {0, 0, 0};
};

namespace {

using namespace gdm;

// accumulator of an N^dim x N^dim matrix with couplings |i_d - j_d| <= R per
// direction (DoF index = ix + N iy): one dense slot row per DoF
struct Slots {
  int64_t N = 0, rows = 0;
  int dim = 1, R = 0, SW = 1, SL = 1;
  std::vector<double> v;
  std::vector<uint8_t> touched;
  void init(int dim_, int64_t N_, int R_) {
    dim = dim_;
    N = N_;
    R = R_;
    SW = 2 * R + 1;
    SL = dim == 1 ? SW : SW * SW;
    rows = dim == 1 ? N : N * N;
    v.assign((size_t)rows * SL, 0.0);
    touched.assign(v.size(), 0);
  }
  int64_t slot(int64_t i, int64_t j) const {
    if (dim == 1) return j - i + R;
    return (j / N - i / N + R) * SW + (j % N - i % N + R);
  }
  void add(int64_t i, int64_t j, double x) {
    const size_t o = (size_t)i * SL + (size_t)slot(i, j);
    v[o] += x;
    touched[o] = 1;
  }
  void csr(std::vector<int64_t> &rp, std::vector<uint32_t> &ci, std::vector<double> &vals, bool unit_diag) const {
    rp.assign((size_t)rows + 1, 0);
    ci.clear();
    vals.clear();
    for (int64_t i = 0; i < rows; ++i) {
      const int64_t ix = dim == 1 ? i : i % N, iy = dim == 1 ? 0 : i / N;
      for (int k = 0; k < SL; ++k) {
        const int64_t dx = (dim == 1 ? k : k % SW) - R, dy = dim == 1 ? 0 : k / SW - R;
        const int64_t jx = ix + dx, jy = iy + dy;
        if (jx < 0 || jx >= N || jy < 0 || (dim == 2 && jy >= N)) continue;
        const int64_t j = dim == 1 ? jx : jy * N + jx;
        const bool diag = j == i;
        const size_t o = (size_t)i * SL + (size_t)k;
        if (!touched[o] && !(diag && unit_diag)) continue;
        double x = v[o];
        if (diag && unit_diag && x == 0.0) x = 1.0;
        ci.push_back((uint32_t)j);
        vals.push_back(x);
      }
      rp[(size_t)i + 1] = (int64_t)ci.size();
    }
  }
};

// CSR from (row, col, value) triplets, duplicates summed in insertion order
struct Trip {
  int64_t r, c;
  double v;
};
void triplets_csr(std::vector<Trip> t, int64_t rows, std::vector<int64_t> &rp, std::vector<uint32_t> &ci,
                  std::vector<double> &vals) {
  std::stable_sort(t.begin(), t.end(), [](const Trip &a, const Trip &b) { return a.r != b.r ? a.r < b.r : a.c < b.c; });
  rp.assign((size_t)rows + 1, 0);
  ci.clear();
  vals.clear();
  for (size_t q = 0; q < t.size(); ++q) {
    if (q > 0 && t[q - 1].r == t[q].r && t[q - 1].c == t[q].c) {
      vals.back() += t[q].v;
      continue;
    }
    ci.push_back((uint32_t)t[q].c);
    vals.push_back(t[q].v);
    ++rp[(size_t)t[q].r + 1];
  }
  for (int64_t r = 0; r < rows; ++r) rp[(size_t)r + 1] += rp[(size_t)r];
}

// The field of S.location (INSIDE: phi < 0, OUTSIDE: phi > 0); inv = the
// other region.  Cells of location inv are skipped, ghost-penalty faces have
// an intersected cell and a neighbour not of location inv
// (wave/mass.h:86-105).  S.dirichlet bit 0: interface data (II, surface
// points, stiffness.h:205-259; normal flipped for OUTSIDE), bit 1: domain
// data (IV, boundary faces in the region, :262-330).  S.coupled: the
// composite interface terms of compute_rhs(BlockVector) (:420-575): the own
// field's part into C, the partner's into X.
void assemble1d(gdm_cut_wave_system &S, const double *ls_values) {
  const int p = S.p, n = S.n, k = S.k, n1 = p + 1, loc_f = S.location, inv = -loc_f;
  const int64_t N = n + 1;
  const double h = S.h;
  std::vector<double> gx, gw;
  gauss_unit(n1, gx, gw);
  const std::vector<double> gl = gauss_lobatto(k + 1);
  S.loc.assign(n, OUTSIDE);
  // per cell: the region's quadrature (reference s, reference weight) and the surface (s, level-set normal)
  std::vector<std::vector<std::pair<double, double>>> cq(n), cs(n);
  for (int c = 0; c < n; ++c) {
    const double *vals = ls_values + (size_t)c * (k + 1);
    const int where = bernstein_location(1, k, vals, gl);
    auto phi = [&](double s) {
      double r = 0.0;
      for (int a = 0; a <= k; ++a) {
        double la = 1.0;
        for (int b = 0; b <= k; ++b)
          if (b != a) la *= (s - gl[b]) / (gl[a] - gl[b]);
        r += vals[a] * la;
      }
      return r;
    };
    S.loc[c] = (int8_t)where;
    if (where != INTERSECTED) {
      if (where == loc_f)
        for (int q = 0; q < n1; ++q) cq[c].push_back({gx[q], gw[q]});
      continue;
    }
    constexpr int G = 64;
    double pv[G + 1];
    for (int a = 0; a <= G; ++a) pv[a] = phi((double)a / G);
    std::vector<double> roots;
    for (int a = 0; a < G; ++a) {
      const double s0 = (double)a / G, s1 = (double)(a + 1) / G;
      if (pv[a] == 0.0) {
        roots.push_back(s0);
      } else if (pv[a] * pv[a + 1] < 0.0) {
        double lo = s0, hi = s1, flo = pv[a];
        for (int it = 0; it < 200; ++it) {
          const double mid = 0.5 * (lo + hi);
          if (mid == lo || mid == hi) break;
          const double fm = phi(mid);
          if ((fm < 0.0) == (flo < 0.0)) {
            lo = mid;
            flo = fm;
          } else {
            hi = mid;
          }
        }
        roots.push_back(0.5 * (lo + hi));
      }
    }
    std::vector<double> pts;
    pts.push_back(0.0);
    pts.insert(pts.end(), roots.begin(), roots.end());
    pts.push_back(1.0);
    for (size_t a = 0; a + 1 < pts.size(); ++a) {
      const double s0 = pts[a], s1 = pts[a + 1];
      if ((phi(0.5 * (s0 + s1)) < 0.0) == (loc_f == INSIDE))
        for (int q = 0; q < n1; ++q) cq[c].push_back({s0 + (s1 - s0) * gx[q], (s1 - s0) * gw[q]});
    }
    for (double r : roots) {
      const double e = 1e-7;
      const double g = phi(std::min(r + e, 1.0)) - phi(std::max(r - e, 0.0));
      cs[c].push_back({r, g > 0.0 ? 1.0 : -1.0});
    }
  }
  for (int c = 0; c < n; ++c) ++S.cells[S.loc[c] == INSIDE ? 0 : (S.loc[c] == INTERSECTED ? 1 : 2)];
  auto cat_of = [&](int c) { return (int)category((unsigned)c, (unsigned)p, (unsigned)n); };
  auto off_of = [&](int c) { return (int64_t)box_offset((unsigned)c, (unsigned)p, (unsigned)n); };
  std::vector<uint8_t> full_row((size_t)N, 0);
  for (int c = 0; c < n; ++c)
    if (S.loc[c] != loc_f)
      for (int i = 0; i < n1; ++i) full_row[(size_t)(off_of(c) + i)] = 1;
  for (int64_t r = 0; r < N; ++r)
    if (full_row[(size_t)r]) S.zero_rows.push_back(r);
  Slots C, M, K, X;
  C.init(1, N, p + 1);
  M.init(1, N, p + 1);
  K.init(1, N, p + 1);
  X.init(1, N, p + 1);
  std::vector<Trip> ff, fg, ev;
  Shapes sh{};
  const double gd = S.nitsche / h, tau = 0.5 * S.nitsche / h;
  // Nitsche terms of one Dirichlet point (normal nrm): into C (impl part, minus), K, and data column di
  auto dirichlet_point = [&](int c, double s, double nrm, double xg) {
    shapes_1d(p, cat_of(c), s, sh);
    const int64_t off = off_of(c), di = (int64_t)S.sx.size();
    S.sx.push_back(xg);
    S.sn.push_back(nrm);
    for (int i = 0; i < n1; ++i) {
      const double vi = sh.v[i], gi = sh.d[i] / h;
      fg.push_back({off + i, di, gd * vi - nrm * gi});
      for (int j = 0; j < n1; ++j) {
        const double vj = sh.v[j], gj = sh.d[j] / h;
        const double a = -nrm * gi * vj - nrm * vi * gj + gd * vi * vj;
        C.add(off + i, off + j, -a);
        K.add(off + i, off + j, a);
      }
    }
  };
  for (int c = 0; c < n; ++c) {
    if (S.loc[c] == inv) continue;
    const int cat = cat_of(c);
    const int64_t off = off_of(c);
    const double x0 = S.lo + c * h;
    for (const auto &q : cq[c]) {
      shapes_1d(p, cat, q.first, sh);
      const double jxw = q.second * h;
      const int64_t qi = (int64_t)S.qx.size();
      S.qx.push_back(x0 + q.first * h);
      S.qw.push_back(jxw);
      for (int i = 0; i < n1; ++i) {
        const double gi = sh.d[i] / h;
        ff.push_back({off + i, qi, sh.v[i] * jxw});
        ev.push_back({qi, off + i, sh.v[i]});
        for (int j = 0; j < n1; ++j) {
          const double gj = sh.d[j] / h;
          if (S.loc[c] == INTERSECTED || full_row[(size_t)(off + i)]) C.add(off + i, off + j, -gi * gj * jxw);
          M.add(off + i, off + j, sh.v[i] * sh.v[j] * jxw);
          K.add(off + i, off + j, gi * gj * jxw);
        }
      }
    }
    if (S.dirichlet & 1)
      for (const auto &sp : cs[c]) dirichlet_point(c, sp.first, loc_f == INSIDE ? sp.second : -sp.second, x0 + sp.first * h);
    if (S.dirichlet & 2) {
      // boundary faces whose point lies in the region (the level set's sign there)
      if (c == 0 && ((ls_values[0] < 0.0) == (loc_f == INSIDE)) && ls_values[0] != 0.0)
        dirichlet_point(c, 0.0, -1.0, S.lo);
      if (c == n - 1) {
        const double v1 = ls_values[(size_t)c * (k + 1) + k];
        if ((v1 < 0.0) == (loc_f == INSIDE) && v1 != 0.0) dirichlet_point(c, 1.0, 1.0, S.lo + n * h);
      }
    }
    if (S.coupled && S.loc[c] == INTERSECTED)
      for (const auto &sp : cs[c]) {
        // r_own -= (-0.5 n v' [u] -+ v n {u'} +- tau v [u]), [u] = u_in - u_out, {u'} = (u_in' + u_out') / 2
        shapes_1d(p, cat, sp.first, sh);
        const double nr = sp.second, sg = loc_f == INSIDE ? 1.0 : -1.0;
        for (int i = 0; i < n1; ++i) {
          const double vi = sh.v[i], gi = sh.d[i] / h;
          for (int j = 0; j < n1; ++j) {
            const double vj = sh.v[j], gj = sh.d[j] / h;
            // coefficients of u_in_j and u_out_j in the bracket
            const double a_in = -0.5 * nr * gi * vj - sg * 0.5 * nr * vi * gj + sg * tau * vi * vj;
            const double a_out = 0.5 * nr * gi * vj - sg * 0.5 * nr * vi * gj - sg * tau * vi * vj;
            C.add(off + i, off + j, -(loc_f == INSIDE ? a_in : a_out));
            X.add(off + i, off + j, -(loc_f == INSIDE ? a_out : a_in));
          }
        }
      }
  }
  // ghost penalty faces (mass.h:86-105, stiffness.h:80-98): every face of a
  // cell not of location inv to a neighbour where one of the two is
  // intersected and the other not of location inv, visited from both cells
  for (int c = 0; c < n; ++c) {
    if (S.loc[c] == inv) continue;
    for (int f = 0; f < 2; ++f) {
      const int nb = f == 0 ? c - 1 : c + 1;
      if (nb < 0 || nb >= n) continue;
      const int ln = S.loc[nb];
      if (!((S.loc[c] == INTERSECTED && ln != inv) || (ln == INTERSECTED && S.loc[c] != inv))) continue;
      // [dphi/dx] at the face: from cell c minus from the neighbour, per global DoF
      std::map<int64_t, double> jump;
      const double sc = (double)f, sn = 1.0 - f;  // face point in c's / the neighbour's reference coordinate
      shapes_1d(p, cat_of(c), sc, sh);
      for (int i = 0; i < n1; ++i) jump[off_of(c) + i] += sh.d[i] / h;
      shapes_1d(p, cat_of(nb), sn, sh);
      for (int i = 0; i < n1; ++i) jump[off_of(nb) + i] -= sh.d[i] / h;
      for (const auto &a : jump)
        for (const auto &b : jump) {
          C.add(a.first, b.first, -0.5 * S.gA * h * a.second * b.second);
          if (S.gM >= 0.0) M.add(a.first, b.first, 0.5 * S.gM * h * h * h * a.second * b.second);
          K.add(a.first, b.first, 0.5 * S.gA * h * h * h * a.second * b.second);
        }
    }
  }
  C.csr(S.c_rp, S.c_ci, S.c_v, false);
  M.csr(S.m_rp, S.m_ci, S.m_v, true);
  K.csr(S.s_rp, S.s_ci, S.s_v, true);
  X.csr(S.x_rp, S.x_ci, S.x_v, false);
  triplets_csr(ff, N, S.ff_rp, S.ff_ci, S.ff_v);
  triplets_csr(fg, N, S.fg_rp, S.fg_ci, S.fg_v);
  triplets_csr(ev, (int64_t)S.qx.size(), S.e_rp, S.e_ci, S.e_v);
}

// dim = 2: cells (cx, cy) lexicographic, DoF (ix, iy) -> ix + N iy; the
// caller's level-set values per cell at the (k+1)^2 Gauss-Lobatto points
// (a along x fastest); quadrature by saye_poly (gdm_cut.cpp), the region of
// S.location from the same pass.  Field, data and coupling terms as in
// assemble1d: interface data on the surface points (normal flipped for
// OUTSIDE), domain data on the boundary faces in the region (QGauss(p+1) on
// the face, outward normal; the face's location from the Bernstein
// coefficients of the level set on it -- an intersected boundary face is
// refused), the composite coupling on the surface points of intersected cells.
void assemble2d(gdm_cut_wave_system &S, const double *ls_values) {
  const int p = S.p, n = S.n, k = S.k, n1 = p + 1, nd = n1 * n1, nk = (k + 1) * (k + 1);
  const int loc_f = S.location, inv = -loc_f;
  const int64_t N = n + 1, NN = N * N;
  const double h = S.h;
  std::vector<double> gx, gw;
  gauss_unit(n1, gx, gw);
  const std::vector<double> gl = gauss_lobatto(k + 1);
  S.loc.assign((size_t)n * n, OUTSIDE);
  std::vector<std::vector<QPoint>> cq((size_t)n * n);
  std::vector<std::vector<SPoint>> cs((size_t)n * n);
  std::vector<QPoint> other;
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx) {
      const size_t c = (size_t)cy * n + cx;
      const double *vals = ls_values + c * nk;
      S.loc[c] = (int8_t)bernstein_location(2, k, vals, gl);
      if (S.loc[c] == loc_f) {
        for (int b = 0; b < n1; ++b)
          for (int a = 0; a < n1; ++a) cq[c].push_back({gx[a], gx[b], gw[a] * gw[b]});
      } else if (S.loc[c] == INTERSECTED) {
        TensorPoly f;
        f.interpolate(k, vals, gl);
        if (loc_f == INSIDE) {
          saye_poly(f, gx, gw, cq[c], cs[c], &S.n_splits);
        } else {
          saye_poly(f, gx, gw, other, cs[c], &S.n_splits, &cq[c]);
        }
      }
    }
  for (int8_t l : S.loc) ++S.cells[l == INSIDE ? 0 : (l == INTERSECTED ? 1 : 2)];
  auto cat_of = [&](int c) { return (int)category((unsigned)c, (unsigned)p, (unsigned)n); };
  auto off_of = [&](int c) { return (int64_t)box_offset((unsigned)c, (unsigned)p, (unsigned)n); };
  auto dofs = [&](int cx, int cy, int64_t *d) {
    for (int iy = 0; iy < n1; ++iy)
      for (int ix = 0; ix < n1; ++ix) d[iy * n1 + ix] = (off_of(cy) + iy) * N + off_of(cx) + ix;
  };
  std::vector<uint8_t> full_row((size_t)NN, 0);
  int64_t d[100], e[100];
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx)
      if (S.loc[(size_t)cy * n + cx] != loc_f) {
        dofs(cx, cy, d);
        for (int i = 0; i < nd; ++i) full_row[(size_t)d[i]] = 1;
      }
  for (int64_t r = 0; r < NN; ++r)
    if (full_row[(size_t)r]) S.zero_rows.push_back(r);
  Slots C, M, K, X;
  C.init(2, N, p + 1);
  M.init(2, N, p + 1);
  K.init(2, N, p + 1);
  X.init(2, N, p + 1);
  std::vector<Trip> ff, fg, ev;
  std::vector<double> val(nd), grx(nd), gry(nd), dn(nd);
  auto eval = [&](int cx, int cy, double s, double t) {
    Shapes sx, sy;
    shapes_1d(p, cat_of(cx), s, sx);
    shapes_1d(p, cat_of(cy), t, sy);
    for (int iy = 0; iy < n1; ++iy)
      for (int ix = 0; ix < n1; ++ix) {
        const int i = iy * n1 + ix;
        val[i] = sx.v[ix] * sy.v[iy];
        grx[i] = sx.d[ix] * sy.v[iy] / h;
        gry[i] = sx.v[ix] * sy.d[iy] / h;
      }
  };
  const double gd = S.nitsche / h, tau = 0.5 * S.nitsche / h;
  // Nitsche terms of one Dirichlet point (after eval; normal (nx, ny), weight
  // jxw at global (xg, yg)): -(-d_n v u - d_n u v + gamma_D / h v u) into C, +
  // into K, the data (gamma_D / h v - d_n v) into column si of Fg
  auto dirichlet_point = [&](double nx, double ny, double jxw, double xg, double yg) {
    const int64_t si = (int64_t)S.sx.size() / 2;
    S.sx.push_back(xg);
    S.sx.push_back(yg);
    S.sn.push_back(nx);
    S.sn.push_back(ny);
    for (int i = 0; i < nd; ++i) dn[i] = grx[i] * nx + gry[i] * ny;
    for (int i = 0; i < nd; ++i) {
      fg.push_back({d[i], si, (gd * val[i] - dn[i]) * jxw});
      for (int j = 0; j < nd; ++j) {
        const double a = (-dn[i] * val[j] - val[i] * dn[j] + gd * val[i] * val[j]) * jxw;
        C.add(d[i], d[j], -a);
        K.add(d[i], d[j], a);
      }
    }
  };
  const double sg = loc_f == INSIDE ? 1.0 : -1.0;
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx) {
      const size_t c = (size_t)cy * n + cx;
      if (S.loc[c] == inv) continue;
      dofs(cx, cy, d);
      const double x0 = S.lo + cx * h, y0 = S.lo + cy * h;
      for (const QPoint &q : cq[c]) {
        eval(cx, cy, q.s, q.t);
        const double jxw = q.w * h * h;
        const int64_t qi = (int64_t)S.qw.size();
        S.qx.push_back(x0 + q.s * h);
        S.qx.push_back(y0 + q.t * h);
        S.qw.push_back(jxw);
        for (int i = 0; i < nd; ++i) {
          ff.push_back({d[i], qi, val[i] * jxw});
          ev.push_back({qi, d[i], val[i]});
          const bool crow = S.loc[c] == INTERSECTED || full_row[(size_t)d[i]];
          for (int j = 0; j < nd; ++j) {
            const double gg = grx[i] * grx[j] + gry[i] * gry[j];
            if (crow) C.add(d[i], d[j], -gg * jxw);
            M.add(d[i], d[j], val[i] * val[j] * jxw);
            K.add(d[i], d[j], gg * jxw);
          }
        }
      }
      if (S.dirichlet & 1)
        for (const SPoint &sp : cs[c]) {
          eval(cx, cy, sp.s, sp.t);
          dirichlet_point(sg * sp.nx, sg * sp.ny, sp.w * h, x0 + sp.s * h, y0 + sp.t * h);
        }
      if (S.dirichlet & 2)
        for (int f = 0; f < 4; ++f) {
          const int axis = f / 2, side = f % 2;
          if ((axis == 0 ? cx : cy) != (side == 0 ? 0 : n - 1)) continue;
          // the level set on the face: the support points with s (axis 0) or t (axis 1) = side
          const double *vals = ls_values + c * nk;
          double line[10];
          for (int a = 0; a <= k; ++a)
            line[a] = axis == 0 ? vals[(side ? k : 0) + (k + 1) * a] : vals[a + (k + 1) * (side ? k : 0)];
          const int where = bernstein_location(1, k, line, gl);
          if (where == INTERSECTED)
            throw std::invalid_argument("cut_wave: the level set crosses a domain boundary face (not supported)");
          if (where != loc_f) continue;
          const double nv = 2.0 * side - 1.0;
          for (int q = 0; q < n1; ++q) {
            const double s = axis == 0 ? (double)side : gx[q], t = axis == 0 ? gx[q] : (double)side;
            eval(cx, cy, s, t);
            dirichlet_point(axis == 0 ? nv : 0.0, axis == 0 ? 0.0 : nv, gw[q] * h, x0 + s * h, y0 + t * h);
          }
        }
      if (S.coupled)
        for (const SPoint &sp : cs[c]) {
          // r_own -= (-0.5 d_n v [u] -+ v n.{grad u} +- tau v [u]), [u] = u_in - u_out,
          // {grad u} = (grad u_in + grad u_out) / 2, n the level-set normal
          eval(cx, cy, sp.s, sp.t);
          const double jxw = sp.w * h;
          for (int i = 0; i < nd; ++i) dn[i] = grx[i] * sp.nx + gry[i] * sp.ny;
          for (int i = 0; i < nd; ++i)
            for (int j = 0; j < nd; ++j) {
              const double vdn = dn[i] * val[j], vnd = val[i] * dn[j], vv = val[i] * val[j];
              const double a_in = (-0.5 * vdn - sg * 0.5 * vnd + sg * tau * vv) * jxw;
              const double a_out = (0.5 * vdn - sg * 0.5 * vnd - sg * tau * vv) * jxw;
              C.add(d[i], d[j], -(loc_f == INSIDE ? a_in : a_out));
              X.add(d[i], d[j], -(loc_f == INSIDE ? a_out : a_in));
            }
        }
    }
  // ghost penalty faces (mass.h:86-105, stiffness.h:80-98, 330-395): QGauss(p+1)
  // on every face of a cell not of location inv to a neighbour where one of the
  // two is intersected and the other not of location inv, visited from both cells
  std::map<int64_t, std::vector<double>> jump;
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx) {
      const int lc = S.loc[(size_t)cy * n + cx];
      if (lc == inv) continue;
      for (int f = 0; f < 4; ++f) {
        const int axis = f / 2, side = f % 2;
        const int nx = cx + (axis == 0 ? 2 * side - 1 : 0), ny = cy + (axis == 1 ? 2 * side - 1 : 0);
        if (nx < 0 || nx >= n || ny < 0 || ny >= n) continue;
        const int ln = S.loc[(size_t)ny * n + nx];
        if (!((lc == INTERSECTED && ln != inv) || (ln == INTERSECTED && lc != inv))) continue;
        jump.clear();
        dofs(cx, cy, d);
        dofs(nx, ny, e);
        for (int q = 0; q < n1; ++q) {
          // [d phi / dx_axis] at face point q: from the cell minus from the neighbour
          const double sc = axis == 0 ? (double)side : gx[q], tc = axis == 0 ? gx[q] : (double)side;
          const double sn = axis == 0 ? 1.0 - side : gx[q], tn = axis == 0 ? gx[q] : 1.0 - side;
          eval(cx, cy, sc, tc);
          for (int i = 0; i < nd; ++i) {
            auto &jv = jump[d[i]];
            jv.resize(n1, 0.0);
            jv[q] += axis == 0 ? grx[i] : gry[i];
          }
          eval(nx, ny, sn, tn);
          for (int i = 0; i < nd; ++i) {
            auto &jv = jump[e[i]];
            jv.resize(n1, 0.0);
            jv[q] -= axis == 0 ? grx[i] : gry[i];
          }
        }
        for (const auto &a : jump)
          for (const auto &b : jump) {
            double J = 0.0;
            for (int q = 0; q < n1; ++q) J += a.second[q] * b.second[q] * gw[q] * h;
            C.add(a.first, b.first, -0.5 * S.gA * h * J);
            if (S.gM >= 0.0) M.add(a.first, b.first, 0.5 * S.gM * h * h * h * J);
            K.add(a.first, b.first, 0.5 * S.gA * h * h * h * J);
          }
      }
    }
  C.csr(S.c_rp, S.c_ci, S.c_v, false);
  M.csr(S.m_rp, S.m_ci, S.m_v, true);
  K.csr(S.s_rp, S.s_ci, S.s_v, true);
  X.csr(S.x_rp, S.x_ci, S.x_v, false);
  triplets_csr(ff, NN, S.ff_rp, S.ff_ci, S.ff_v);
  triplets_csr(fg, NN, S.fg_rp, S.fg_ci, S.fg_v);
  triplets_csr(ev, (int64_t)S.qw.size(), S.e_rp, S.e_ci, S.e_v);
}

}  // namespace

extern "C" {

// banded Cholesky of a CSR SPD matrix (half-bandwidth taken from the pattern):
// lband [n][bw + 1], L(i, i - bw + k); returns bw, -1 if not positive definite,
// -2 if n (bw + 1) exceeds kBandMaxEntries (the mesh is too large for the dense band)
constexpr int64_t kBandMaxEntries = int64_t(1) << 28;
int64_t gdmh_band_cholesky(int64_t n, const int64_t *rp, const uint32_t *ci, const double *v, double alpha,
                           const int64_t *rp2, const uint32_t *ci2, const double *v2, std::vector<double> &lband);

int gdmh_cut_wave_create(int dim, int p, int n_sub, double lo, double hi, int ls_degree, const double *ls_values,
                         int location, int flags, double gamma_M, double gamma_A, double nitsche,
                         gdm_cut_wave_system **out, char *err, size_t err_len) {
  try {
    if ((location != INSIDE && location != OUTSIDE) || (flags & ~7))
      throw std::invalid_argument("cut_wave: location must be -1 (inside) or 1 (outside), flags in bits 0-2");
    if (!out || !ls_values || (dim != 1 && dim != 2) || p < 1 || p > 9 || p % 2 == 0 || n_sub < p || !(hi > lo) ||
        ls_degree < 1 || ls_degree > 9)
      throw std::invalid_argument(
          "cut_wave: invalid arguments (dim 1 or 2, p odd in [1, 9], n_sub >= p, hi > lo, 1 <= k <= 9)");
    if (dim == 2 && (int64_t)(n_sub + 1) * (n_sub + 1) > (int64_t)1 << 31)
      throw std::invalid_argument("cut_wave: mesh too large for 32-bit column indices");
    auto *S = new gdm_cut_wave_system();
    S->dim = dim;
    S->location = location;
    S->dirichlet = flags & 3;
    S->coupled = (flags & 4) != 0;
    S->p = p;
    S->n = n_sub;
    S->k = ls_degree;
    S->lo = lo;
    S->h = (hi - lo) / n_sub;
    S->gM = gamma_M;
    S->gA = gamma_A;
    S->nitsche = nitsche;
    try {
      if (dim == 1)
        assemble1d(*S, ls_values);
      else
        assemble2d(*S, ls_values);
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

void gdmh_cut_wave_info(const gdm_cut_wave_system *S, int64_t *n_dofs, int64_t *n_quad, int64_t *n_surface,
                        int64_t *cells) {
  *n_dofs = S->dim == 1 ? S->n + 1 : (int64_t)(S->n + 1) * (S->n + 1);
  *n_quad = (int64_t)S->qw.size();
  *n_surface = (int64_t)S->sx.size() / S->dim;
  for (int q = 0; q < 3; ++q) cells[q] = S->cells[q];
}

// which: 0 C, 1 Ff, 2 Fg, 3 E, 4 M, 5 K (stiffness matrix), 6 X (coupling to the partner field)
void gdmh_cut_wave_csr(const gdm_cut_wave_system *S, int which, const int64_t **rp, const uint32_t **ci,
                       const double **v) {
  switch (which) {
    case 0: *rp = S->c_rp.data(); *ci = S->c_ci.data(); *v = S->c_v.data(); return;
    case 1: *rp = S->ff_rp.data(); *ci = S->ff_ci.data(); *v = S->ff_v.data(); return;
    case 2: *rp = S->fg_rp.data(); *ci = S->fg_ci.data(); *v = S->fg_v.data(); return;
    case 3: *rp = S->e_rp.data(); *ci = S->e_ci.data(); *v = S->e_v.data(); return;
    case 4: *rp = S->m_rp.data(); *ci = S->m_ci.data(); *v = S->m_v.data(); return;
    case 5: *rp = S->s_rp.data(); *ci = S->s_ci.data(); *v = S->s_v.data(); return;
    default: *rp = S->x_rp.data(); *ci = S->x_ci.data(); *v = S->x_v.data(); return;
  }
}

void gdmh_cut_wave_points(const gdm_cut_wave_system *S, const double **qx, const double **qw, const double **sx,
                          const double **sn, const int64_t **zero_rows, int64_t *n_zero) {
  *qx = S->qx.data();
  *qw = S->qw.data();
  *sx = S->sx.data();
  *sn = S->sn.data();
  *zero_rows = S->zero_rows.data();
  *n_zero = (int64_t)S->zero_rows.size();
}

int gdmh_cut_wave_splits(const gdm_cut_wave_system *S) { return S->n_splits; }

void gdmh_cut_wave_destroy(gdm_cut_wave_system *S) { delete S; }

int64_t gdmh_band_cholesky(int64_t n, const int64_t *rp, const uint32_t *ci, const double *v, double alpha,
                           const int64_t *rp2, const uint32_t *ci2, const double *v2, std::vector<double> &lband) {
  // A = M + alpha K (rp2 may be NULL: A = M)
  int64_t bw = 0;
  for (int64_t r = 0; r < n; ++r) {
    for (int64_t q = rp[r]; q < rp[r + 1]; ++q) bw = std::max<int64_t>(bw, r - (int64_t)ci[q]);
    if (rp2)
      for (int64_t q = rp2[r]; q < rp2[r + 1]; ++q) bw = std::max<int64_t>(bw, r - (int64_t)ci2[q]);
  }
  const int64_t W = bw + 1;
  // the band is dense inside (O(n bw) memory, O(n bw^2) work, bw ~ p (n_sub + 1)
  // in 2D): refuse factors beyond kBandMaxEntries doubles (2 GiB) instead of an
  // out-of-memory death or a multi-hour factorisation
  if (n * W > kBandMaxEntries) return -2;
  std::vector<double> A((size_t)n * W, 0.0);
  for (int64_t r = 0; r < n; ++r) {
    for (int64_t q = rp[r]; q < rp[r + 1]; ++q)
      if ((int64_t)ci[q] <= r) A[(size_t)r * W + (ci[q] - r + bw)] += v[q];
    if (rp2)
      for (int64_t q = rp2[r]; q < rp2[r + 1]; ++q)
        if ((int64_t)ci2[q] <= r) A[(size_t)r * W + (ci2[q] - r + bw)] += alpha * v2[q];
  }
  lband.assign((size_t)n * W, 0.0);
  double *L = lband.data();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j0 = std::max<int64_t>(0, i - bw);
    for (int64_t j = j0; j <= i; ++j) {
      double s = A[(size_t)i * W + (j - i + bw)];
      const int64_t k0 = std::max(j0, j - bw);
      const double *Li = L + (size_t)i * W - i + bw;
      const double *Lj = L + (size_t)j * W - j + bw;
      for (int64_t k = k0; k < j; ++k) s -= Li[k] * Lj[k];
      if (j < i) {
        L[(size_t)i * W + (j - i + bw)] = s / Lj[j];
      } else {
        if (!(s > 0.0)) return -1;
        L[(size_t)i * W + bw] = std::sqrt(s);
      }
    }
  }
  return bw;
}

}  // extern "C"
