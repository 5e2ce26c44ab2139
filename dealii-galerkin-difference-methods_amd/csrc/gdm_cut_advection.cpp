// gdm_cut_advection.cpp -- host assembly of the cut-cell parts of the 2D
// advection application (applications/advection, alpha = 0) for the device
// operator of gdm_capi.cpp ("Cut-cell advection" in include/gdm_hip.h).
// Composite (advection-app.cc's preset, problem.h:103-181): one system per
// field; the outside field is this assembly on the negated level set (its
// inside = the outside of the level set, the surface normal flipped as in
// stiffness.h:437, the ghost-penalty faces and the mass of
// MassMatrixOperator(location = outside)), and the inflow value u+ of the
// cut-surface term (II) is the partner field (stiffness.h:448-453): a
// coupling matrix P instead of stage boundary points.
//
// The device evaluates compute_rhs (advection/stiffness.h:196-606) as
//   rhs = Z (S u) + C u + F bc
// with S the uncut fused Kronecker stencil of the whole box (the advection
// operator kind of gdm_op with the box outflow traces, no inflow data), Z the
// projection that zeroes the rows of DoFs in the box of a cell that is not
// fully inside (`zero_rows`), and the two sparse matrices assembled here:
//   C = the cut operator's rows of those DoFs in full -- the volume term (I)
//       and the outflow box-face term (III) of every inside cell, their cut
//       versions on intersected cells, the outflow part of the cut surface
//       term (II) -- plus the ghost penalty (IV), -0.5 gamma_A h^2
//       [d_n v][d_n u] on interior faces with an intersected cell and a
//       non-outside neighbour, visited from both cells (stiffness.h:534-598).
//       (A correction form C = K_cut - K_box on top of the unprojected S
//       cancels the full-cell terms of outside / cut cells in fp64; the cut
//       mass matrix (cond 1e12 at p = 5) amplified that rounding to 1e-3 of
//       the surface error norms of test_01.)
//   F = the inflow (a.n < 0) parts of (II) and (III), one column per stage
//       boundary point, points in the reference's point_counter order (per
//       cell: surface points, then the boundary faces; stiffness.h:40-160)
// and the mass solve (advection/problem.h:236-267) as an exact banded
// Cholesky solve of the cut mass matrix (mass.h:47-243: (v, u)_inside +
// 0.5 gamma_M h^3 [d_n v][d_n u], zero diagonals -> 1), the reference's
// `SolverDirect` branch; the factor is computed here, the triangular solves
// run on the device.
//
// Quadrature: QGauss(p+1)^2 on inside cells, deal.II's QuadratureGenerator
// (Saye, gdm_cut.cpp saye_unit) on intersected cells, QGauss(p+1) on the
// inside sub-intervals of boundary faces (NonMatching::FEInterfaceValues),
// QGauss(p+1) on full faces for the ghost penalty.  Level set = the FE_Q(1)
// interpolant given by its vertex values.  Test oracle:
// oracle/cut_advection2d.py, pinned by applications/advection/tests/
// test_01.output.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "gdm_cut.h"
#include "gdm_setup.h"

struct gdm_cut_adv_system {
  int p = 0, n = 0;
  bool composite = false;  // (II)'s inflow value is the partner field's u (coupling P), not stage data
  double lo = 0.0, h = 0.0, a[2] = {0.0, 0.0}, gA = 0.0, gM = 0.0;
  std::vector<double> ls;   // vertex level set [iy][ix]
  std::vector<int8_t> loc;  // [cy][cx]
  std::vector<int64_t> c_rp, f_rp;
  std::vector<uint32_t> c_ci, f_ci;
  std::vector<double> c_v, f_v;
  std::vector<double> bc_xy;  // [n_bc][2]
  int64_t bw = 0;             // half-bandwidth of the mass factor
  std::vector<double> lband;  // [n_rows][bw + 1]: L(i, i - bw + k)
  int64_t n_inside = 0, n_intersected = 0, n_outside = 0;
  std::vector<int64_t> zero_rows;  // rows of S u the device zeroes (C holds them in full)
  std::vector<int64_t> m_rp;  // the assembled cut mass matrix (host checks)
  std::vector<uint32_t> m_ci;
  std::vector<double> m_v;
  std::vector<int64_t> p_rp;  // composite: the partner coupling of (II), rhs += P u_partner
  std::vector<uint32_t> p_ci;
  std::vector<double> p_v;
};

namespace {

using namespace gdm;

// rows x (2R+1)^2 slot accumulator of a 2D operator whose couplings stay
// within |dx|, |dy| <= R
struct SlotMatrix {
  int64_t N = 0, rows = 0;
  int R = 0, SW = 0, SL = 0;
  std::vector<double> v;
  std::vector<uint8_t> touched;
  void init(int64_t N_, int R_) {
    N = N_;
    rows = N_ * N_;
    R = R_;
    SW = 2 * R + 1;
    SL = SW * SW;
    v.assign((size_t)rows * SL, 0.0);
    touched.assign((size_t)rows * SL, 0);
  }
  void add(int64_t row, int64_t col, double x) {
    const int64_t ry = row / N, rx = row % N, cy = col / N, cx = col % N;
    const int64_t k = (cy - ry + R) * SW + (cx - rx + R);
    v[(size_t)row * SL + k] += x;
    touched[(size_t)row * SL + k] = 1;
  }
  // CSR of the touched entries, columns ascending; unit_diag: every diagonal, zero -> 1
  void csr(std::vector<int64_t> &rp, std::vector<uint32_t> &ci, std::vector<double> &vals, bool unit_diag) const {
    rp.assign((size_t)rows + 1, 0);
    ci.clear();
    vals.clear();
    for (int64_t row = 0; row < rows; ++row) {
      const int64_t ry = row / N, rx = row % N;
      for (int k = 0; k < SL; ++k) {
        const int dy = k / SW - R, dx = k % SW - R;
        const bool diag = dx == 0 && dy == 0;
        if (!touched[(size_t)row * SL + k] && !(diag && unit_diag)) continue;
        const int64_t cy = ry + dy, cx = rx + dx;
        if (cy < 0 || cy >= N || cx < 0 || cx >= N) continue;
        double x = v[(size_t)row * SL + k];
        if (diag && unit_diag && x == 0.0) x = 1.0;
        ci.push_back((uint32_t)(cy * N + cx));
        vals.push_back(x);
      }
      rp[(size_t)row + 1] = (int64_t)ci.size();
    }
  }
};

void assemble(gdm_cut_adv_system &S) {
  const int p = S.p, n = S.n, N = n + 1, n1 = p + 1, nd = n1 * n1;
  const double h = S.h, ax = S.a[0], ay = S.a[1];
  std::vector<double> qx, qw;
  gauss_unit(n1, qx, qw);
  SlotMatrix C, M, Pc;
  C.init(N, p + 1);
  M.init(N, p + 1);
  if (S.composite) Pc.init(N, p + 1);
  struct FEntry {
    int64_t row, col;
    double v;
  };
  std::vector<FEntry> fent;
  std::vector<double> val(nd), gx(nd), gy(nd);
  auto eval = [&](int catx, int caty, double s, double t) {
    Shapes sx{}, sy{};
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
  auto dofs = [&](int cx, int cy, int64_t *d) {
    const int ox = (int)box_offset((unsigned)cx, (unsigned)p, (unsigned)n);
    const int oy = (int)box_offset((unsigned)cy, (unsigned)p, (unsigned)n);
    for (int iy = 0; iy < n1; ++iy)
      for (int ix = 0; ix < n1; ++ix) d[iy * n1 + ix] = (int64_t)(oy + iy) * N + (ox + ix);
  };
  auto lsv = [&](int ix, int iy) { return S.ls[(size_t)iy * N + ix]; };
  // inside part of face f of a cell: [(s, t, reference weight)]
  auto face_quadrature = [&](int cx, int cy, int f, std::vector<QPoint> &out) {
    out.clear();
    double f0, f1;
    if (f < 2) {
      f0 = lsv(cx + f, cy);
      f1 = lsv(cx + f, cy + 1);
    } else {
      f0 = lsv(cx, cy + f - 2);
      f1 = lsv(cx + 1, cy + f - 2);
    }
    const double r = linear_root(f0, f1);
    double e[3];
    int ne = 0;
    e[ne++] = 0.0;
    if (r >= 0.0) e[ne++] = r;
    e[ne++] = 1.0;
    for (int k = 0; k + 1 < ne; ++k) {
      const double a = e[k], L = e[k + 1] - a;
      if (!(L > 0.0) || !(f0 + (f1 - f0) * (a + 0.5 * L) < 0.0)) continue;
      for (int q = 0; q < n1; ++q) {
        const double c = a + L * qx[q];
        out.push_back(f < 2 ? QPoint{(double)f, c, qw[q] * L} : QPoint{c, (double)(f - 2), qw[q] * L});
      }
    }
  };
  std::vector<QPoint> full_cell, ins, fq, ffull;
  std::vector<SPoint> sur;
  for (int b = 0; b < n1; ++b)
    for (int a = 0; a < n1; ++a) full_cell.push_back({qx[a], qx[b], qw[a] * qw[b]});
  const double nrm[4][2] = {{-1.0, 0.0}, {1.0, 0.0}, {0.0, -1.0}, {0.0, 1.0}};
  std::vector<double> Kl((size_t)nd * nd), Ml((size_t)nd * nd);
  int64_t d[256], e[256];
  int64_t n_bc = 0;
  // rows in the box of a cell that is not fully inside: C carries their whole cut row
  std::vector<uint8_t> full_row((size_t)N * N, 0);
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx)
      if (S.loc[(size_t)cy * n + cx] != INSIDE) {
        dofs(cx, cy, d);
        for (int i = 0; i < nd; ++i) full_row[(size_t)d[i]] = 1;
      }
  S.zero_rows.clear();
  for (int64_t r = 0; r < (int64_t)N * N; ++r)
    if (full_row[(size_t)r]) S.zero_rows.push_back(r);
  for (int cy = 0; cy < n; ++cy)
    for (int cx = 0; cx < n; ++cx) {
      const int loc = S.loc[(size_t)cy * n + cx];
      const int catx = (int)category((unsigned)cx, (unsigned)p, (unsigned)n);
      const int caty = (int)category((unsigned)cy, (unsigned)p, (unsigned)n);
      dofs(cx, cy, d);
      const bool at_bnd[4] = {cx == 0, cx == n - 1, cy == 0, cy == n - 1};
      std::fill(Kl.begin(), Kl.end(), 0.0);
      std::fill(Ml.begin(), Ml.end(), 0.0);
      // volume term (I) (a u, grad v) and mass (v, u) over a quadrature, scaled by sign
      auto volume = [&](const std::vector<QPoint> &Q, double sgn, bool mass) {
        for (const QPoint &q : Q) {
          eval(catx, caty, q.s, q.t);
          const double w = q.w * h * h;
          for (int i = 0; i < nd; ++i) {
            const double agi = (ax * gx[i] + ay * gy[i]) * w * sgn;
            for (int j = 0; j < nd; ++j) {
              Kl[(size_t)i * nd + j] += agi * val[j];
              if (mass) Ml[(size_t)i * nd + j] += val[i] * val[j] * w;
            }
          }
        }
      };
      // outflow part (flux >= 0) of an upwind boundary term on K: -flux phi_i phi_j w; inflow -> F columns
      auto upwind = [&](double s, double t, double flux, double w, double sgn, bool inflow_data) {
        eval(catx, caty, s, t);
        if (flux >= 0.0) {
          for (int i = 0; i < nd; ++i)
            for (int j = 0; j < nd; ++j) Kl[(size_t)i * nd + j] -= sgn * flux * val[i] * val[j] * w;
        } else if (inflow_data) {
          for (int i = 0; i < nd; ++i)
            if (val[i] != 0.0) fent.push_back({d[i], n_bc, -flux * val[i] * w});
        }
      };
      auto add_point = [&](double s, double t) {
        S.bc_xy.push_back(S.lo + (cx + s) * h);
        S.bc_xy.push_back(S.lo + (cy + t) * h);
      };
      if (loc == OUTSIDE) {
        ++S.n_outside;  // no terms (its rows are zeroed in S u and carry the cut terms of their other cells)
      } else {
        if (loc == INSIDE) {
          ++S.n_inside;
          volume(full_cell, 1.0, true);  // (I) == S's cell term: kept below for the full rows only
        } else {
          ++S.n_intersected;
          const double v00 = lsv(cx, cy), v10 = lsv(cx + 1, cy), v01 = lsv(cx, cy + 1), v11 = lsv(cx + 1, cy + 1);
          Bilinear fl{v00, v10 - v00, v01 - v00, v11 - v10 - v01 + v00};
          saye_unit(fl, qx, qw, ins, sur);
          volume(ins, 1.0, true);
          for (const SPoint &q : sur) {  // (II) cut surface
            const double flux = q.nx * ax + q.ny * ay;
            if (S.composite) {
              // u+ = the partner field at the point (stiffness.h:448-453): the inflow part couples to its
              // DoFs through this cell's basis, no stage boundary point (collect_boundary_points :115)
              upwind(q.s, q.t, flux, q.w * h, 1.0, false);
              if (flux < 0.0)
                for (int i = 0; i < nd; ++i)
                  for (int j = 0; j < nd; ++j) Pc.add(d[i], d[j], -flux * val[i] * val[j] * q.w * h);
            } else {
              add_point(q.s, q.t);
              upwind(q.s, q.t, flux, q.w * h, 1.0, true);
              ++n_bc;
            }
          }
        }
        for (int f = 0; f < 4; ++f) {  // (III) box faces: outflow into K, inflow into F
          if (!at_bnd[f]) continue;
          const double flux = nrm[f][0] * ax + nrm[f][1] * ay;
          face_quadrature(cx, cy, f, fq);
          for (const QPoint &q : fq) {
            add_point(q.s, q.t);
            upwind(q.s, q.t, flux, q.w * h, 1.0, true);
            ++n_bc;
          }
        }
        // (IV) ghost penalty on the faces to (intersected | non-outside) neighbours
        const int nb[4][2] = {{cx - 1, cy}, {cx + 1, cy}, {cx, cy - 1}, {cx, cy + 1}};
        for (int f = 0; f < 4; ++f) {
          const int nx = nb[f][0], ny = nb[f][1];
          if (nx < 0 || ny < 0 || nx >= n || ny >= n) continue;
          const int lb = S.loc[(size_t)ny * n + nx];
          if (!((loc == INTERSECTED && lb != OUTSIDE) || (lb == INTERSECTED && loc != OUTSIDE))) continue;
          dofs(nx, ny, e);
          const int c1x = (int)category((unsigned)nx, (unsigned)p, (unsigned)n);
          const int c1y = (int)category((unsigned)ny, (unsigned)p, (unsigned)n);
          const int axis = f < 2 ? 0 : 1, side = f % 2;
          std::vector<double> jump((size_t)2 * nd), S2((size_t)4 * nd * nd, 0.0);
          for (int q = 0; q < n1; ++q) {
            const double s0 = axis == 0 ? side : qx[q], t0 = axis == 0 ? qx[q] : side;
            const double s1 = axis == 0 ? 1 - side : qx[q], t1 = axis == 0 ? qx[q] : 1 - side;
            eval(catx, caty, s0, t0);
            for (int i = 0; i < nd; ++i) jump[i] = axis == 0 ? gx[i] : gy[i];
            eval(c1x, c1y, s1, t1);
            for (int i = 0; i < nd; ++i) jump[nd + i] = -(axis == 0 ? gx[i] : gy[i]);
            const double w = qw[q] * h;
            for (int i = 0; i < 2 * nd; ++i)
              for (int j = 0; j < 2 * nd; ++j) S2[(size_t)i * 2 * nd + j] += jump[i] * jump[j] * w;
          }
          for (int i = 0; i < 2 * nd; ++i)
            for (int j = 0; j < 2 * nd; ++j) {
              const int64_t r = i < nd ? d[i] : e[i - nd], c = j < nd ? d[j] : e[j - nd];
              const double x = S2[(size_t)i * 2 * nd + j];
              C.add(r, c, -0.5 * S.gA * h * h * x);
              M.add(r, c, 0.5 * S.gM * h * h * h * x);
            }
        }
      }
      if (loc != OUTSIDE)
        for (int i = 0; i < nd; ++i) {
          // inside cells: S u carries row d[i] unless it is a full row
          const bool to_c = loc == INTERSECTED || full_row[(size_t)d[i]];
          for (int j = 0; j < nd; ++j) {
            if (to_c) C.add(d[i], d[j], Kl[(size_t)i * nd + j]);
            M.add(d[i], d[j], Ml[(size_t)i * nd + j]);
          }
        }
    }
  C.csr(S.c_rp, S.c_ci, S.c_v, false);
  M.csr(S.m_rp, S.m_ci, S.m_v, true);
  if (S.composite) Pc.csr(S.p_rp, S.p_ci, S.p_v, false);
  // F: CSR rows = DoFs, columns = boundary points (ascending point index)
  std::sort(fent.begin(), fent.end(), [](const FEntry &x, const FEntry &y) {
    return x.row != y.row ? x.row < y.row : x.col < y.col;
  });
  const int64_t rows = (int64_t)N * N;
  S.f_rp.assign((size_t)rows + 1, 0);
  S.f_ci.clear();
  S.f_v.clear();
  for (size_t k = 0; k < fent.size(); ++k) {
    if (k > 0 && fent[k - 1].row == fent[k].row && fent[k - 1].col == fent[k].col) {
      S.f_v.back() += fent[k].v;
      continue;
    }
    S.f_ci.push_back((uint32_t)fent[k].col);
    S.f_v.push_back(fent[k].v);
    ++S.f_rp[(size_t)fent[k].row + 1];
  }
  for (int64_t r = 0; r < rows; ++r) S.f_rp[(size_t)r + 1] += S.f_rp[(size_t)r];
  // banded Cholesky of the cut mass matrix: M = L L^T, L(i, j) for j in [i - bw, i]
  int64_t bw = 0;
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t k = S.m_rp[(size_t)r]; k < S.m_rp[(size_t)r + 1]; ++k)
      bw = std::max<int64_t>(bw, r - (int64_t)S.m_ci[(size_t)k]);
  S.bw = bw;
  const int64_t W = bw + 1;
  std::vector<double> A((size_t)rows * W, 0.0);  // lower band of M, row form
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t k = S.m_rp[(size_t)r]; k < S.m_rp[(size_t)r + 1]; ++k) {
      const int64_t c = S.m_ci[(size_t)k];
      if (c <= r) A[(size_t)r * W + (c - r + bw)] = S.m_v[(size_t)k];
    }
  S.lband.assign((size_t)rows * W, 0.0);
  double *L = S.lband.data();
  for (int64_t i = 0; i < rows; ++i) {
    const int64_t j0 = std::max<int64_t>(0, i - bw);
    for (int64_t j = j0; j <= i; ++j) {
      double s = A[(size_t)i * W + (j - i + bw)];
      const int64_t k0 = std::max(j0, j - bw);
      const double *Li = L + (size_t)i * W - i + bw;  // Li[k] = L(i, k)
      const double *Lj = L + (size_t)j * W - j + bw;
      for (int64_t k = k0; k < j; ++k) s -= Li[k] * Lj[k];
      if (j < i) {
        L[(size_t)i * W + (j - i + bw)] = s / Lj[j];
      } else {
        if (!(s > 0.0)) throw std::runtime_error("cut advection: mass matrix not positive definite");
        L[(size_t)i * W + bw] = std::sqrt(s);
      }
    }
  }
}

}  // namespace

extern "C" {

int gdmh_cut_adv_create(int p, int n_sub, double lo, double hi, const double *level_set, const double *advection,
                        double gamma_A, double gamma_M, int composite, gdm_cut_adv_system **out, char *err,
                        size_t err_len) {
  try {
    if (!out || !level_set || !advection || p < 1 || p > 9 || p % 2 == 0 || n_sub < p || !(hi > lo))
      throw std::invalid_argument("cut_advection: invalid arguments (p odd in [1, 9], n_sub >= p, hi > lo)");
    if ((int64_t)(n_sub + 1) * (n_sub + 1) > (int64_t)1 << 22)
      throw std::invalid_argument("cut_advection: at most 2^22 DoFs (the direct banded mass solve)");
    auto *S = new gdm_cut_adv_system();
    S->p = p;
    S->n = n_sub;
    S->lo = lo;
    S->h = (hi - lo) / n_sub;
    S->a[0] = advection[0];
    S->a[1] = advection[1];
    S->gA = gamma_A;
    S->gM = gamma_M;
    S->composite = composite != 0;
    const int N = n_sub + 1;
    S->ls.assign(level_set, level_set + (size_t)N * N);
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
      assemble(*S);
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

void gdmh_cut_adv_info(const gdm_cut_adv_system *S, int64_t *n_dofs, int64_t *n_bc, int64_t *cells,
                       int64_t *bandwidth) {
  *n_dofs = (int64_t)(S->n + 1) * (S->n + 1);
  *n_bc = (int64_t)S->bc_xy.size() / 2;
  cells[0] = S->n_inside;
  cells[1] = S->n_intersected;
  cells[2] = S->n_outside;
  *bandwidth = S->bw;
}

void gdmh_cut_adv_arrays(const gdm_cut_adv_system *S, const int64_t **c_rp, const uint32_t **c_ci,
                         const double **c_v, const int64_t **f_rp, const uint32_t **f_ci, const double **f_v,
                         const double **bc_xy, const double **lband) {
  *c_rp = S->c_rp.data();
  *c_ci = S->c_ci.data();
  *c_v = S->c_v.data();
  *f_rp = S->f_rp.data();
  *f_ci = S->f_ci.data();
  *f_v = S->f_v.data();
  *bc_xy = S->bc_xy.data();
  *lband = S->lband.data();
}

void gdmh_cut_adv_zero_rows(const gdm_cut_adv_system *S, const int64_t **rows, int64_t *n) {
  *rows = S->zero_rows.data();
  *n = (int64_t)S->zero_rows.size();
}

void gdmh_cut_adv_mass(const gdm_cut_adv_system *S, const int64_t **rp, const uint32_t **ci, const double **v) {
  *rp = S->m_rp.data();
  *ci = S->m_ci.data();
  *v = S->m_v.data();
}

// composite: rhs += P u_partner (rows = DoFs, columns = the partner's DoFs); empty otherwise
void gdmh_cut_adv_coupling(const gdm_cut_adv_system *S, const int64_t **rp, const uint32_t **ci, const double **v,
                           int64_t *nnz) {
  *rp = S->p_rp.data();
  *ci = S->p_ci.data();
  *v = S->p_v.data();
  *nnz = S->p_rp.empty() ? 0 : S->p_rp.back();
}

void gdmh_cut_adv_destroy(gdm_cut_adv_system *S) { delete S; }

}  // extern "C"
