/*
 * gdm_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference algorithm on the GDM hot path, used as the
 * parity checker by tests/, by __graft_entry__.smoke() and as the cpu_baseline
 * leg of bench.py.  Nothing in the product (the HIP library and its host
 * wrappers) links, imports or calls this file.
 *
 * Every routine restates a specific part of peterrum/dealii-galerkin-difference-
 * methods (paths relative to the reference root):
 *   - basis:          include/gdm/fe.h:55-336 (tables produced by
 *                     scripts/create_coefficients.py:7-39, Lagrange polynomials
 *                     through the p+1 nodes {j - category})
 *   - indexing:       include/gdm/system.h:195-246 (get_dof_indices),
 *                     system.h:404-424 (categorize), fe.h:339-397 (lex index)
 *   - partition:      include/gdm/system.h:703-757 (z-slab ownership)
 *   - quadrature:     deal.II QGauss(p+1) on the unit cell, MappingQ1 on an
 *                     axis-aligned uniform grid (advection/discretization.h:82-83)
 *   - advection rhs:  applications/advection/include/gdm/advection/stiffness.h
 *                     :345-418 (cell term, alpha = 0) and :473-532 (box faces)
 *   - convective rhs: prototypes/advection_01_gdm.cc:164-206
 *   - wave rhs:       applications/wave/include/gdm/wave/stiffness.h:151-203
 *                     (cell term -(grad v, grad u)) and :261-330 (Nitsche on box)
 *   - mass matrix:    include/gdm/matrix_creator.h:9-62 and
 *                     applications/advection/include/gdm/advection/mass.h:47-243
 *   - CG:             deal.II SolverCG + ReductionControl semantics as used at
 *                     applications/advection/include/gdm/advection/problem.h:236-267
 *
 * The cell loops are deliberately the reference's O((p+1)^(2 dim)) per-cell
 * FEValues-style evaluation (full shape tables, gather -> quadrature -> test ->
 * scatter-add), not the Kronecker form used by the GPU product.
 *
 * Parity of this restatement is pinned by tests/test_oracle_golden.py against
 * the reference's own golden outputs (tests/poly_01.output, fe_02_gdm.output,
 * poisson_01_gdm.output, mass_01_gdm.output, mass_02_gdm.output,
 * poisson_02_gdm.mpirun=*.output) and against scripts/create_coefficients.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAXP 9
#define MAXN (MAXP + 1)

/* ------------------------------------------------------------------------- */
/* 1D basis: monomial coefficients of the Lagrange polynomial through nodes   */
/* t_j = j - cat, j = 0..p  (fe.h tables; create_coefficients.py:15-24).      */
/* ------------------------------------------------------------------------- */
static void lagrange_monomial(int p, int cat, int i, double *coef /* p+1, ascending */)
{
  double c[MAXN + 1];
  memset(c, 0, sizeof(c));
  c[0] = 1.0;
  int deg = 0;
  double denom = 1.0;
  for (int j = 0; j <= p; ++j) {
    if (j == i)
      continue;
    const double tj = (double)(j - cat);
    /* multiply polynomial by (x - tj) */
    for (int k = deg + 1; k >= 1; --k)
      c[k] = c[k - 1] - tj * c[k];
    c[0] = -tj * c[0];
    deg++;
    denom *= (double)(i - j);
  }
  for (int k = 0; k <= p; ++k)
    coef[k] = c[k] / denom;
}

double gdmo_basis_derivative(int p, int cat, int i, double x, int order)
{
  double c[MAXN + 1];
  lagrange_monomial(p, cat, i, c);
  /* differentiate `order` times */
  int deg = p;
  for (int o = 0; o < order; ++o) {
    for (int k = 0; k < deg; ++k)
      c[k] = c[k + 1] * (double)(k + 1);
    deg--;
  }
  if (deg < 0)
    return 0.0;
  double r = c[deg];
  for (int k = deg - 1; k >= 0; --k)
    r = r * x + c[k];
  return r;
}

double gdmo_basis_value(int p, int cat, int i, double x)
{
  return gdmo_basis_derivative(p, cat, i, x, 0);
}

/* ascending monomial coefficients (for comparison with fe.h / the sympy script) */
void gdmo_basis_coefficients(int p, int cat, int i, double *coef)
{
  lagrange_monomial(p, cat, i, coef);
}

/* ------------------------------------------------------------------------- */
/* Gauss-Legendre on [0,1] with n points (deal.II QGauss<1>(n)), ascending.   */
/* ------------------------------------------------------------------------- */
void gdmo_gauss(int n, double *x, double *w)
{
  for (int i = 0; i < n; ++i) {
    /* i-th root (descending on [-1,1]) via Newton from the Chebyshev guess */
    double z = cos(M_PI * (i + 0.75) / (n + 0.5));
    double pp = 0.0;
    for (int it = 0; it < 100; ++it) {
      double p1 = 1.0, p2 = 0.0;
      for (int j = 1; j <= n; ++j) {
        const double p3 = p2;
        p2 = p1;
        p1 = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
      }
      pp = n * (z * p1 - p2) / (z * z - 1.0);
      const double z1 = z;
      z = z1 - p1 / pp;
      if (fabs(z - z1) < 1e-16)
        break;
    }
    {
      double p1 = 1.0, p2 = 0.0;
      for (int j = 1; j <= n; ++j) {
        const double p3 = p2;
        p2 = p1;
        p1 = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
      }
      pp = n * (z * p1 - p2) / (z * z - 1.0);
    }
    /* map to [0,1]: ascending order -> index n-1-i gets -z */
    x[i] = 0.5 * (1.0 - z);
    w[i] = 1.0 / ((1.0 - z * z) * pp * pp);
  }
}

/* ------------------------------------------------------------------------- */
/* System indexing (system.h:195-246, 404-424).                               */
/* ------------------------------------------------------------------------- */
unsigned gdmo_category(unsigned c, unsigned p, unsigned n)
{
  const unsigned h = p / 2;
  return (c < h) ? c : ((c < n - h) ? h : (p + c - n));
}

unsigned gdmo_offset(unsigned c, unsigned p, unsigned n)
{
  const unsigned h = p / 2;
  if (c < h)
    return 0;
  unsigned e = c + h + 1;
  if (e > n)
    e = n;
  return e - p;
}

/* global dof indices of a cell, lexicographic x-fastest inside the box */
void gdmo_cell_dof_indices(int dim, int p, const unsigned *nsub, unsigned cell, uint64_t *out)
{
  unsigned idx[3] = {0, 0, 0};
  unsigned rem = cell;
  for (int d = 0; d < dim; ++d) {
    idx[d] = rem % nsub[d];
    rem /= nsub[d];
  }
  unsigned off[3] = {0, 0, 0}, N[3] = {1, 1, 1};
  for (int d = 0; d < dim; ++d) {
    off[d] = gdmo_offset(idx[d], (unsigned)p, nsub[d]);
    N[d] = nsub[d] + 1;
  }
  const int nk = (dim >= 3) ? p : 0, nj = (dim >= 2) ? p : 0;
  int c = 0;
  for (int k = 0; k <= nk; ++k)
    for (int j = 0; j <= nj; ++j)
      for (int i = 0; i <= p; ++i, ++c) {
        const uint64_t gx = off[0] + i, gy = off[1] + j, gz = off[2] + k;
        out[c] = gx + (uint64_t)N[0] * (gy + (uint64_t)N[1] * gz);
      }
}

unsigned gdmo_fe_index(int dim, int p, const unsigned *nsub, unsigned cell)
{
  unsigned rem = cell, f = 0, mul = 1;
  for (int d = 0; d < dim; ++d) {
    const unsigned c = rem % nsub[d];
    rem /= nsub[d];
    f += gdmo_category(c, (unsigned)p, nsub[d]) * mul;
    mul *= (unsigned)p;
  }
  return f;
}

/* z-slab (last-coordinate) partition, system.h:720-757.
 * out[0..1] = owned vertex-plane range [b,e), out[2..3] = owned cell-plane range */
void gdmo_partition(unsigned n_last, unsigned n_procs, unsigned rank, unsigned *out)
{
  const unsigned stride = (n_last + n_procs - 1) / n_procs;
  unsigned rs = (rank == 0) ? 0 : stride * rank + 1;
  unsigned re = stride * (rank + 1) + 1;
  if (rs > n_last + 1)
    rs = n_last + 1;
  if (re > n_last + 1)
    re = n_last + 1;
  out[0] = rs;
  out[1] = re;
  unsigned cb = stride * rank, ce = stride * (rank + 1);
  if (cb > n_last)
    cb = n_last;
  if (ce > n_last)
    ce = n_last;
  out[2] = cb;
  out[3] = ce;
}

/* ------------------------------------------------------------------------- */
/* Per-cell shape tables (FEValues restatement on a uniform Cartesian grid).  */
/* ------------------------------------------------------------------------- */
typedef struct {
  int dim, p, nq1, nd;    /* nd = (p+1)^dim dofs = nq */
  double xq[MAXN], wq[MAXN];
  /* 1D tables per category: v[cat][i][q], g[cat][i][q] (reference coords) */
  double v1[MAXP][MAXN][MAXN], g1[MAXP][MAXN][MAXN];
  /* boundary traces per category: value at x=0 and x=1 */
  double t0[MAXP][MAXN], t1[MAXP][MAXN];
} tables_t;

static void build_tables(tables_t *T, int dim, int p)
{
  T->dim = dim;
  T->p = p;
  T->nq1 = p + 1;
  T->nd = 1;
  for (int d = 0; d < dim; ++d)
    T->nd *= (p + 1);
  gdmo_gauss(p + 1, T->xq, T->wq);
  const int ncat = (p == 1) ? 1 : p;
  for (int c = 0; c < ncat; ++c)
    for (int i = 0; i <= p; ++i) {
      for (int q = 0; q <= p; ++q) {
        T->v1[c][i][q] = gdmo_basis_derivative(p, c, i, T->xq[q], 0);
        T->g1[c][i][q] = gdmo_basis_derivative(p, c, i, T->xq[q], 1);
      }
      T->t0[c][i] = gdmo_basis_derivative(p, c, i, 0.0, 0);
      T->t1[c][i] = gdmo_basis_derivative(p, c, i, 1.0, 0);
    }
}

static void cell_coords(int dim, const unsigned *nsub, unsigned cell, unsigned *cidx)
{
  unsigned rem = cell;
  for (int d = 0; d < 3; ++d)
    cidx[d] = 0;
  for (int d = 0; d < dim; ++d) {
    cidx[d] = rem % nsub[d];
    rem /= nsub[d];
  }
}

/* shape value / gradient of local dof i at cell quadrature point q */
static void shape_at(const tables_t *T, const unsigned *cat, int i, int q, const double *h,
                     double *val, double *grad)
{
  const int n1 = T->p + 1;
  int ii[3] = {0, 0, 0}, qq[3] = {0, 0, 0};
  int ri = i, rq = q;
  for (int d = 0; d < T->dim; ++d) {
    ii[d] = ri % n1;
    ri /= n1;
    qq[d] = rq % n1;
    rq /= n1;
  }
  double v = 1.0;
  for (int d = 0; d < T->dim; ++d)
    v *= T->v1[cat[d]][ii[d]][qq[d]];
  *val = v;
  if (grad)
    for (int e = 0; e < T->dim; ++e) {
      double g = 1.0;
      for (int d = 0; d < T->dim; ++d)
        g *= (d == e) ? T->g1[cat[d]][ii[d]][qq[d]] / h[d] : T->v1[cat[d]][ii[d]][qq[d]];
      grad[e] = g;
    }
}

/* reference-cell coordinates of face quadrature point qf on face f
 * (deal.II QProjector::project_to_face ordering, tensor QGauss<dim-1>(p+1)) */
static void face_point(int dim, int f, int qf, int n1, int *qq /* per-dim 1D index or -1 */)
{
  const int d = f / 2;
  int a = qf % n1, b = qf / n1;
  qq[0] = qq[1] = qq[2] = 0;
  if (dim == 1) {
    qq[0] = -1;
  } else if (dim == 2) {
    qq[d] = -1;
    qq[1 - d] = a;
  } else {
    if (d == 0) {
      qq[0] = -1; qq[1] = a; qq[2] = b;
    } else if (d == 1) {
      qq[1] = -1; qq[0] = b; qq[2] = a;
    } else {
      qq[2] = -1; qq[0] = a; qq[1] = b;
    }
  }
}

static int n_face_q(int dim, int p)
{
  int n = 1;
  for (int d = 0; d < dim - 1; ++d)
    n *= (p + 1);
  return n;
}

/* value of local dof i at face point (qq: -1 marks the face-normal direction) */
static double face_shape(const tables_t *T, const unsigned *cat, int i, const int *qq, int side)
{
  const int n1 = T->p + 1;
  int ri = i;
  double v = 1.0;
  for (int d = 0; d < T->dim; ++d) {
    const int id = ri % n1;
    ri /= n1;
    if (qq[d] < 0)
      v *= side ? T->t1[cat[d]][id] : T->t0[cat[d]][id];
    else
      v *= T->v1[cat[d]][id][qq[d]];
  }
  return v;
}

static double face_jxw(const tables_t *T, int dim, int f, const int *qq, const double *h)
{
  double j = 1.0;
  for (int d = 0; d < dim; ++d)
    if (d != f / 2)
      j *= h[d] * T->wq[qq[d]];
  return j;
}

static void cell_setup(int dim, int p, const unsigned *nsub, unsigned cell, const double *lo,
                       const double *hi, unsigned *cidx, unsigned *cat, double *h)
{
  cell_coords(dim, nsub, cell, cidx);
  for (int d = 0; d < 3; ++d) {
    cat[d] = 0;
    h[d] = 1.0;
  }
  for (int d = 0; d < dim; ++d) {
    cat[d] = gdmo_category(cidx[d], (unsigned)p, nsub[d]);
    h[d] = (hi[d] - lo[d]) / nsub[d];
  }
}

static unsigned n_cells_total(int dim, const unsigned *nsub)
{
  unsigned n = 1;
  for (int d = 0; d < dim; ++d)
    n *= nsub[d];
  return n;
}

static unsigned cell_last_coord(int dim, const unsigned *nsub, unsigned cell)
{
  unsigned cidx[3];
  cell_coords(dim, nsub, cell, cidx);
  return cidx[dim - 1];
}

/* number of boundary face points the reference stores in block(0) for the
 * cells whose last coordinate is in [cb, ce) (stiffness.h:40-160, uncut) */
uint64_t gdmo_n_boundary_points(int dim, int p, const unsigned *nsub, unsigned cb, unsigned ce)
{
  uint64_t n = 0;
  const unsigned nc = n_cells_total(dim, nsub);
  const int nfq = n_face_q(dim, p);
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3];
    cell_coords(dim, nsub, c, cidx);
    if (cidx[dim - 1] < cb || cidx[dim - 1] >= ce)
      continue;
    for (int f = 0; f < 2 * dim; ++f) {
      const int d = f / 2;
      const int at = (f % 2 == 0) ? (cidx[d] == 0) : (cidx[d] == nsub[d] - 1);
      if (at)
        n += nfq;
    }
  }
  return n;
}

/* physical coordinates of the stored boundary points, reference order */
void gdmo_boundary_points(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                          unsigned cb, unsigned ce, double *xyz /* n x 3 */)
{
  tables_t T;
  build_tables(&T, dim, p);
  const unsigned nc = n_cells_total(dim, nsub);
  const int nfq = n_face_q(dim, p), n1 = p + 1;
  uint64_t k = 0;
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    double h[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    if (cidx[dim - 1] < cb || cidx[dim - 1] >= ce)
      continue;
    for (int f = 0; f < 2 * dim; ++f) {
      const int d = f / 2;
      const int at = (f % 2 == 0) ? (cidx[d] == 0) : (cidx[d] == nsub[d] - 1);
      if (!at)
        continue;
      for (int q = 0; q < nfq; ++q, ++k) {
        int qq[3];
        face_point(dim, f, q, n1, qq);
        for (int e = 0; e < 3; ++e) {
          double r;
          if (e >= dim)
            r = 0.0;
          else if (qq[e] < 0)
            r = (f % 2) ? 1.0 : 0.0;
          else
            r = T.xq[qq[e]];
          xyz[3 * k + e] = (e < dim) ? lo[e] + (cidx[e] + r) * h[e] : 0.0;
        }
      }
    }
  }
}

/* ------------------------------------------------------------------------- */
/* Advection alpha-form rhs (stiffness.h:196-606, uncut, alpha = 0, constant  */
/* advection field a).  rhs += ... for cells with last coordinate in [cb,ce). */
/* stage_bc: boundary values in reference order for those cells.              */
/* ------------------------------------------------------------------------- */
int gdmo_advection_rhs(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                       const double *a, const double *u, const double *stage_bc, double *rhs,
                       unsigned cb, unsigned ce)
{
  tables_t T;
  build_tables(&T, dim, p);
  const int nd = T.nd, n1 = p + 1, nfq = n_face_q(dim, p);
  const unsigned nc = n_cells_total(dim, nsub);
  uint64_t *dofs = (uint64_t *)malloc(sizeof(uint64_t) * nd);
  double *ul = (double *)malloc(sizeof(double) * nd);
  double *cv = (double *)malloc(sizeof(double) * nd);
  double *sv = (double *)malloc(sizeof(double) * nd * nd);
  double *sg = (double *)malloc(sizeof(double) * nd * nd * 3);
  double uq, gq[3], fv[3];
  uint64_t pc = 0; /* point_counter, stiffness.h:337 */
  unsigned prev_cat[3] = {~0u, ~0u, ~0u};
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    double h[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    if (cidx[dim - 1] < cb || cidx[dim - 1] >= ce)
      continue;
    if (cat[0] != prev_cat[0] || cat[1] != prev_cat[1] || cat[2] != prev_cat[2]) {
      for (int i = 0; i < nd; ++i)
        for (int q = 0; q < nd; ++q)
          shape_at(&T, cat, i, q, h, &sv[i * nd + q], &sg[3 * (i * nd + q)]);
      memcpy(prev_cat, cat, sizeof(cat));
    }
    double jxw_vol = 1.0;
    for (int d = 0; d < dim; ++d)
      jxw_vol *= h[d];
    gdmo_cell_dof_indices(dim, p, nsub, c, dofs);
    for (int i = 0; i < nd; ++i) {
      ul[i] = u[dofs[i]];
      cv[i] = 0.0;
    }
    /* (I) cell integral: cell_i += (a u_q) . grad phi_i JxW   (alpha = 0) */
    for (int q = 0; q < nd; ++q) {
      int rq = q;
      double wq = jxw_vol;
      for (int d = 0; d < dim; ++d) {
        wq *= T.wq[rq % n1];
        rq /= n1;
      }
      uq = 0.0;
      for (int e = 0; e < dim; ++e)
        gq[e] = 0.0;
      for (int j = 0; j < nd; ++j) {
        uq += ul[j] * sv[j * nd + q];
        for (int e = 0; e < dim; ++e)
          gq[e] += ul[j] * sg[3 * (j * nd + q) + e];
      }
      for (int e = 0; e < dim; ++e)
        fv[e] = uq * a[e];
      for (int i = 0; i < nd; ++i) {
        double s = 0.0;
        for (int e = 0; e < dim; ++e)
          s += fv[e] * sg[3 * (i * nd + q) + e];
        cv[i] += s * wq;
      }
    }
    /* (III) box faces (stiffness.h:473-532) */
    for (int f = 0; f < 2 * dim; ++f) {
      const int d = f / 2, side = f % 2;
      const int at = side ? (cidx[d] == nsub[d] - 1) : (cidx[d] == 0);
      if (!at)
        continue;
      const double an = side ? a[d] : -a[d]; /* a . n */
      for (int q = 0; q < nfq; ++q) {
        int qq[3];
        face_point(dim, f, q, n1, qq);
        const double jxw = face_jxw(&T, dim, f, qq, h);
        double uval = 0.0;
        for (int j = 0; j < nd; ++j)
          uval += ul[j] * face_shape(&T, cat, j, qq, side);
        const double uplus = stage_bc ? stage_bc[pc] : 0.0;
        pc++;
        const double upw = (an >= 0.0) ? uval : uplus;
        for (int i = 0; i < nd; ++i)
          cv[i] += an * (0.0 * uval - upw) * face_shape(&T, cat, i, qq, side) * jxw;
      }
    }
    for (int i = 0; i < nd; ++i)
      rhs[dofs[i]] += cv[i];
  }
  free(dofs);
  free(ul);
  free(cv);
  free(sv);
  free(sg);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* The inflow-data part of gdmo_advection_rhs alone: term (III) of            */
/* stiffness.h:473-532 with u = 0, i.e. rhs_i -= (a.n) u+ phi_i JxW on the box */
/* faces with a.n < 0.  Only the boundary cells are visited, in cell order,   */
/* with the reference's point_counter over every boundary face point          */
/* (stiffness.h:337), so stage_bc is the same reference-ordered block(0) as   */
/* gdmo_advection_rhs reads; the face shape values are cached per category    */
/* tuple and face.  Equals gdmo_advection_rhs(u = 0, stage_bc) term by term   */
/* (tests/test_oracle_golden.py), at the cost of the O(n^(dim-1)) boundary    */
/* cells: the full-size C3 inflow check of tests/test_gpu_fullsize.py.        */
/* ------------------------------------------------------------------------- */
int gdmo_advection_inflow(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                          const double *a, const double *stage_bc, double *rhs)
{
  tables_t T;
  build_tables(&T, dim, p);
  const int nd = T.nd, n1 = p + 1, nfq = n_face_q(dim, p);
  const int ncat = (p == 1) ? 1 : p;
  const size_t tsz = (size_t)nfq * nd;
  /* face shape tables, key (cat0, cat1, cat2, f), computed on first use */
  const size_t nkeys = (size_t)ncat * ncat * ncat * 6;
  double **fs = (double **)calloc(nkeys, sizeof(double *));
  uint64_t *dofs = (uint64_t *)malloc(sizeof(uint64_t) * nd);
  double *cv = (double *)malloc(sizeof(double) * nd);
  unsigned n[3] = {1, 1, 1};
  for (int d = 0; d < dim; ++d)
    n[d] = nsub[d];
  uint64_t pc = 0;
  /* rows of cells along x: a row is all boundary cells when any higher
   * coordinate is on the boundary, else only its first and last cell */
  for (unsigned cz = 0; cz < n[2]; ++cz)
    for (unsigned cy = 0; cy < n[1]; ++cy) {
      const int row_bdry = (dim >= 2 && (cy == 0 || cy == n[1] - 1)) || (dim >= 3 && (cz == 0 || cz == n[2] - 1));
      for (unsigned cx = 0; cx < n[0]; ++cx) {
        if (!row_bdry && cx != 0 && cx != n[0] - 1) {
          cx = n[0] - 2; /* skip the interior of the row */
          continue;
        }
        const unsigned c = cx + n[0] * (cy + n[1] * cz);
        unsigned cidx[3], cat[3];
        double h[3];
        cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
        int any = 0;
        for (int i = 0; i < nd; ++i)
          cv[i] = 0.0;
        for (int f = 0; f < 2 * dim; ++f) {
          const int d = f / 2, side = f % 2;
          const int at = side ? (cidx[d] == nsub[d] - 1) : (cidx[d] == 0);
          if (!at)
            continue;
          const double an = side ? a[d] : -a[d]; /* a . n */
          if (an >= 0.0) {
            pc += nfq; /* outflow face: u = 0 contributes nothing */
            continue;
          }
          const size_t key = (((size_t)cat[0] * ncat + cat[1]) * ncat + cat[2]) * 6 + f;
          if (!fs[key]) {
            fs[key] = (double *)malloc(sizeof(double) * tsz);
            for (int q = 0; q < nfq; ++q) {
              int qq[3];
              face_point(dim, f, q, n1, qq);
              for (int i = 0; i < nd; ++i)
                fs[key][(size_t)q * nd + i] = face_shape(&T, cat, i, qq, side);
            }
          }
          const double *tab = fs[key];
          for (int q = 0; q < nfq; ++q) {
            int qq[3];
            face_point(dim, f, q, n1, qq);
            const double jxw = face_jxw(&T, dim, f, qq, h);
            const double uplus = stage_bc[pc++];
            for (int i = 0; i < nd; ++i)
              cv[i] += an * (0.0 * 0.0 - uplus) * tab[(size_t)q * nd + i] * jxw;
          }
          any = 1;
        }
        if (!any)
          continue;
        gdmo_cell_dof_indices(dim, p, nsub, c, dofs);
        for (int i = 0; i < nd; ++i)
          rhs[dofs[i]] += cv[i];
      }
    }
  for (size_t k = 0; k < nkeys; ++k)
    free(fs[k]);
  free(fs);
  free(dofs);
  free(cv);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Convective-form rhs of prototypes/advection_01_gdm.cc:164-206:             */
/* cell_i -= (a . grad u_q) phi_i JxW  (no face terms; constraints applied by */
/* the caller).                                                                */
/* ------------------------------------------------------------------------- */
int gdmo_convective_rhs(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                        const double *a, const double *u, double *rhs)
{
  tables_t T;
  build_tables(&T, dim, p);
  const int nd = T.nd, n1 = p + 1;
  const unsigned nc = n_cells_total(dim, nsub);
  uint64_t *dofs = (uint64_t *)malloc(sizeof(uint64_t) * nd);
  double *ul = (double *)malloc(sizeof(double) * nd);
  double *cv = (double *)malloc(sizeof(double) * nd);
  double *sv = (double *)malloc(sizeof(double) * nd * nd);
  double *sg = (double *)malloc(sizeof(double) * nd * nd * 3);
  unsigned prev_cat[3] = {~0u, ~0u, ~0u};
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    double h[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    if (cat[0] != prev_cat[0] || cat[1] != prev_cat[1] || cat[2] != prev_cat[2]) {
      for (int i = 0; i < nd; ++i)
        for (int q = 0; q < nd; ++q)
          shape_at(&T, cat, i, q, h, &sv[i * nd + q], &sg[3 * (i * nd + q)]);
      memcpy(prev_cat, cat, sizeof(cat));
    }
    double jxw_vol = 1.0;
    for (int d = 0; d < dim; ++d)
      jxw_vol *= h[d];
    gdmo_cell_dof_indices(dim, p, nsub, c, dofs);
    for (int i = 0; i < nd; ++i) {
      ul[i] = u[dofs[i]];
      cv[i] = 0.0;
    }
    for (int q = 0; q < nd; ++q) {
      int rq = q;
      double wq = jxw_vol;
      for (int d = 0; d < dim; ++d) {
        wq *= T.wq[rq % n1];
        rq /= n1;
      }
      double flux = 0.0;
      for (int e = 0; e < dim; ++e) {
        double g = 0.0;
        for (int j = 0; j < nd; ++j)
          g += ul[j] * sg[3 * (j * nd + q) + e];
        flux += g * a[e];
      }
      for (int i = 0; i < nd; ++i)
        cv[i] -= flux * sv[i * nd + q] * wq;
    }
    for (int i = 0; i < nd; ++i)
      rhs[dofs[i]] += cv[i];
  }
  free(dofs);
  free(ul);
  free(cv);
  free(sv);
  free(sg);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Wave / heat rhs, uncut (wave/stiffness.h:151-203, 261-330):                 */
/*   cell_i -= grad phi_i . grad u_q JxW                 (compute_impl_part)  */
/*   cell_i += f_q phi_i JxW          (f given at cell quadrature points,      */
/*                                     cell-major order, nullable)             */
/*   box Nitsche (function_domain_dbc, nitsche > 0) with g at the boundary     */
/*   points in reference order (nullable g -> homogeneous data)               */
/* ------------------------------------------------------------------------- */
int gdmo_wave_rhs(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                  const double *u, int impl, const double *fq, double nitsche, const double *gbc,
                  double *rhs, unsigned cb, unsigned ce)
{
  tables_t T;
  build_tables(&T, dim, p);
  const int nd = T.nd, n1 = p + 1, nfq = n_face_q(dim, p);
  const unsigned nc = n_cells_total(dim, nsub);
  uint64_t *dofs = (uint64_t *)malloc(sizeof(uint64_t) * nd);
  double *ul = (double *)malloc(sizeof(double) * nd);
  double *cv = (double *)malloc(sizeof(double) * nd);
  double *sv = (double *)malloc(sizeof(double) * nd * nd);
  double *sg = (double *)malloc(sizeof(double) * nd * nd * 3);
  unsigned prev_cat[3] = {~0u, ~0u, ~0u};
  uint64_t pc = 0;
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    double h[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    if (cidx[dim - 1] < cb || cidx[dim - 1] >= ce)
      continue;
    if (cat[0] != prev_cat[0] || cat[1] != prev_cat[1] || cat[2] != prev_cat[2]) {
      for (int i = 0; i < nd; ++i)
        for (int q = 0; q < nd; ++q)
          shape_at(&T, cat, i, q, h, &sv[i * nd + q], &sg[3 * (i * nd + q)]);
      memcpy(prev_cat, cat, sizeof(cat));
    }
    double jxw_vol = 1.0, hmin = 1e300;
    for (int d = 0; d < dim; ++d) {
      jxw_vol *= h[d];
      if (h[d] < hmin)
        hmin = h[d];
    }
    gdmo_cell_dof_indices(dim, p, nsub, c, dofs);
    for (int i = 0; i < nd; ++i) {
      ul[i] = u[dofs[i]];
      cv[i] = 0.0;
    }
    for (int q = 0; q < nd; ++q) {
      int rq = q;
      double wq = jxw_vol;
      for (int d = 0; d < dim; ++d) {
        wq *= T.wq[rq % n1];
        rq /= n1;
      }
      double gq[3] = {0, 0, 0};
      for (int j = 0; j < nd; ++j)
        for (int e = 0; e < dim; ++e)
          gq[e] += ul[j] * sg[3 * (j * nd + q) + e];
      const double f = fq ? fq[(uint64_t)c * nd + q] : 0.0;
      for (int i = 0; i < nd; ++i) {
        if (impl) {
          double s = 0.0;
          for (int e = 0; e < dim; ++e)
            s += sg[3 * (i * nd + q) + e] * gq[e];
          cv[i] -= s * wq;
        }
        if (fq)
          cv[i] += f * sv[i * nd + q] * wq;
      }
    }
    if (nitsche > 0.0) {
      /* (IV) box faces, Nitsche: h = minimum vertex distance of the cell */
      for (int f = 0; f < 2 * dim; ++f) {
        const int d = f / 2, side = f % 2;
        const int at = side ? (cidx[d] == nsub[d] - 1) : (cidx[d] == 0);
        if (!at)
          continue;
        const double nrm = side ? 1.0 : -1.0;
        for (int q = 0; q < nfq; ++q, ++pc) {
          int qq[3];
          face_point(dim, f, q, n1, qq);
          const double jxw = face_jxw(&T, dim, f, qq, h);
          /* u, du/dn at the face point */
          double uval = 0.0, dun = 0.0;
          for (int j = 0; j < nd; ++j) {
            uval += ul[j] * face_shape(&T, cat, j, qq, side);
          }
          /* normal derivative: replace the face-normal factor by the 1D
           * derivative trace of the shape */
          for (int j = 0; j < nd; ++j) {
            int rj = j;
            double v = 1.0;
            for (int e = 0; e < dim; ++e) {
              const int id = rj % n1;
              rj /= n1;
              if (qq[e] < 0)
                v *= gdmo_basis_derivative(p, cat[e], id, (double)side, 1) / h[e];
              else
                v *= T.v1[cat[e]][id][qq[e]];
            }
            dun += ul[j] * v * nrm;
          }
          const double g = gbc ? gbc[pc] : 0.0;
          for (int i = 0; i < nd; ++i) {
            const double phi = face_shape(&T, cat, i, qq, side);
            int ri = i;
            double dphin = 1.0;
            for (int e = 0; e < dim; ++e) {
              const int id = ri % n1;
              ri /= n1;
              if (qq[e] < 0)
                dphin *= gdmo_basis_derivative(p, cat[e], id, (double)side, 1) / h[e];
              else
                dphin *= T.v1[cat[e]][id][qq[e]];
            }
            dphin *= nrm;
            if (impl)
              cv[i] -= (-dphin * uval - dun * phi + nitsche / hmin * phi * uval) * jxw;
            cv[i] += g * (nitsche / hmin * phi - dphin) * jxw;
          }
        }
      }
    }
    for (int i = 0; i < nd; ++i)
      rhs[dofs[i]] += cv[i];
  }
  free(dofs);
  free(ul);
  free(cv);
  free(sv);
  free(sg);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Mass / Laplace matrix assembly into a dense-row CSR with the full           */
/* structural stencil (system.h:586-599); matrix_creator.h:9-62.              */
/* kind 0 = mass (v,u), kind 1 = Laplace (grad v, grad u).                     */
/* Returns nnz; rowptr (n+1), cols, vals preallocated by caller with           */
/* capacity cap (call with cols == NULL to query nnz).                        */
/* ------------------------------------------------------------------------- */
int64_t gdmo_matrix_csr(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                        int kind, int64_t *rowptr, int64_t *cols, double *vals)
{
  /* sparsity: |i_d - j_d| <= p in every direction */
  unsigned N[3] = {1, 1, 1};
  int64_t n = 1;
  for (int d = 0; d < dim; ++d) {
    N[d] = nsub[d] + 1;
    n *= N[d];
  }
  int64_t nnz = 0;
  for (int64_t r = 0; r < n; ++r) {
    int64_t cnt = 1;
    int64_t rem = r;
    for (int d = 0; d < dim; ++d) {
      const int64_t id = rem % N[d];
      rem /= N[d];
      int64_t lo_ = id - p < 0 ? 0 : id - p, hi_ = id + p > (int64_t)N[d] - 1 ? N[d] - 1 : id + p;
      cnt *= (hi_ - lo_ + 1);
    }
    if (rowptr)
      rowptr[r] = nnz;
    nnz += cnt;
  }
  if (rowptr)
    rowptr[n] = nnz;
  if (!cols)
    return nnz;
  /* fill column indices (sorted) */
  for (int64_t r = 0; r < n; ++r) {
    int64_t id[3] = {0, 0, 0}, rem = r;
    for (int d = 0; d < dim; ++d) {
      id[d] = rem % N[d];
      rem /= N[d];
    }
    int64_t lo_[3] = {0, 0, 0}, hi_[3] = {0, 0, 0};
    for (int d = 0; d < dim; ++d) {
      lo_[d] = id[d] - p < 0 ? 0 : id[d] - p;
      hi_[d] = id[d] + p > (int64_t)N[d] - 1 ? N[d] - 1 : id[d] + p;
    }
    int64_t k = rowptr[r];
    for (int64_t z = lo_[2]; z <= hi_[2]; ++z)
      for (int64_t y = lo_[1]; y <= hi_[1]; ++y)
        for (int64_t x = lo_[0]; x <= hi_[0]; ++x) {
          cols[k] = x + (int64_t)N[0] * (y + (int64_t)N[1] * z);
          vals[k] = 0.0;
          ++k;
        }
  }
  tables_t T;
  build_tables(&T, dim, p);
  const int nd = T.nd, n1 = p + 1;
  const unsigned nc = n_cells_total(dim, nsub);
  uint64_t *dofs = (uint64_t *)malloc(sizeof(uint64_t) * nd);
  const unsigned ncat = MAXP;
  double **cache = (double **)calloc((size_t)ncat * ncat * ncat, sizeof(double *));
  /* element matrix in the reference's summation order (mass.h:160-170,
     matrix_creator.h:45-50): q outer, cell_matrix(i, j) += (phi_i phi_j) JxW
     for mass, (grad phi_i . grad phi_j) JxW for Laplace. On the uniform mesh
     the matrix depends only on the category tuple, so it is computed once per
     tuple present (bit-identical to recomputing it per cell; the tuples are
     independent, so they run in parallel), then scattered in cell order. */
  unsigned *keys = (unsigned *)malloc(sizeof(unsigned) * ncat * ncat * ncat);
  unsigned (*kcat)[3] = malloc(sizeof(unsigned[3]) * ncat * ncat * ncat);
  int n_keys = 0;
  double h[3];
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    const unsigned key = cat[0] + ncat * (cat[1] + ncat * cat[2]);
    if (!cache[key]) {
      cache[key] = (double *)calloc((size_t)nd * nd, sizeof(double));
      keys[n_keys] = key;
      memcpy(kcat[n_keys], cat, sizeof(cat));
      ++n_keys;
    }
  }
  double jxw_vol = 1.0;
  for (int d = 0; d < dim; ++d)
    jxw_vol *= h[d];
#pragma omp parallel for schedule(dynamic, 1)
  for (int t = 0; t < n_keys; ++t) {
    const unsigned *cat = kcat[t];
    double *m = cache[keys[t]];
    double *svT = (double *)malloc(sizeof(double) * nd * nd);
    double *sg = kind == 0 ? NULL : (double *)malloc(sizeof(double) * nd * nd * 3);
    for (int i = 0; i < nd; ++i)
      for (int q = 0; q < nd; ++q)
        shape_at(&T, cat, i, q, h, &svT[q * nd + i], kind == 0 ? NULL : &sg[3 * (i * nd + q)]);
    for (int q = 0; q < nd; ++q) {
      int rq = q;
      double wq = jxw_vol;
      for (int d = 0; d < dim; ++d) {
        wq *= T.wq[rq % n1];
        rq /= n1;
      }
      const double *sq = &svT[q * nd];
      for (int i = 0; i < nd; ++i) {
        double *mi = &m[(size_t)i * nd];
        if (kind == 0) {
          const double a = sq[i];
          for (int j = 0; j < nd; ++j)
            mi[j] += a * sq[j] * wq;
        } else {
          const double *gi = &sg[3 * (i * nd + q)];
          for (int j = 0; j < nd; ++j) {
            const double *gj = &sg[3 * (j * nd + q)];
            double s = 0.0;
            for (int e = 0; e < dim; ++e)
              s += gi[e] * gj[e];
            mi[j] += s * wq;
          }
        }
      }
    }
    free(svT);
    free(sg);
  }
  free(keys);
  free(kcat);
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    const unsigned key = cat[0] + ncat * (cat[1] + ncat * cat[2]);
    const double *cm = cache[key];
    gdmo_cell_dof_indices(dim, p, nsub, c, dofs);
    for (int i = 0; i < nd; ++i) {
      /* row r's columns are its |i_d - j_d| <= p box, sorted z, y, x: the
         position of column c is arithmetic */
      const int64_t r = (int64_t)dofs[i];
      int64_t id[3] = {0, 0, 0}, rem = r, lo_[3] = {0, 0, 0}, w[3] = {1, 1, 1};
      for (int d = 0; d < dim; ++d) {
        id[d] = rem % N[d];
        rem /= N[d];
        lo_[d] = id[d] - p < 0 ? 0 : id[d] - p;
        const int64_t hi_ = id[d] + p > (int64_t)N[d] - 1 ? N[d] - 1 : id[d] + p;
        w[d] = hi_ - lo_[d] + 1;
      }
      for (int j = 0; j < nd; ++j) {
        int64_t cj = (int64_t)dofs[j], jd[3] = {0, 0, 0};
        for (int d = 0; d < dim; ++d) {
          jd[d] = cj % N[d];
          cj /= N[d];
        }
        const int64_t k = rowptr[r] + ((jd[2] - lo_[2]) * w[1] + (jd[1] - lo_[1])) * w[0] + (jd[0] - lo_[0]);
        vals[k] += cm[i * nd + j];
      }
    }
  }
  for (unsigned k = 0; k < ncat * ncat * ncat; ++k)
    free(cache[k]);
  free(cache);
  free(dofs);
  return nnz;
}

void gdmo_csr_vmult(int64_t n, const int64_t *rowptr, const int64_t *cols, const double *vals,
                    const double *x, double *y)
{
  for (int64_t r = 0; r < n; ++r) {
    double s = 0.0;
    for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k)
      s += vals[k] * x[cols[k]];
    y[r] = s;
  }
}

/* ------------------------------------------------------------------------- */
/* deal.II SolverCG with ReductionControl(max_it, abs_tol, rel_tol); x is    */
/* the initial guess (zero in all reference call sites).                       */
/* precond: 0 identity, 1 Jacobi (PreconditionJacobi, omega = 1).             */
/* Returns the number of iterations (last_step), or -1 on no convergence.     */
/* ------------------------------------------------------------------------- */
/* hist (nullable, max_it + 1 entries): the residual norm before iteration 1
   and after every iteration; *tol_out (nullable): the stopping threshold. */
int gdmo_cg_history(int64_t n, const int64_t *rowptr, const int64_t *cols, const double *vals,
                    const double *b, double *x, int precond, int max_it, double abs_tol, double rel_tol,
                    double *hist, double *tol_out)
{
  double *r = (double *)malloc(sizeof(double) * n);
  double *pv = (double *)malloc(sizeof(double) * n);
  double *v = (double *)malloc(sizeof(double) * n);
  double *dinv = (double *)malloc(sizeof(double) * n);
  for (int64_t i = 0; i < n; ++i) {
    dinv[i] = 1.0;
    if (precond == 1)
      for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
        if (cols[k] == i)
          dinv[i] = 1.0 / vals[k];
  }
  gdmo_csr_vmult(n, rowptr, cols, vals, x, r);
  double res = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    r[i] = b[i] - r[i];
    res += r[i] * r[i];
  }
  res = sqrt(res);
  const double tol = fmax(abs_tol, rel_tol * res);
  if (hist)
    hist[0] = res;
  if (tol_out)
    *tol_out = tol;
  int it = 0, ret = -1;
  if (res <= tol) {
    ret = 0;
    goto done;
  }
  double gh_old = 0.0;
  for (it = 1; it <= max_it; ++it) {
    double gh = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      v[i] = dinv[i] * r[i];
      gh += r[i] * v[i];
    }
    if (it == 1)
      for (int64_t i = 0; i < n; ++i)
        pv[i] = v[i];
    else {
      const double beta = gh / gh_old;
      for (int64_t i = 0; i < n; ++i)
        pv[i] = v[i] + beta * pv[i];
    }
    gh_old = gh;
    gdmo_csr_vmult(n, rowptr, cols, vals, pv, v);
    double pap = 0.0;
    for (int64_t i = 0; i < n; ++i)
      pap += pv[i] * v[i];
    const double alpha = gh / pap;
    res = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      x[i] += alpha * pv[i];
      r[i] -= alpha * v[i];
      res += r[i] * r[i];
    }
    res = sqrt(res);
    if (hist)
      hist[it] = res;
    if (res <= tol) {
      ret = it;
      break;
    }
  }
done:
  free(r);
  free(pv);
  free(v);
  free(dinv);
  return ret;
}

int gdmo_cg(int64_t n, const int64_t *rowptr, const int64_t *cols, const double *vals,
            const double *b, double *x, int precond, int max_it, double abs_tol, double rel_tol)
{
  return gdmo_cg_history(n, rowptr, cols, vals, b, x, precond, max_it, abs_tol, rel_tol, NULL, NULL);
}

/* ------------------------------------------------------------------------- */
/* Error norms against cell-quadrature-point values of the exact solution      */
/* (vector_tools.h:25-86 integrate_difference(L2) per cell + compute_global_   */
/* error; the volume part of advection/problem.h:269-425 postprocess: Linf,    */
/* L1, L2 over QGauss(p+1)); exact given at cell quadrature points, cell-major */
/* (n_cells x (p+1)^dim, q lexicographic, x fastest).  out = {Linf, L1, L2};   */
/* cell_l2 (optional) = the per-cell L2 errors of integrate_difference.        */
/* ------------------------------------------------------------------------- */
void gdmo_error_norms(int dim, int p, const unsigned *nsub, const double *lo, const double *hi, const double *u,
                      const double *exact_q, double *out, double *cell_l2)
{
  tables_t T;
  build_tables(&T, dim, p);
  const int nd = T.nd, n1 = p + 1;
  const unsigned nc = n_cells_total(dim, nsub);
  uint64_t *dofs = (uint64_t *)malloc(sizeof(uint64_t) * nd);
  double *sv = (double *)malloc(sizeof(double) * nd * nd);
  unsigned prev_cat[3] = {~0u, ~0u, ~0u};
  double l2 = 0.0, l1 = 0.0, linf = 0.0;
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3], cat[3];
    double h[3];
    cell_setup(dim, p, nsub, c, lo, hi, cidx, cat, h);
    if (cat[0] != prev_cat[0] || cat[1] != prev_cat[1] || cat[2] != prev_cat[2]) {
      for (int i = 0; i < nd; ++i)
        for (int q = 0; q < nd; ++q)
          shape_at(&T, cat, i, q, h, &sv[i * nd + q], NULL);
      memcpy(prev_cat, cat, sizeof(cat));
    }
    double jxw_vol = 1.0;
    for (int d = 0; d < dim; ++d)
      jxw_vol *= h[d];
    gdmo_cell_dof_indices(dim, p, nsub, c, dofs);
    double diff = 0.0;
    for (int q = 0; q < nd; ++q) {
      int rq = q;
      double wq = jxw_vol;
      for (int d = 0; d < dim; ++d) {
        wq *= T.wq[rq % n1];
        rq /= n1;
      }
      double uq = 0.0;
      for (int j = 0; j < nd; ++j)
        uq += u[dofs[j]] * sv[j * nd + q];
      const double e = uq - exact_q[(uint64_t)c * nd + q];
      diff += e * e * wq;
      l1 += fabs(e) * wq;
      if (fabs(e) > linf)
        linf = fabs(e);
    }
    if (cell_l2)
      cell_l2[c] = sqrt(diff);
    l2 += diff; /* sqrt per cell then squared sum == same */
  }
  free(dofs);
  free(sv);
  out[0] = linf;
  out[1] = l1;
  out[2] = sqrt(l2);
}

double gdmo_l2_error(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                     const double *u, const double *exact_q)
{
  double out[3];
  gdmo_error_norms(dim, p, nsub, lo, hi, u, exact_q, out, NULL);
  return out[2];
}

/* physical coordinates of all cell quadrature points, cell-major */
void gdmo_cell_qpoints(int dim, int p, const unsigned *nsub, const double *lo, const double *hi,
                       double *xyz)
{
  double xq[MAXN], wq[MAXN];
  gdmo_gauss(p + 1, xq, wq);
  const int n1 = p + 1;
  int nd = 1;
  for (int d = 0; d < dim; ++d)
    nd *= n1;
  const unsigned nc = n_cells_total(dim, nsub);
  for (unsigned c = 0; c < nc; ++c) {
    unsigned cidx[3];
    cell_coords(dim, nsub, c, cidx);
    for (int q = 0; q < nd; ++q) {
      int rq = q;
      for (int e = 0; e < 3; ++e) {
        double v = 0.0;
        if (e < dim) {
          const double h = (hi[e] - lo[e]) / nsub[e];
          v = lo[e] + (cidx[e] + xq[rq % n1]) * h;
          rq /= n1;
        }
        xyz[3 * ((uint64_t)c * nd + q) + e] = v;
      }
    }
  }
}
