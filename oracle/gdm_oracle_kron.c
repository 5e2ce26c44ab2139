/*
 * gdm_oracle_kron.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Second CPU restatement of the same operators in Kronecker / stencil form,
 * used (a) to cross-check the reference-faithful cell loops in gdm_oracle.c
 * on the same inputs (agreement ~1e-13) and (b) as the checker at sizes where
 * the O((p+1)^(2 dim)) cell loop is too slow.
 *
 * On an uncut uniform Cartesian mesh the GDM global basis is the tensor
 * product of the 1D global bases (categories and DoF boxes are per direction,
 * include/gdm/system.h:195-246 and :404-424), so
 *   mass      M   = M_z (x) M_y (x) M_x
 *   advection K   = sum_d (B_d (x) M (x) M),  B_d = a_d C_d - outflow trace
 *             (applications/advection/include/gdm/advection/stiffness.h:411-417
 *              with alpha = 0 and the (III) face term :473-532 for a.n >= 0)
 *   wave      K   = -sum_d (L_d (x) M (x) M)
 *             (applications/wave/include/gdm/wave/stiffness.h:171-203)
 * with the 1D matrices assembled cell by cell exactly as the reference's
 * FEValues loop does in 1D.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

double gdmo_basis_derivative(int p, int cat, int i, double x, int order);
void gdmo_gauss(int n, double *x, double *w);
unsigned gdmo_category(unsigned c, unsigned p, unsigned n);
unsigned gdmo_offset(unsigned c, unsigned p, unsigned n);

/* 1D matrices in band storage: row i, column j = i - p + k, k = 0..2p.
 * M_ij = int phi_i phi_j, C_ij = int phi_i' phi_j, L_ij = int phi_i' phi_j'. */
void gdmo_matrices_1d(int p, unsigned nsub, double h, double *M, double *C, double *L)
{
  const int W = 2 * p + 1, n1 = p + 1;
  const unsigned N = nsub + 1;
  memset(M, 0, sizeof(double) * N * W);
  memset(C, 0, sizeof(double) * N * W);
  memset(L, 0, sizeof(double) * N * W);
  double xq[16], wq[16], v[16][16], g[16][16];
  gdmo_gauss(n1, xq, wq);
  for (unsigned c = 0; c < nsub; ++c) {
    const unsigned cat = gdmo_category(c, (unsigned)p, nsub);
    const unsigned off = gdmo_offset(c, (unsigned)p, nsub);
    for (int i = 0; i < n1; ++i)
      for (int q = 0; q < n1; ++q) {
        v[i][q] = gdmo_basis_derivative(p, (int)cat, i, xq[q], 0);
        g[i][q] = gdmo_basis_derivative(p, (int)cat, i, xq[q], 1) / h;
      }
    for (int i = 0; i < n1; ++i)
      for (int j = 0; j < n1; ++j) {
        double m = 0, cc = 0, l = 0;
        for (int q = 0; q < n1; ++q) {
          const double w = wq[q] * h;
          m += v[i][q] * v[j][q] * w;
          cc += g[i][q] * v[j][q] * w;
          l += g[i][q] * g[j][q] * w;
        }
        const unsigned gi = off + i, gj = off + j;
        const int k = (int)gj - (int)gi + p;
        M[gi * W + k] += m;
        C[gi * W + k] += cc;
        L[gi * W + k] += l;
      }
  }
}

/* y = sum over the listed terms of (op_z (x) op_y (x) op_x) u, with per
 * direction band matrices.  terms: n_terms x dim indices into ops[d][...]. */
static void apply_1d(int dim_sel, const unsigned *N, int p, const double *B, const double *in,
                     double *out)
{
  const int W = 2 * p + 1;
  const int64_t Nx = N[0], Ny = N[1], Nz = N[2];
  const int64_t total = Nx * Ny * Nz;
#pragma omp parallel for schedule(static)
  for (int64_t idx = 0; idx < total; ++idx) {
    const int64_t x = idx % Nx, y = (idx / Nx) % Ny, z = idx / (Nx * Ny);
    int64_t pos = (dim_sel == 0) ? x : ((dim_sel == 1) ? y : z);
    const int64_t len = (dim_sel == 0) ? Nx : ((dim_sel == 1) ? Ny : Nz);
    const int64_t stride = (dim_sel == 0) ? 1 : ((dim_sel == 1) ? Nx : Nx * Ny);
    double s = 0.0;
    for (int k = 0; k < W; ++k) {
      const int64_t j = pos - p + k;
      if (j < 0 || j >= len)
        continue;
      s += B[pos * W + k] * in[idx + (j - pos) * stride];
    }
    out[idx] = s;
  }
}

/* General Kronecker apply: result = sum_{t} (A[t][2] (x) A[t][1] (x) A[t][0]) u
 * where each A is a band matrix pointer for that direction (NULL = identity).
 * N[] = vertices per direction (1 for unused directions). */
void gdmo_kron_apply(const unsigned *N, int p, int n_terms, const double *const *ops, const double *u,
                     double *y)
{
  const int64_t total = (int64_t)N[0] * N[1] * N[2];
  double *t1 = (double *)malloc(sizeof(double) * total);
  double *t2 = (double *)malloc(sizeof(double) * total);
  memset(y, 0, sizeof(double) * total);
  for (int t = 0; t < n_terms; ++t) {
    const double *cur = u;
    double *bufs[2] = {t1, t2};
    int b = 0;
    for (int d = 0; d < 3; ++d) {
      const double *A = ops[3 * t + d];
      if (!A)
        continue;
      apply_1d(d, N, p, A, cur, bufs[b]);
      cur = bufs[b];
      b ^= 1;
    }
    for (int64_t i = 0; i < total; ++i)
      y[i] += cur[i];
  }
  free(t1);
  free(t2);
}

/* Dense banded Cholesky-free exact inverse of the Kronecker mass via per-line
 * dense LU (small sizes only): x = (M_z^-1 (x) M_y^-1 (x) M_x^-1) r. */
static void solve_lines(int dsel, const unsigned *N, int p, const double *Mb, double *v)
{
  const int W = 2 * p + 1;
  const int64_t len = N[dsel];
  const int64_t stride = (dsel == 0) ? 1 : ((dsel == 1) ? N[0] : (int64_t)N[0] * N[1]);
  const int64_t total = (int64_t)N[0] * N[1] * N[2];
  /* dense LU of the 1D matrix once */
  double *A = (double *)calloc(len * len, sizeof(double));
  int64_t *piv = (int64_t *)malloc(sizeof(int64_t) * len);
  for (int64_t i = 0; i < len; ++i)
    for (int k = 0; k < W; ++k) {
      const int64_t j = i - p + k;
      if (j >= 0 && j < len)
        A[i * len + j] = Mb[i * W + k];
    }
  for (int64_t k = 0; k < len; ++k) {
    int64_t pm = k;
    for (int64_t i = k + 1; i < len; ++i)
      if (fabs(A[i * len + k]) > fabs(A[pm * len + k]))
        pm = i;
    piv[k] = pm;
    if (pm != k)
      for (int64_t j = 0; j < len; ++j) {
        const double t = A[k * len + j];
        A[k * len + j] = A[pm * len + j];
        A[pm * len + j] = t;
      }
    for (int64_t i = k + 1; i < len; ++i) {
      A[i * len + k] /= A[k * len + k];
      for (int64_t j = k + 1; j < len; ++j)
        A[i * len + j] -= A[i * len + k] * A[k * len + j];
    }
  }
  const int64_t nlines = total / len;
#pragma omp parallel
  {
    double *line = (double *)malloc(sizeof(double) * len);
#pragma omp for schedule(static)
    for (int64_t l = 0; l < nlines; ++l) {
      int64_t base;
      if (dsel == 0)
        base = l * len;
      else if (dsel == 1)
        base = (l / N[0]) * N[0] * N[1] + (l % N[0]);
      else
        base = l;
      for (int64_t i = 0; i < len; ++i)
        line[i] = v[base + i * stride];
      for (int64_t k = 0; k < len; ++k) {
        const double t = line[k];
        line[k] = line[piv[k]];
        line[piv[k]] = t;
      }
      for (int64_t i = 0; i < len; ++i)
        for (int64_t j = 0; j < i; ++j)
          line[i] -= A[i * len + j] * line[j];
      for (int64_t i = len - 1; i >= 0; --i) {
        for (int64_t j = i + 1; j < len; ++j)
          line[i] -= A[i * len + j] * line[j];
        line[i] /= A[i * len + i];
      }
      for (int64_t i = 0; i < len; ++i)
        v[base + i * stride] = line[i];
    }
    free(line);
  }
  free(A);
  free(piv);
}

void gdmo_kron_mass_inverse(const unsigned *N, int p, const double *const *Mb, const double *r, double *x)
{
  const int64_t total = (int64_t)N[0] * N[1] * N[2];
  memcpy(x, r, sizeof(double) * total);
  for (int d = 0; d < 3; ++d)
    if (Mb[d] && N[d] > 1)
      solve_lines(d, N, p, Mb[d], x);
}
