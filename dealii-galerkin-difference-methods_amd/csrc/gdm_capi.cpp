// gdm_capi.cpp -- C ABI of libgdm_hip.so (declared in include/gdm_hip.h).
//
// Owns the device-side operator state: 1D band tables in kernel order, the
// banded Cholesky factors of the 1D mass matrices, the inflow-face projection
// tables and the slab layout.  All launches go to the operator's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gdm_hip.h"
#include "gdm_coeffs.h"
#include "gdm_kernels.h"
#include "gdm_post.h"
#include "gdm_rk.h"
#include "gdm_setup.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
T *dev_upload(const std::vector<T> &h) {
  T *d = nullptr;
  const size_t bytes = std::max<size_t>(h.size(), 1) * sizeof(T);
  hip_check(hipMalloc(&d, bytes), "hipMalloc");
  if (!h.empty()) hip_check(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
  return d;
}

// one tangential direction of a boundary face
struct FaceDir {
  int dim_index = -1;     // reference direction, -1 = trivial
  int n_nodes = 1;        // nodes along this direction
  int Q = 1;              // quadrature points along this direction (local cells x (p+1))
  int cell_begin = 0;     // first local cell
  int node_begin = 0, node_end = 1;  // output node range (owned)
  int64_t stride = 0;     // global index stride
  int wmax = 1;
  int qmax = 1;           // largest q-range of FACE_CHUNK consecutive owned nodes
  int *qs = nullptr, *qc = nullptr;
  double *w = nullptr;    // [n_nodes][wmax]
  double *wT = nullptr;   // [wmax][n_nodes]
  double *phi = nullptr;  // [p][p+1][p+1] cell tables (cell form of the face step 1)
  int *crange = nullptr;  // [n_nodes][2] first / last local cell of each node
  int ncell_total = 0;
};

struct Face {
  int d = 0, side = 0;
  double scale = 0.0;     // |a.n| for inflow faces, 0 otherwise
  int64_t offset = 0;     // offset into the device bc array
  int64_t n_points = 0;
  FaceDir t0, t1;
  int64_t base = 0;       // owned index of node (i0 = 0, i1 = t1.node_begin)
  double *T = nullptr;    // step-1 result of this face (faces run concurrently)
};

}  // namespace

// shared with the sparse-matrix entry points (gdm_csr.hip)
int gdm_internal_set_error(int code, const char *msg) { return fail(code, msg); }

// line-solve tables of one banded SPD matrix (build_line_tables)
struct LineTables {
  double *lrow = nullptr, *invd = nullptr;               // v2 row form
  double *l3 = nullptr, *u3 = nullptr, *d3 = nullptr;    // v3 split rows
  std::vector<double> cst;                               // v3 interior fixed-point row
  int row_lo = 0, row_hi = 0;
};

// Distributed exact mass inverse along the partitioned direction (truncated
// SPIKE, gdm_mass_solve_slab / gdm_mass_solve_interface): the slab's own
// diagonal block A_r of M_q, its spikes V = A_r^-1 B_r (coupling to the next
// slab's first p planes) and W = A_r^-1 C_r (previous slab's last p planes),
// and the two p x 2p rows of the interface-system inverses.
struct SpikeTables {
  bool built = false;
  double eps = 0.0;        // largest dropped far-spike entry over all slabs
  int rounds = 0;          // refinement exchanges (-1: partition refused)
  int next_round = -1;     // progress of the current solve: -1 no slab solve
                           // pending, k: rounds [0, k) done
  double *G0 = nullptr;    // device [2p][plane]: saved slab-solve edge planes (rounds > 0)
  int n_planes = 0;        // owned planes of this rank
  int has_lo = 0, has_hi = 0;
  LineTables slab;         // A_r
  double *VW = nullptr;    // device [n_planes][2p]: V row k | W row k
  double *S = nullptr;     // device [2][p][2p]: lower-interface rows (x_{r-1}^bot), upper (x_{r+1}^top)
  int k_begin = 0, k_end = 0;  // planes the correction touches
};

struct gdm_op {
  int device = 0;
  hipStream_t own_stream = nullptr, stream = nullptr;
  bool concurrent = true;  // compute_rhs: face step 1 in the stencil's tail (apply_with_faces)
  gdm_mesh_desc mesh{};
  int kind = 0, p = 1, dim = 1;
  int N[3] = {1, 1, 1};        // vertices per reference direction
  int K[3] = {1, 1, 1};        // kernel-space extents (X, Y, Z)
  int kdir[3] = {-1, -1, -1};  // kernel axis -> reference direction (-1 trivial)
  int part_axis = 2;           // kernel axis of the slab partition (1 = Y, 2 = Z)
  gdm_layout layout{};
  double a[3] = {0, 0, 0};
  double nitsche = 0.0;
  // device tables
  // stencil tables (kernel axes) and the scalars of the compile-time bands
  double *corrX = nullptr, *yT1 = nullptr, *yT3 = nullptr, *zt = nullptr;
  int x_corr_left = 0, x_corr_right = 0, x_toep = 0, y_toep = 0, z_toep = 0;
  double sx = 0, cy[19] = {0};
  // v8 variants: E pre-scaled by h_z (sx, cy, corrX's B part, yT3), z table e = M_z / h_z
  double *corrX8 = nullptr, *yT3_8 = nullptr, *zt8 = nullptr;
  double *yT1d = nullptr, *yT3d = nullptr, *m_yT3d = nullptr;  // v8 y corrections
  double sx8 = 0, cy8[19] = {0}, cxs8[19] = {0};
  double dint = 0, m_dint = 0;  // interior z scales of D (operator, mass)
  double zd8[19] = {0}, m_zd8[19] = {0};  // dint * dhat[2p - k] (operator, mass)
  int xcd_map = 1;
  // the same for the mass operator of an advection/wave op (gdm_mass_apply)
  double *m_corrX = nullptr, *m_zt = nullptr;
  double *lrow[3] = {nullptr, nullptr, nullptr}, *invd[3] = {nullptr, nullptr, nullptr};
  // mass inverse v3 tables (gdm_mass.hip): [rows][p] lower / upper factor rows,
  // inverse diagonal, the interior fixed-point row and its row range
  double *l3[3] = {nullptr, nullptr, nullptr}, *u3[3] = {nullptr, nullptr, nullptr}, *d3[3] = {nullptr, nullptr, nullptr};
  double *cst3[3] = {nullptr, nullptr, nullptr};
  int row_lo3[3] = {0, 0, 0}, row_hi3[3] = {0, 0, 0};
  std::vector<double> cst3_host[3];
  double *bc_tab = nullptr;  // gdm_eval_boundary: per-face 1D factor tables
  SpikeTables spike;         // distributed mass inverse (n_ranks > 1)
  // gdm_error_norms: shape values per category, per-workgroup partials, result
  double *err_S = nullptr, *err_partial = nullptr;
  static constexpr int n_err_partial = 1024;
  int bc_tab_ld = 0;
  double *bc_stage_tab = nullptr;  // gdm_apply_bc_fn: BcStage factor tables (2 x 6 faces)
  double *bc_stage_vals = nullptr;  // gdm_apply_bc_fn: the stage boundary values (n_bc_points)
  int bc_stage_ld = 0;
  // periodicity constraints (system.h:427-463): scratch copy of the input for
  // distribute; CG work vectors and the Jacobi inverse diagonal
  double *pscratch = nullptr;
  double *cg_r = nullptr, *cg_p = nullptr, *cg_Ap = nullptr, *cg_z = nullptr, *cg_invdiag = nullptr;
  std::vector<Face> faces;
  double *face_tmp = nullptr;
  // the stencil's tail work (face step 1, gdmk_launch_stencil8): device claim
  // counter, 0 between launches (each launch resets it with its last claim)
  unsigned long long *tail_counter = nullptr;
  double *mass_tmp = nullptr;  // ping-pong vector of the segmented mass passes (small meshes)
  int64_t mass_tmp_size = 0;
  int64_t face_tmp_size = 0;
  double *dot_partial = nullptr, *dot_out = nullptr;
  int n_dot_partial = 1024;
  int zchunk = 64;
  // host copies for bc ordering
  std::vector<double> xq;
  gdm::Slab slab{};
  std::vector<void *> allocations;
};

namespace {

void free_op(gdm_op *op) {
  if (!op) return;
  for (void *ptr : op->allocations) (void)hipFree(ptr);
  if (op->own_stream) (void)hipStreamDestroy(op->own_stream);
  delete op;
}

// diag of the condensed mass P^T M P = kron_d diag(P_d^T M_d P_d) on the owned
// DoFs (global lexicographic order from the owned plane range); constrained
// rows of periodic directions 1
std::vector<double> mass_diagonal_owned(const gdm_op *op) {
  std::vector<double> dg[3];
  for (int d = 0; d < 3; ++d) {
    if (d >= op->dim) {
      dg[d].assign(1, 1.0);
      continue;
    }
    const unsigned nc = (unsigned)op->mesh.n_subdivisions[d];
    const double h = (op->mesh.hi[d] - op->mesh.lo[d]) / nc;
    const gdm::Band M = gdm::assemble_1d(op->p, nc, h).M;
    dg[d].resize(M.n);
    for (int i = 0; i < M.n; ++i) dg[d][i] = M(i, i);
    if (op->mesh.periodic & (1 << d)) {
      dg[d][0] += M(M.n - 1, M.n - 1) + M(0, M.n - 1) + M(M.n - 1, 0);
      dg[d][M.n - 1] = 1.0;
    }
  }
  const int64_t n = op->layout.n_owned;
  const int64_t g0 = (int64_t)op->layout.owned_plane_begin * op->layout.plane_size;
  std::vector<double> out((size_t)n);
  const int64_t N0 = op->N[0], N1 = op->N[1];
  for (int64_t l = 0; l < n; ++l) {
    const int64_t g = g0 + l;
    const int64_t i0 = g % N0, i1 = (g / N0) % N1, i2 = g / (N0 * N1);
    bool constrained = false;
    const int64_t id[3] = {i0, i1, i2};
    for (int d = 0; d < op->dim; ++d)
      if ((op->mesh.periodic & (1 << d)) && id[d] == op->N[d] - 1) constrained = true;
    out[l] = constrained ? 1.0 : dg[0][i0] * dg[1][op->dim > 1 ? i1 : 0] * dg[2][op->dim > 2 ? i2 : 0];
  }
  return out;
}

template <typename T>
T *keep(gdm_op *op, T *ptr) {
  op->allocations.push_back((void *)ptr);
  return ptr;
}

// Build the row (x) or column (y, z) band table of a kernel axis in kernel
// order.  For column tables entry [s][k] holds A(s - p + k, s).
std::vector<double> band_cols(const gdm::Band &A, int pad, int pad_back) {
  // rows [0, pad) and [pad + n, pad + n + pad_back) are zero: the kernel reads
  // them for halo rows outside the domain and for rows of a partial last tile
  const int n = A.n, hb = A.hb, W = 2 * hb + 1;
  std::vector<double> t((size_t)(n + pad + pad_back) * W, 0.0);
  for (int s = 0; s < n; ++s)
    for (int k = 0; k < W; ++k) t[(size_t)(s + pad) * W + k] = A(s - hb + k, s);
  return t;
}

// interior (Toeplitz) band of the unit-h 1D matrices: which 0 = M, 1 = C, 2 = L
// -- exactly the compile-time constants the kernels use (gdm_coeffs.h)
template <int P>
std::vector<double> interior_band_t(int which) {
  using IR = gdmk::InteriorRows<P>;
  const double *src = which == 0 ? IR::m : (which == 1 ? IR::c : IR::l);
  return std::vector<double>(src, src + 2 * P + 1);
}

std::vector<double> interior_band(int p, int which) {
  switch (p) {
    case 1: return interior_band_t<1>(which);
    case 3: return interior_band_t<3>(which);
    case 5: return interior_band_t<5>(which);
    case 7: return interior_band_t<7>(which);
    default: return interior_band_t<9>(which);
  }
}

gdm::Band identity_band(int p) {
  gdm::Band b(1, p);
  b(0, 0) = 1.0;
  return b;
}

// Line-solve tables of one SPD band matrix M = L L^T (gdm_mass.hip): the v2
// row form (lrow / invd, zero-padded for the backward sweep) and, where the v3
// single-sweep kernel exists for p, its split rows prescaled by 1 / L_ii,
// zero-padded by 3C + p rows, plus the run of rows around the middle that equal
// the middle row bitwise (the interior fixed point of the factorisation).
LineTables build_line_tables(gdm_op *op, const gdm::Band &M) {
  const int p = op->p;
  LineTables t;
  std::vector<double> lrow, invd;
  gdm::cholesky_band(M, lrow, invd);
  std::vector<double> lrow_pad = lrow;
  lrow_pad.resize(lrow.size() + (size_t)p * (p + 1), 0.0);  // zero pad for the backward sweep
  t.lrow = keep(op, dev_upload(lrow_pad));
  t.invd = keep(op, dev_upload(invd));
  const int C3 = gdmk_mass3_chunk(p);
  if (C3 > 0) {
    const int n = M.n, rows = n + 3 * C3 + p;
    const int wl = p + 1;
    std::vector<double> l3((size_t)rows * p, 0.0), u3((size_t)rows * p, 0.0), d3((size_t)rows, 0.0);
    for (int i = 0; i < n; ++i) {
      for (int k = 0; k < p; ++k) l3[(size_t)i * p + k] = lrow[(size_t)i * wl + k] * invd[i];
      for (int m = 1; m <= p; ++m)
        if (i + m < n) u3[(size_t)i * p + m - 1] = lrow[(size_t)(i + m) * wl + (p - m)] * invd[i];
      d3[i] = invd[i];
    }
    const int mid = n / 2;
    auto same = [&](int i) {
      if (d3[i] != d3[mid]) return false;
      for (int k = 0; k < p; ++k)
        if (l3[(size_t)i * p + k] != l3[(size_t)mid * p + k] || u3[(size_t)i * p + k] != u3[(size_t)mid * p + k])
          return false;
      return true;
    };
    int lo = mid, hi = mid + 1;
    while (lo > 0 && same(lo - 1)) --lo;
    while (hi < n && same(hi)) ++hi;
    std::vector<double> cst(2 * p + 1);
    for (int k = 0; k < p; ++k) {
      cst[k] = l3[(size_t)mid * p + k];
      cst[p + k] = u3[(size_t)mid * p + k];
    }
    cst[2 * p] = d3[mid];
    t.l3 = keep(op, dev_upload(l3));
    t.u3 = keep(op, dev_upload(u3));
    t.d3 = keep(op, dev_upload(d3));
    t.cst = cst;
    t.row_lo = lo;
    t.row_hi = hi;
  }
  return t;
}

void build_tables(gdm_op *op) {
  const int p = op->p;
  gdm::Band M[3], B[3];
  for (int ax = 0; ax < 3; ++ax) {
    const int d = op->kdir[ax];
    if (d < 0) {
      M[ax] = identity_band(p);
      B[ax] = gdm::Band(1, p);
      continue;
    }
    const unsigned ncell = (unsigned)op->mesh.n_subdivisions[d];
    const double h = (op->mesh.hi[d] - op->mesh.lo[d]) / ncell;
    gdm::Matrices1D m = gdm::assemble_1d(p, ncell, h);
    M[ax] = m.M;
    const int n = m.M.n, last = n - 1;
    gdm::Band b(n, p);
    switch (op->kind) {
      case GDM_OP_ADVECTION: {
        // (a u, grad v): a_d C_d; outflow faces (a.n >= 0) add -(a.n) u v
        // (stiffness.h:411-417, :520-529)
        const double ad = op->a[d];
        for (int i = 0; i < n; ++i)
          for (int j = std::max(0, i - p); j <= std::min(last, i + p); ++j) b(i, j) = ad * m.C(i, j);
        if (ad >= 0.0) b(last, last) -= ad;    // right face, a.n = a_d
        if (-ad >= 0.0) b(0, 0) += ad;         // left face, a.n = -a_d
        break;
      }
      case GDM_OP_CONVECTIVE: {
        // -(a . grad u, v): -a_d C^T (advection_01_gdm.cc:199-203)
        const double ad = op->a[d];
        for (int i = 0; i < n; ++i)
          for (int j = std::max(0, i - p); j <= std::min(last, i + p); ++j) b(i, j) = -ad * m.C(j, i);
        break;
      }
      case GDM_OP_WAVE: {
        // -(grad v, grad u) (wave/stiffness.h:171-181) + box Nitsche
        // (:296-310): -[-dv/dn u - v du/dn + gamma/h v u] on each box face
        for (int i = 0; i < n; ++i)
          for (int j = std::max(0, i - p); j <= std::min(last, i + p); ++j) b(i, j) = -m.L(i, j);
        if (op->nitsche > 0.0) {
          double hmin = 1e300;
          for (int e = 0; e < op->dim; ++e)
            hmin = std::min(hmin, (op->mesh.hi[e] - op->mesh.lo[e]) / op->mesh.n_subdivisions[e]);
          // traces of the boundary cells
          const unsigned cl = 0, cr = ncell - 1;
          const int catl = (int)gdm::category(cl, p, ncell), catr = (int)gdm::category(cr, p, ncell);
          const int offl = (int)gdm::box_offset(cl, p, ncell), offr = (int)gdm::box_offset(cr, p, ncell);
          for (int side = 0; side < 2; ++side) {
            const int cat = side ? catr : catl, off = side ? offr : offl;
            const double x = side ? 1.0 : 0.0, nrm = side ? 1.0 : -1.0;
            for (int ii = 0; ii <= p; ++ii)
              for (int jj = 0; jj <= p; ++jj) {
                const double vi = gdm::shape_1d(p, cat, ii, x, 0), vj = gdm::shape_1d(p, cat, jj, x, 0);
                const double di = gdm::shape_1d(p, cat, ii, x, 1) / h * nrm;
                const double dj = gdm::shape_1d(p, cat, jj, x, 1) / h * nrm;
                b(off + ii, off + jj) -= (-di * vj - vi * dj + op->nitsche / hmin * vi * vj);
              }
          }
        }
        break;
      }
      default:
        break;  // mass: B unused
    }
    B[ax] = b;
  }
  // Kernel tables.  Interior rows use the compile-time bands (gdm_coeffs.h):
  // M = h mhat, B = beta bhat with bhat = chat (advection, convective) or
  // lhat (wave) and beta = a_d resp. -1/h_d; see StencilArgs for the scalings.
  const int W = 2 * p + 1;
  double h[3], beta[3];
  for (int ax = 0; ax < 3; ++ax) {
    const int d = op->kdir[ax];
    h[ax] = d < 0 ? 1.0 : (op->mesh.hi[d] - op->mesh.lo[d]) / op->mesh.n_subdivisions[d];
    beta[ax] = 0.0;
    if (d >= 0 && (op->kind == GDM_OP_ADVECTION || op->kind == GDM_OP_CONVECTIVE)) beta[ax] = op->a[d];
    if (d >= 0 && op->kind == GDM_OP_WAVE) beta[ax] = -1.0 / h[ax];
  }
  auto toep = [&](int ax) { return op->K[ax] >= 2 * p + 3 ? 1 : 0; };
  op->x_toep = toep(0);
  op->y_toep = toep(1);
  op->z_toep = toep(2);
  const std::vector<double> mhat = interior_band(p, 0), bhat = interior_band(p, op->kind == GDM_OP_WAVE ? 2 : 1);
  // x wall-column corrections (rows x <= p and x >= n - p use one-sided categories)
  auto corr_table = [&](const gdm::Band &Mx, const gdm::Band &Bx, int &left, int &right, double bscale = 1.0) {
    const int n = Mx.n;
    left = std::min(p + 1, n);
    const int right_begin = std::max(p + 1, n - p - 1);
    right = std::max(0, n - right_begin);
    std::vector<double> corr((size_t)2 * (p + 1) * 2 * W, 0.0);
    auto fill = [&](int slot, int x) {
      for (int k = 0; k < W; ++k) {
        const double tm = op->x_toep ? h[0] * mhat[k] : 0.0, tb = op->x_toep ? beta[0] * bhat[k] : 0.0;
        corr[(size_t)slot * 2 * W + k] = (Mx(x, x - p + k) - tm) / h[0];
        corr[(size_t)slot * 2 * W + W + k] = bscale * h[1] * (Bx(x, x - p + k) - tb);
      }
    };
    for (int x = 0; x < left; ++x) fill(x, x);
    for (int j = 0; j < right; ++j) fill(p + 1 + j, right_begin + j);
    return corr;
  };
  auto scaled = [](const gdm::Band &A, double f) {
    gdm::Band b = A;
    for (double &v : b.a) v *= f;
    return b;
  };
  // z column table: rows 0..2p = planes 0..2p, rows 2p+1..4p+1 = planes
  // Nz-2p-1..Nz-1, row 4p+2 = the interior column; (e, d) pairs per entry
  auto z_table = [&](const gdm::Band *Ez, const gdm::Band &Dz, double e_int, double d_int, const std::vector<double> &dhat) {
    const int Nz = Dz.n;
    std::vector<double> t((size_t)(2 * W + 1) * W * 2, 0.0);
    auto col = [&](int row, int zz) {
      if (zz < 0 || zz >= Nz) return;
      for (int k = 0; k < W; ++k) {
        const int zr = zz - p + k;
        t[((size_t)row * W + k) * 2 + 0] = Ez ? (*Ez)(zr, zz) : 0.0;
        t[((size_t)row * W + k) * 2 + 1] = Dz(zr, zz);
      }
    };
    for (int r = 0; r < W; ++r) col(r, r);
    for (int r = 0; r < W; ++r) col(W + r, Nz - W + r);
    for (int k = 0; k < W; ++k) {
      t[((size_t)2 * W * W + k) * 2 + 0] = Ez ? e_int * mhat[2 * p - k] : 0.0;
      t[((size_t)2 * W * W + k) * 2 + 1] = d_int * dhat[2 * p - k];
    }
    return t;
  };
  const int ypad = p + 64;  // >= p + max tile rows
  const bool mass = op->kind == GDM_OP_MASS;
  const gdm::Band Bz = scaled(B[2], h[0] * h[1]), Mz = scaled(M[2], h[0] * h[1]);
  op->corrX = keep(op, dev_upload(corr_table(M[0], B[0], op->x_corr_left, op->x_corr_right)));
  op->yT1 = keep(op, dev_upload(band_cols(scaled(M[1], 1.0 / h[1]), p, ypad)));
  op->yT3 = keep(op, dev_upload(band_cols(scaled(B[1], h[0]), p, ypad)));
  op->m_zt = keep(op, dev_upload(z_table(nullptr, Mz, 0.0, h[0] * h[1] * h[2], mhat)));
  op->zt = mass ? op->m_zt : keep(op, dev_upload(z_table(&M[2], Bz, h[2], beta[2] * h[0] * h[1], bhat)));
  op->sx = h[1] * beta[0];
  for (int k = 0; k < W; ++k) op->cy[k] = h[0] * beta[1] * bhat[k];
  op->m_dint = h[0] * h[1] * h[2];
  for (int k = 0; k < W; ++k) op->m_zd8[k] = op->m_dint * mhat[2 * p - k];
  // v8 y tables: (wall row - Toeplitz row) corrections, column form; zero away
  // from the walls (the kernel adds them only for waves with wall rows)
  {
    auto delta = [&](const gdm::Band &A, const std::vector<double> &toep) {
      gdm::Band d = A;
      for (int i = 0; i < A.n; ++i)
        for (int j = std::max(0, i - p); j <= std::min(A.n - 1, i + p); ++j) d(i, j) = A(i, j) - toep[j - i + p];
      return d;
    };
    std::vector<double> tm(W), tc(W, 0.0);
    for (int k = 0; k < W; ++k) tm[k] = mhat[k];
    if (!mass)
      for (int k = 0; k < W; ++k) tc[k] = h[0] * beta[1] * bhat[k] * h[2];
    op->yT1d = keep(op, dev_upload(band_cols(delta(scaled(M[1], 1.0 / h[1]), tm), p, ypad)));
    op->yT3d = keep(op, dev_upload(band_cols(delta(scaled(B[1], h[0] * h[2]), tc), p, ypad)));
    op->m_yT3d = keep(op, dev_upload(band_cols(gdm::Band(M[1].n, p), p, ypad)));
  }
  if (!mass) {
    int l8 = 0, r8 = 0;
    op->corrX8 = keep(op, dev_upload(corr_table(M[0], B[0], l8, r8, h[2])));
    op->yT3_8 = keep(op, dev_upload(band_cols(scaled(B[1], h[0] * h[2]), p, ypad)));
    const gdm::Band Mz8 = scaled(M[2], 1.0 / h[2]);
    op->zt8 = keep(op, dev_upload(z_table(&Mz8, Bz, 1.0, beta[2] * h[0] * h[1], bhat)));
    op->sx8 = op->sx * h[2];
    for (int k = 0; k < W; ++k) op->cxs8[k] = op->sx8 * bhat[k];
    op->dint = beta[2] * h[0] * h[1];
    for (int k = 0; k < W; ++k) op->zd8[k] = op->dint * bhat[2 * p - k];
    for (int k = 0; k < W; ++k) op->cy8[k] = op->cy[k] * h[2];
  }
  // mass operator tables for gdm_mass_apply on a non-mass op
  {
    gdm::Band zero0(M[0].n, p);
    int l = 0, r = 0;
    op->m_corrX = keep(op, dev_upload(corr_table(M[0], zero0, l, r)));
  }
  // banded Cholesky factors of the 1D mass matrices (exact Kronecker inverse)
  for (int ax = 0; ax < 3; ++ax) {
    if (op->K[ax] <= 1) continue;
    LineTables t = build_line_tables(op, M[ax]);
    op->lrow[ax] = t.lrow;
    op->invd[ax] = t.invd;
    op->l3[ax] = t.l3;
    op->u3[ax] = t.u3;
    op->d3[ax] = t.d3;
    op->cst3_host[ax] = t.cst;
    op->row_lo3[ax] = t.row_lo;
    op->row_hi3[ax] = t.row_hi;
  }
}

void build_layout(gdm_op *op) {
  const int q = op->dim - 1;  // partition direction (reference)
  const unsigned ncq = (unsigned)op->mesh.n_subdivisions[q];
  op->slab = gdm::slab_partition(ncq, (unsigned)op->mesh.n_ranks, (unsigned)op->mesh.rank);
  gdm_layout &L = op->layout;
  L.n_dofs_global = (int64_t)op->N[0] * op->N[1] * op->N[2];
  L.plane_size = L.n_dofs_global / op->N[q];
  L.n_planes_global = op->N[q];
  L.owned_plane_begin = (int32_t)op->slab.plane_begin;
  L.owned_plane_end = (int32_t)std::max(op->slab.plane_begin, op->slab.plane_end);
  L.cell_plane_begin = (int32_t)op->slab.cell_begin;
  L.cell_plane_end = (int32_t)std::max(op->slab.cell_begin, op->slab.cell_end);
  L.halo_depth = op->p;
  const int nown = L.owned_plane_end - L.owned_plane_begin;
  if (nown > 0) {
    L.ghost_planes_below = std::min(op->p, L.owned_plane_begin);
    L.ghost_planes_above = std::min(op->p, op->N[q] - L.owned_plane_end);
  } else {
    L.ghost_planes_below = L.ghost_planes_above = 0;
  }
  L.n_owned = (int64_t)nown * L.plane_size;
  L.n_local = (int64_t)(nown + L.ghost_planes_below + L.ghost_planes_above) * L.plane_size;
}

void build_faces(gdm_op *op) {
  const int p = op->p, n1 = p + 1, dim = op->dim, q = dim - 1;
  const gdm_layout &L = op->layout;
  int64_t stride[3] = {1, op->N[0], (int64_t)op->N[0] * op->N[1]};
  const int64_t own_off = (int64_t)L.owned_plane_begin * L.plane_size;
  int64_t offset = 0;
  int64_t max_tmp = 1;
  const bool have_cells = L.cell_plane_end > L.cell_plane_begin;
  for (int f = 0; f < 2 * dim && have_cells; ++f) {
    const int d = f / 2, side = f % 2;
    const unsigned ncd = (unsigned)op->mesh.n_subdivisions[d];
    // does this rank own cells adjacent to the face?
    if (d == q) {
      if (side == 0 && L.cell_plane_begin != 0) continue;
      if (side == 1 && L.cell_plane_end != (int)ncd) continue;
    }
    Face F;
    F.d = d;
    F.side = side;
    const double an = side ? op->a[d] : -op->a[d];
    F.scale = (op->kind == GDM_OP_ADVECTION && an < 0.0) ? -an : 0.0;
    int tang[2] = {-1, -1}, nt = 0;
    for (int e = 0; e < dim; ++e)
      if (e != d) tang[nt++] = e;
    FaceDir *T[2] = {&F.t0, &F.t1};
    for (int k = 0; k < 2; ++k) {
      FaceDir &t = *T[k];
      const int e = tang[k];
      t.dim_index = e;
      if (e < 0) {
        std::vector<int32_t> qs{0}, qc{1};
        std::vector<double> w{1.0};
        t.n_nodes = 1;
        t.Q = 1;
        t.node_begin = 0;
        t.node_end = 1;
        t.stride = 0;
        t.wmax = 1;
        t.qmax = 1;
        t.qs = keep(op, dev_upload(qs));
        t.qc = keep(op, dev_upload(qc));
        t.w = keep(op, dev_upload(w));
        t.wT = t.w;
        continue;
      }
      const unsigned nce = (unsigned)op->mesh.n_subdivisions[e];
      const double h = (op->mesh.hi[e] - op->mesh.lo[e]) / nce;
      unsigned cb = 0, ce = nce;
      int nb = 0, ne = op->N[e];
      if (e == q) {
        // owner-computes: every cell whose DoF box reaches an owned node, the
        // neighbour ranks' cells included (their points are ghost points)
        nb = L.owned_plane_begin;
        ne = L.owned_plane_end;
        cb = nce;
        ce = 0;
        for (unsigned c = 0; c < nce; ++c) {
          const int off = (int)gdm::box_offset(c, p, nce);
          if (off + p >= nb && off <= ne - 1) {
            cb = std::min(cb, c);
            ce = std::max(ce, c + 1);
          }
        }
        if (ce <= cb) cb = ce = (unsigned)L.cell_plane_begin;
      }
      gdm::FaceTable ft = gdm::face_table_1d(p, nce, h, cb, ce);
      t.n_nodes = op->N[e];
      t.Q = int(ce - cb) * n1;
      t.cell_begin = (int)cb;
      t.node_begin = nb;
      t.node_end = ne;
      t.stride = stride[e];
      t.wmax = ft.wmax;
      {
        std::vector<double> wT((size_t)ft.wmax * ft.n_nodes);
        for (int i = 0; i < ft.n_nodes; ++i)
          for (int m = 0; m < ft.wmax; ++m) wT[(size_t)m * ft.n_nodes + i] = ft.w[(size_t)i * ft.wmax + m];
        t.wT = keep(op, dev_upload(wT));
        // LDS row length of the step-1 kernel: q-range of each chunk of owned nodes
        t.qmax = 1;
        for (int ia = nb; ia < ne; ia += gdmk::FACE_CHUNK) {
          const int ib = std::min(ne, ia + gdmk::FACE_CHUNK) - 1;
          t.qmax = std::max(t.qmax, std::min(t.Q, ft.qstart[ib] + ft.wmax) - ft.qstart[ia]);
        }
      }
      t.qs = keep(op, dev_upload(ft.qstart));
      t.qc = keep(op, dev_upload(ft.qcount));
      t.w = keep(op, dev_upload(ft.w));
      {
        // cell form: per-category tables and the cell range of every node
        std::vector<double> xq, wq;
        gdm::gauss_unit(n1, xq, wq);
        std::vector<double> phi((size_t)p * n1 * n1);
        for (int cat = 0; cat < p; ++cat)
          for (int l = 0; l < n1; ++l)
            for (int qq = 0; qq < n1; ++qq)
              phi[((size_t)cat * n1 + l) * n1 + qq] = gdm::shape_1d(p, cat, l, xq[qq], 0) * wq[qq] * h;
        std::vector<int32_t> cr((size_t)2 * ft.n_nodes);
        for (int i = 0; i < ft.n_nodes; ++i) {
          cr[2 * i] = ft.qstart[i] / n1;
          cr[2 * i + 1] = ft.qstart[i] / n1 + ft.qcount[i] / n1 - 1;
        }
        t.phi = keep(op, dev_upload(phi));
        t.crange = keep(op, dev_upload(cr));
        t.ncell_total = (int)nce;
      }
    }
    F.n_points = (int64_t)F.t0.Q * F.t1.Q;
    F.offset = offset;
    offset += F.n_points;
    const int64_t node_d = side ? (op->N[d] - 1) : 0;
    F.base = node_d * stride[d] + (int64_t)F.t0.node_begin * F.t0.stride + (int64_t)F.t1.node_begin * F.t1.stride -
             own_off;
    max_tmp = std::max<int64_t>(max_tmp, (int64_t)F.t1.Q * (F.t0.node_end - F.t0.node_begin));
    if (F.scale != 0.0) {
      const int64_t tsz = std::max<int64_t>(1, (int64_t)F.t1.Q * (F.t0.node_end - F.t0.node_begin));
      hip_check(hipMalloc(&F.T, sizeof(double) * tsz), "hipMalloc");
      keep(op, F.T);
    }
    op->faces.push_back(F);
  }
  op->layout.n_bc_points = offset;
  // the reference's block(0): points of the owned cells only
  {
    int64_t nref = 0;
    const int n1q = p + 1;
    const int nfq = dim == 1 ? 1 : (dim == 2 ? n1q : n1q * n1q);
    int ncell[3] = {1, 1, 1};
    for (int d = 0; d < dim; ++d) ncell[d] = op->mesh.n_subdivisions[d];
    for (const Face &F : op->faces) {
      // owned cells adjacent to face F: product of the tangential owned cell counts
      int64_t cells = 1;
      for (int e = 0; e < dim; ++e) {
        if (e == F.d) continue;
        cells *= e == q ? (L.cell_plane_end - L.cell_plane_begin) : ncell[e];
      }
      nref += cells * nfq;
    }
    op->layout.n_bc_points_ref = nref;
  }
  op->face_tmp_size = max_tmp;
  hip_check(hipMalloc(&op->face_tmp, sizeof(double) * max_tmp), "hipMalloc");
  keep(op, op->face_tmp);
}

// Output planes [zb, ze) of the owned range (3D: z planes; the full owned
// range otherwise).  dst is the owned vector; only those planes are written.
// tail / n_tail: inflow faces whose step 1 the stencil's workgroups run once
// their chunk is done (v8 only); *tail_done reports whether it ran
hipError_t launch_stencil(gdm_op *op, bool mass, const double *src, double *dst, int zb = -1, int ze = -1,
                          const gdmk::FaceArgs *tail = nullptr, int n_tail = 0, bool *tail_done = nullptr,
                          int zb2 = 0, int ze2 = 0) {
  if (tail_done) *tail_done = false;
  const gdm_layout &L = op->layout;
  gdmk::StencilArgs a{};
  a.src = src;
  a.dst = dst;
  a.Nx = op->K[0];
  a.Ny = op->K[1];
  a.Nz = op->K[2];
  const int ib = L.owned_plane_begin - L.ghost_planes_below, ie = L.owned_plane_end + L.ghost_planes_above;
  if (op->part_axis == 2) {
    a.in_y0 = 0; a.in_y1 = a.Ny; a.in_z0 = ib; a.in_z1 = ie;
    a.out_y0 = 0; a.out_y1 = a.Ny; a.out_z0 = L.owned_plane_begin; a.out_z1 = L.owned_plane_end;
  } else {
    a.in_z0 = 0; a.in_z1 = 1; a.in_y0 = ib; a.in_y1 = ie;
    a.out_z0 = 0; a.out_z1 = 1; a.out_y0 = L.owned_plane_begin; a.out_y1 = L.owned_plane_end;
  }
  if (zb < 0) zb = a.out_z0;
  if (ze < 0) ze = a.out_z1;
  zb = std::max(zb, a.out_z0);
  ze = std::min(ze, a.out_z1);
  if (ze <= zb) return hipSuccess;
  a.zchunk = std::max(1, std::min(op->zchunk, ze - zb));
  a.x_toep = op->x_toep;
  a.y_toep = op->y_toep;
  a.z_toep = op->z_toep;
  a.x_corr_left = op->x_corr_left;
  a.x_corr_right = op->x_corr_right;
  const bool as_mass = mass || op->kind == GDM_OP_MASS;
  a.yT1 = op->yT1;
  a.yT3 = op->yT3;
  // v8 needs every x and y tile to touch at most one wall; smaller meshes use v7
  int ty8 = 32, wgs8 = 1;
  gdmk_stencil8_geom(op->p, &ty8, &wgs8);
  const bool v8 = op->K[1] >= ty8 + 2 * op->p + 2 && op->K[0] >= 64 + 2 * op->p + 2;
  if (v8) a.yT1 = op->yT1d;
  a.xcd_map = op->xcd_map;
  if (as_mass) {
    a.sx = 0.0;
    a.corrX = op->m_corrX;
    a.zt = op->m_zt;
    a.dint = op->m_dint;
    for (int k = 0; k < 19; ++k) a.zd[k] = op->m_zd8[k];
    if (v8) a.yT3 = op->m_yT3d;
  } else if (v8) {
    a.dint = op->dint;
    for (int k = 0; k < 19; ++k) a.zd[k] = op->zd8[k];
    a.sx = op->sx8;
    for (int k = 0; k < 19; ++k) a.cxs[k] = op->cxs8[k];
    for (int k = 0; k < 19; ++k) a.cy[k] = op->cy8[k];
    a.corrX = op->corrX8;
    a.yT3 = op->yT3d;
    a.zt = op->zt8;
  } else {
    a.sx = op->sx;
    for (int k = 0; k < 19; ++k) a.cy[k] = op->cy[k];
    a.corrX = op->corrX;
    a.zt = op->zt;
  }
  if (L.n_owned == 0) return hipSuccess;
  const int bk = as_mass ? 0 : (op->kind == GDM_OP_WAVE ? 2 : 1);
  if (!v8) {
    // v7 indexes dst relative to out_z0: shift both to the sub-range
    a.dst = dst + (int64_t)(zb - a.out_z0) * L.plane_size;
    a.out_z0 = zb;
    a.out_z1 = ze;
    return gdmk_launch_stencil(op->p, bk, a, op->stream);
  }
  // v8: one launch for all output planes, z-wall planes included (each input
  // plane takes its own z column: wall columns from the LDS table, interior
  // ones from the compile-time bands, with the same bits in every plane range)
  const int ty = ty8, wgs = wgs8;
  const int64_t tiles = (int64_t)((a.Nx + 63) / 64) * ((a.out_y1 - a.out_y0 + ty - 1) / ty);
  // one round of workgroups on 256 CUs (two rounds measured 0.93 vs 0.85 ms
  // at C3, 0.27 vs 0.22 ms at C4: profiles/r3g/variants.txt)
  const int64_t chunks = std::max<int64_t>(1, (256 * wgs + tiles - 1) / tiles);
  // a second range (gdm_apply_planes2), clipped to the owned planes like the first
  zb2 = std::max(zb2, a.out_z0);
  ze2 = std::min(ze2, a.out_z1);
  const int len2 = std::max(0, ze2 - zb2);
  const int len = ze - zb + len2;
  a.cz0[0] = zb; a.cz1[0] = ze; a.cz0[1] = len2 ? zb2 : 0; a.cz1[1] = len2 ? ze2 : 0;
  a.zchunk = (int)std::max<int64_t>(std::min(len, 8), (len + chunks - 1) / chunks);
  a.nchunk0 = (ze - zb + a.zchunk - 1) / a.zchunk;
  const bool with_tail = n_tail > 0 && tail && op->tail_counter;
  bool ran = false;
  const hipError_t e = gdmk_launch_stencil8(op->p, bk, a, with_tail ? tail : nullptr, with_tail ? n_tail : 0,
                                            op->tail_counter, &ran, op->stream);
  if (e == hipSuccess && tail_done) *tail_done = ran;
  return e;
}

// the inflow faces' launch arguments (faces with |a.n| > 0, in face order)
int face_args(gdm_op *op, const double *bc_values, double *dst_owned, int phase, gdmk::FaceArgs *fas) {
  constexpr int kMax = gdmk::BcStage::kMaxFaces;
  if (op->faces.size() > (size_t)kMax) throw std::runtime_error("more than 6 boundary faces");
  int nf = 0;
  for (size_t fi = 0; fi < op->faces.size(); ++fi) {
    const Face &F = op->faces[fi];
    if (F.scale == 0.0) continue;
    gdmk::FaceArgs &fa = fas[nf];
    fa.U = bc_values + F.offset;
    fa.Q0 = F.t0.Q;
    fa.Q1 = F.t1.Q;
    fa.i0_begin = F.t0.node_begin;
    fa.i0_end = F.t0.node_end;
    fa.i1_begin = F.t1.node_begin;
    fa.i1_end = F.t1.node_end;
    fa.qs0 = F.t0.qs;
    fa.w0T = F.t0.wT;
    fa.wmax0 = F.t0.wmax;
    fa.ldw0 = F.t0.n_nodes;
    fa.qmax0 = F.t0.qmax;
    fa.qs1 = F.t1.qs;
    fa.qc1 = F.t1.qc;
    fa.w1 = F.t1.w;
    fa.wmax1 = F.t1.wmax;
    fa.phi0 = F.t0.phi;
    fa.crange0 = F.t0.crange;
    fa.p = op->p;
    fa.ncell0_total = F.t0.ncell_total;
    fa.cell0_begin = F.t0.cell_begin;
    fa.T = F.T ? F.T : op->face_tmp;
    fa.dst = dst_owned;
    fa.base = F.base;
    fa.stride0 = F.t0.stride;
    fa.stride1 = F.t1.stride;
    fa.scale = F.scale;
    fa.phase = phase;
    ++nf;
  }
  return nf;
}

// phase 0: both steps on op->stream; 1: step 1 (bc values -> per-face T) on
// stream `st`; 2: step 2 (T -> dst) on op->stream; 3: every face's step 1 on
// stream `st`; 4: every face's step 2 + ordered adds into dst on op->stream
// stage (non-NULL): the boundary values are evaluated from its function
// (gdm_apply_bc_fn) instead of read from bc_values
void launch_boundary_data(gdm_op *op, const double *bc_values, double *dst_owned, int phase = 0,
                          hipStream_t st = nullptr) {
  if (op->kind != GDM_OP_ADVECTION) return;
  if (phase == 0) {
    // both steps on op->stream: step 1 of every face, then step 2 + adds
    launch_boundary_data(op, bc_values, dst_owned, 3, op->stream);
    launch_boundary_data(op, bc_values, dst_owned, 4);
    return;
  }
  constexpr int kMax = gdmk::BcStage::kMaxFaces;
  gdmk::FaceArgs fas[kMax] = {};
  const int nf = face_args(op, bc_values, dst_owned, phase, fas);
  // Phase 3 (side stream): every face's step 1 into its own T while the
  // stencil runs (one launch); phase 4, after the join: every face's step 2
  // fused with the adds into dst, each node's terms added in face order by
  // one thread (the roundings of phase 0's face-by-face dst += scale s).  Two
  // faces share the box-edge nodes: a concurrent add (fp64 atomics on the
  // edges) made the edge sums order-dependent, which the bit-exact rank /
  // communicator comparisons of tests/test_host_mpi.py catch.
  const hipStream_t fst = (phase == 1 || phase == 3) && st ? st : op->stream;
  bool all_t = true;
  for (int i = 0; i < nf; ++i) all_t = all_t && fas[i].T != op->face_tmp;
  if (phase == 4 && all_t && op->dim == 3) {
    gdmk::FaceAddFace ff[kMax] = {};
    int m = 0;
    bool ok = true;
    for (size_t fi = 0; fi < op->faces.size(); ++fi) {
      const Face &F = op->faces[fi];
      if (F.scale == 0.0) continue;
      gdmk::FaceAddFace &a = ff[m++];
      a.base = F.base;
      a.stride0 = F.t0.stride;
      a.stride1 = F.t1.stride;
      a.d = F.d;
      a.plane = F.side ? (int)(op->N[F.d] - 1) : 0;
      a.a0 = F.t0.dim_index;
      a.b0 = F.t0.node_begin;
      a.e0 = F.t0.node_end;
      a.a1 = F.t1.dim_index;
      a.b1 = F.t1.node_begin;
      a.e1 = F.t1.node_end;
      ok = ok && a.a0 >= 0 && a.a1 >= 0;
    }
    if (ok) {
      const int64_t own_off = (int64_t)op->layout.owned_plane_begin * op->layout.plane_size;
      const hipError_t e =
          gdmk_launch_faces_step2_add(fas, ff, m, op->N[0], op->N[1], own_off, dst_owned, op->stream);
      if (e == hipSuccess) return;
      if (e != hipErrorNotSupported) hip_check(e, "face step 2 + adds");
    }
  }
  if (phase == 3 && all_t) {
    const hipError_t e = gdmk_launch_faces_step1(fas, nf, fst);
    if (e == hipSuccess) return;
    if (e != hipErrorNotSupported) hip_check(e, "faces step 1");
  }
  // face by face: phase 3 = step 1 into T, phase 4 = step 2 from T into dst
  for (int i = 0; i < nf; ++i) {
    if (phase == 3) fas[i].phase = 1;
    if (phase == 4) fas[i].phase = 2;
    hip_check(gdmk_launch_face(fas[i], fst), "face launch");
  }
}

// compute_rhs = stencil + inflow data.  The inflow faces' step 1 runs in the
// tail of the stencil launch (its workgroups take the face rows once their
// chunk is done); where that is not available (v7 meshes) after the stencil;
// then step 2 with the ordered adds.
void apply_with_faces(gdm_op *op, bool mass, const double *src_local, double *dst_owned, const double *bc_values) {
  constexpr int kMax = gdmk::BcStage::kMaxFaces;
  gdmk::FaceArgs fas[kMax] = {};
  const int nf = bc_values && op->kind == GDM_OP_ADVECTION ? face_args(op, bc_values, dst_owned, 1, fas) : 0;
  bool tail_done = false;
  if (nf > 0) {
    hip_check(launch_stencil(op, mass, src_local, dst_owned, -1, -1, fas, nf, &tail_done), "stencil launch");
    if (tail_done) {
      launch_boundary_data(op, bc_values, dst_owned, 4);
      return;
    }
    // the stencil ran without the tail work: step 1 after it
    launch_boundary_data(op, bc_values, dst_owned, 3, op->stream);
    launch_boundary_data(op, bc_values, dst_owned, 4);
    return;
  }
  hip_check(launch_stencil(op, mass, src_local, dst_owned), "stencil launch");
}

int choose_zchunk(const gdm_op *op) {
  const int nz = op->part_axis == 2 ? (op->layout.owned_plane_end - op->layout.owned_plane_begin) : 1;
  const int ty = gdmk_stencil_tile_rows(op->p);
  const int64_t tiles = (int64_t)((op->K[0] + 63) / 64) * ((op->K[1] + ty - 1) / ty);
  // aim for one round of ~256 workgroups (one 16-wave workgroup per CU)
  const int64_t chunks = std::max<int64_t>(1, (256 + tiles - 1) / tiles);
  int zc = (int)std::max<int64_t>(8, (nz + chunks - 1) / chunks);
  return std::max(1, zc);
}

#define GDM_GUARD_BEGIN try {
#define GDM_GUARD_END                                             \
  }                                                               \
  catch (const HipError &e) { return fail(GDM_ERR_HIP, e.what()); } \
  catch (const std::bad_alloc &) { return fail(GDM_ERR_NOMEM, "out of host memory"); } \
  catch (const std::invalid_argument &e) { return fail(GDM_ERR_ARG, e.what()); } \
  catch (const std::exception &e) { return fail(GDM_ERR_STATE, e.what()); }

}  // namespace

namespace {

constexpr double kSpikeTol = 1e-15;

// x = M^-1 b with the row-form banded Cholesky factor of gdm::cholesky_band
void band_chol_solve(const std::vector<double> &lrow, const std::vector<double> &invd, int n, int hb, double *b) {
  const int wl = hb + 1;
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < hb; ++k) {
      const int j = i - hb + k;
      if (j >= 0) s -= lrow[(size_t)i * wl + k] * b[j];
    }
    b[i] = s * invd[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int m = 1; m <= hb && i + m < n; ++m) s -= lrow[(size_t)(i + m) * wl + (hb - m)] * b[i + m];
    b[i] = s * invd[i];
  }
}

// diagonal block of M on planes [pb, pe) and its spikes:
// V[k][j] = (A^-1 M[pb:pe, pe + j])_k, W[k][j] = (A^-1 M[pb:pe, pb - p + j])_k
struct SlabSpikes {
  gdm::Band A;
  std::vector<double> V, W;
};
SlabSpikes slab_spikes(const gdm::Band &M, int p, int pb, int pe) {
  const int n = pe - pb;
  SlabSpikes r;
  r.A = gdm::Band(n, p);
  for (int i = 0; i < n; ++i)
    for (int j = std::max(0, i - p); j <= std::min(n - 1, i + p); ++j) r.A(i, j) = M(pb + i, pb + j);
  std::vector<double> lrow, invd, col(n);
  gdm::cholesky_band(r.A, lrow, invd);
  r.V.assign((size_t)n * p, 0.0);
  r.W.assign((size_t)n * p, 0.0);
  for (int j = 0; j < p; ++j) {
    for (int i = 0; i < n; ++i) col[i] = M(pb + i, pe + j);
    band_chol_solve(lrow, invd, n, p, col.data());
    for (int i = 0; i < n; ++i) r.V[(size_t)i * p + j] = col[i];
    for (int i = 0; i < n; ++i) col[i] = M(pb + i, pb - p + j);
    band_chol_solve(lrow, invd, n, p, col.data());
    for (int i = 0; i < n; ++i) r.W[(size_t)i * p + j] = col[i];
  }
  return r;
}

// Rows [r0, r0 + p) of the inverse of the interface system
// [[I, Vb], [Wt, I]] (2p x 2p) by Gauss-Jordan with partial pivoting.
std::vector<double> interface_rows(const std::vector<double> &Vb, const std::vector<double> &Wt, int p, int r0) {
  const int m = 2 * p;
  std::vector<double> a((size_t)m * 2 * m, 0.0);
  for (int i = 0; i < m; ++i) {
    a[(size_t)i * 2 * m + i] = 1.0;
    a[(size_t)i * 2 * m + m + i] = 1.0;
  }
  for (int i = 0; i < p; ++i)
    for (int j = 0; j < p; ++j) {
      a[(size_t)i * 2 * m + p + j] = Vb[(size_t)i * p + j];
      a[(size_t)(p + i) * 2 * m + j] = Wt[(size_t)i * p + j];
    }
  for (int c = 0; c < m; ++c) {
    int piv = c;
    for (int i = c + 1; i < m; ++i)
      if (std::abs(a[(size_t)i * 2 * m + c]) > std::abs(a[(size_t)piv * 2 * m + c])) piv = i;
    if (piv != c)
      for (int k = 0; k < 2 * m; ++k) std::swap(a[(size_t)c * 2 * m + k], a[(size_t)piv * 2 * m + k]);
    const double d = a[(size_t)c * 2 * m + c];
    if (d == 0.0) throw std::runtime_error("singular interface system");
    for (int k = 0; k < 2 * m; ++k) a[(size_t)c * 2 * m + k] /= d;
    for (int i = 0; i < m; ++i) {
      if (i == c) continue;
      const double f = a[(size_t)i * 2 * m + c];
      if (f != 0.0)
        for (int k = 0; k < 2 * m; ++k) a[(size_t)i * 2 * m + k] -= f * a[(size_t)c * 2 * m + k];
    }
  }
  std::vector<double> out((size_t)p * m);
  for (int i = 0; i < p; ++i)
    for (int k = 0; k < m; ++k) out[(size_t)i * m + k] = a[(size_t)(r0 + i) * 2 * m + m + k];
  return out;
}

// Largest entry of the couplings the truncated interface systems drop: the
// far spikes W_s^bot (slab s's last p rows of W) and V_s^top over all slabs;
// min_planes = the thinnest slab.
double spike_eps(const gdm::Band &M, int p, unsigned n_cells, unsigned n_ranks, int *min_planes = nullptr) {
  double eps = 0.0;
  int mn = 1 << 30;
  for (unsigned s = 0; s < n_ranks; ++s) {
    const gdm::Slab sl = gdm::slab_partition(n_cells, n_ranks, s);
    const int pb = (int)sl.plane_begin, pe = (int)std::max(sl.plane_begin, sl.plane_end), n = pe - pb;
    mn = std::min(mn, n);
    if (min_planes) *min_planes = mn;
    if (n_ranks == 1) return 0.0;
    if (n < p) return 1.0;  // a slab thinner than the interface
    const SlabSpikes sp = slab_spikes(M, p, pb, pe);
    for (int a = 0; a < p; ++a)
      for (int j = 0; j < p; ++j) {
        if (s > 0) eps = std::max(eps, std::abs(sp.W[(size_t)(n - p + a) * p + j]));
        if (s + 1 < n_ranks) eps = std::max(eps, std::abs(sp.V[(size_t)a * p + j]));
      }
  }
  return eps;
}

// Refinement rounds of the truncated interface systems.  The 2p x 2p system
// of interface (r, r+1) drops the couplings W_r^bot x_{r-1}^bot and
// V_{r+1}^top x_{r+2}^top (entries <= eps).  A round evaluates them at the
// current interface values, moves them to the right-hand sides (one more
// p-plane exchange) and re-solves: block Jacobi on the reduced SPIKE system,
// error ~ eps^(m+1) after m rounds (C4 at 8 ranks: eps = 2e-8, one round,
// 4e-16).  Rounds need the first and last p planes of every slab distinct.
constexpr int kSpikeMaxRounds = 3;
int spike_rounds(double eps, int min_planes, int p) {
  if (eps <= kSpikeTol) return 0;
  if (eps >= 1e-2 || min_planes < 2 * p) return -1;
  double e = eps;
  for (int m = 1; m <= kSpikeMaxRounds; ++m) {
    e *= eps;
    if (e <= kSpikeTol) return m;
  }
  return -1;
}

void build_spike(gdm_op *op) {
  SpikeTables &T = op->spike;
  const int p = op->p, q = op->dim - 1;
  const unsigned nc = (unsigned)op->mesh.n_subdivisions[q], R = (unsigned)op->mesh.n_ranks, r = (unsigned)op->mesh.rank;
  const gdm::Band M = gdm::assemble_1d(p, nc, (op->mesh.hi[q] - op->mesh.lo[q]) / nc).M;
  T.built = true;
  int min_planes = 0;
  T.eps = spike_eps(M, p, nc, R, &min_planes);
  T.rounds = spike_rounds(T.eps, min_planes, p);
  if (T.rounds < 0) return;
  auto planes = [&](unsigned s) {
    const gdm::Slab sl = gdm::slab_partition(nc, R, s);
    return std::make_pair((int)sl.plane_begin, (int)std::max(sl.plane_begin, sl.plane_end));
  };
  const auto [pb, pe] = planes(r);
  const int n = pe - pb;
  T.n_planes = n;
  T.has_lo = r > 0;
  T.has_hi = r + 1 < R;
  const gdm_layout &L = op->layout;
  if ((T.has_lo && L.ghost_planes_below != p) || (T.has_hi && L.ghost_planes_above != p))
    throw std::runtime_error("spike: ghost layer shallower than p planes");
  const SlabSpikes me = slab_spikes(M, p, pb, pe);
  T.slab = build_line_tables(op, me.A);
  std::vector<double> VW((size_t)n * 2 * p), S((size_t)2 * p * 2 * p, 0.0);
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < p; ++j) {
      VW[(size_t)k * 2 * p + j] = T.has_hi ? me.V[(size_t)k * p + j] : 0.0;
      VW[(size_t)k * 2 * p + p + j] = T.has_lo ? me.W[(size_t)k * p + j] : 0.0;
    }
  auto rows = [&](const std::vector<double> &X, int first) {
    return std::vector<double>(X.begin() + (size_t)first * p, X.begin() + (size_t)(first + p) * p);
  };
  if (T.has_lo) {  // interface (r-1, r): x_{r-1}^bot = rows [0, p)
    const auto [qb, qe] = planes(r - 1);
    const SlabSpikes lo = slab_spikes(M, p, qb, qe);
    const std::vector<double> X = interface_rows(rows(lo.V, qe - qb - p), rows(me.W, 0), p, 0);
    std::copy(X.begin(), X.end(), S.begin());
  }
  if (T.has_hi) {  // interface (r, r+1): x_{r+1}^top = rows [p, 2p)
    const auto [qb, qe] = planes(r + 1);
    const SlabSpikes hi = slab_spikes(M, p, qb, qe);
    const std::vector<double> X = interface_rows(rows(me.V, n - p), rows(hi.W, 0), p, p);
    std::copy(X.begin(), X.end(), S.begin() + (size_t)p * 2 * p);
  }
  // planes whose correction can change x (spike rows above 1e-18)
  T.k_begin = n;
  T.k_end = 0;
  for (int k = 0; k < n; ++k) {
    double mx = 0.0;
    for (int j = 0; j < 2 * p; ++j) mx = std::max(mx, std::abs(VW[(size_t)k * 2 * p + j]));
    if (mx > 1e-18) {
      T.k_begin = std::min(T.k_begin, k);
      T.k_end = k + 1;
    }
  }
  T.VW = keep(op, dev_upload(VW));
  T.S = keep(op, dev_upload(S));
  if (T.rounds > 0)
    T.G0 = keep(op, dev_upload(std::vector<double>((size_t)2 * p * std::max<int64_t>(L.plane_size, 1), 0.0)));
}

// the line solves of M^-1 along every kernel axis; `part` replaces the
// partitioned axis' tables by the slab's diagonal block (multi-rank)
// rk (single rank): the RK stage update of gdm_mass_solve_rk fused into the
// last pass when that is the unsegmented v3 x pass; returns whether it was
// (else x_owned holds M^-1 rhs and the caller updates)
bool mass_solve_passes(gdm_op *op, const double *rhs_owned, double *x_owned, const LineTables *part,
                       const gdmk::RkOut *rk = nullptr) {
  const int64_t n = op->layout.n_owned;
  if (n <= 0) return false;
  int64_t K[3] = {op->K[0], op->K[1], op->K[2]};
  LineTables tab[3];
  for (int ax = 0; ax < 3; ++ax) {
    tab[ax].lrow = op->lrow[ax];
    tab[ax].invd = op->invd[ax];
    tab[ax].l3 = op->l3[ax];
    tab[ax].u3 = op->u3[ax];
    tab[ax].d3 = op->d3[ax];
    tab[ax].cst = op->cst3_host[ax];
    tab[ax].row_lo = op->row_lo3[ax];
    tab[ax].row_hi = op->row_hi3[ax];
  }
  if (part) {
    tab[op->part_axis] = *part;
    K[op->part_axis] = op->layout.owned_plane_end - op->layout.owned_plane_begin;
  }
  const int64_t X = K[0], Y = K[1], Z = K[2];
  // v3 (gdm_mass.hip, single sweep per direction) where supported, else v2
  // (two sweeps).  Large meshes: the first pass reads rhs and writes x, later
  // passes in place.  A pass with fewer than gdmk_mass3_seg_waves() waves of
  // lines (2D C2: 16; the y and x passes of a C3 / C4 rank's slab) splits its
  // lines into segments, which read their neighbours' input: such a pass runs
  // out of place (x <-> the scratch vector), the others in place, the outputs
  // chosen from the last pass (x) backwards so that no copy is needed unless
  // the first pass is segmented and rhs is x
  const bool v3 = gdmk_mass3_chunk(op->p) > 0;
  struct Pass {
    int ax, dir_kind;
    int64_t len, stride, n_lines, A, B;
    const char *what;
  };
  std::vector<Pass> passes;
  const bool part_z = part && op->part_axis == 2, part_y = part && op->part_axis == 1;
  if (Z > 1 || part_z) passes.push_back({2, 1, Z, X * Y, X * Y, X * Y, 0, "mass z"});  // base = l, step X*Y
  if (Y > 1 || part_y) passes.push_back({1, 1, Y, X, X * Z, X, X * Y, "mass y"});      // base = z*X*Y + x, step X
  if (X > 1) passes.push_back({0, 0, X, 1, Y * Z, 1, 0, "mass x"});                   // contiguous rows of length X
  auto use_v3 = [&](const Pass &q, const double *src, const double *dst) {
    const LineTables &t = tab[q.ax];
    // strided lines no longer than one v3 chunk (a slab's z lines at C4 on 8
    // ranks: 32 planes) run the two-sweep kernel: the single-sweep one spends
    // such a line in its table-row path (every row of a 32-line is a boundary
    // row); C4 rank SPIKE solve 0.146 -> 0.142 ms (profiles/r5_experiments)
    if (q.dir_kind == 1 && q.len <= gdmk_mass3_chunk(op->p)) return false;
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    // the v3 strided kernel addresses a wave's 64 lines through one buffer
    // resource (num_records 0x7fffffff) with 32-bit position offsets: the
    // line span (len - 1) * stride plus the 64 lanes must stay below 2^31
    // bytes (3D meshes up to 645 vertices per direction), else the v2 kernel
    // (64-bit addresses) runs
    const int64_t lanes = q.A == 1 ? 63 * q.B + 1 : 64;  // a wave's lane span (A = 1: x lines, B apart)
    const bool span_ok = q.dir_kind != 1 || ((q.len - 1) * q.stride + lanes) * 8 < (int64_t)0x7fffffff;
    return v3 && t.l3 && span_ok && (q.dir_kind == 1 || (q.len % 2 == 0 && aligned));
  };
  const int np = (int)passes.size();
  bool seg[3] = {false, false, false}, segmented = false;
  for (int i = 0; i < np; ++i) {
    const Pass &q = passes[(size_t)i];
    seg[i] = v3 && tab[q.ax].l3 && (q.n_lines + 63) / 64 < gdmk_mass3_seg_waves();
    segmented = segmented || seg[i];
  }
  double *tmp = nullptr;
  if (segmented) {
    if (op->mass_tmp_size < n) {  // once per operator (n is the owned size), freed with it
      hip_check(hipMalloc(&op->mass_tmp, sizeof(double) * n), "hipMalloc");
      keep(op, op->mass_tmp);
      op->mass_tmp_size = n;
    }
    tmp = op->mass_tmp;
  }
  // pass outputs, last to first: a segmented pass reads the other buffer than
  // it writes, an unsegmented one may run in place
  double *outs[3] = {x_owned, x_owned, x_owned};
  for (int i = np - 1; i > 0; --i) outs[i - 1] = seg[i] ? (outs[i] == x_owned ? tmp : x_owned) : outs[i];
  const double *in = rhs_owned;
  for (int i = 0; i < np; ++i) {
    const Pass &q = passes[(size_t)i];
    double *out = outs[i];
    if (seg[i] && out == in) {  // rhs aliases the first pass's output: move it aside
      double *other = out == x_owned ? tmp : x_owned;
      hip_check(hipMemcpyAsync(other, in, sizeof(double) * n, hipMemcpyDeviceToDevice, op->stream), "copy");
      in = other;
    }
    const LineTables &t = tab[q.ax];
    if (rk && i == np - 1 && !segmented && !part && q.dir_kind == 0 && use_v3(q, in, in)) {
      const hipError_t e = gdmk_launch_mass3_rk(op->p, in, (int)q.len, q.n_lines, t.l3, t.u3, t.d3, t.cst.data(),
                                                t.row_lo, t.row_hi, *rk, op->stream);
      if (e == hipSuccess) return true;
      if (e != hipErrorNotSupported) hip_check(e, "mass x + rk update");
    }
    if (use_v3(q, in, out))
      hip_check(gdmk_launch_mass3(op->p, q.dir_kind, in, out, (int)q.len, q.stride, q.n_lines, q.A, q.B, t.l3, t.u3,
                                  t.d3, t.cst.data(), t.row_lo, t.row_hi, seg[i] ? 1 : 0, op->stream),
                q.what);
    else
      hip_check(gdmk_launch_mass_lines(op->p, q.dir_kind, in, out, (int)q.len, q.stride, q.n_lines, q.A, q.B, t.lrow,
                                       t.invd, 0, op->stream),
                q.what);
    in = out;
  }
  if (in != x_owned)
    hip_check(hipMemcpyAsync(x_owned, in, sizeof(double) * n, hipMemcpyDeviceToDevice, op->stream), "copy");
  return false;
}

}  // namespace

extern "C" {

int gdm_last_error(char *buf, size_t len) {
  if (!buf || len == 0) return GDM_ERR_ARG;
  std::snprintf(buf, len, "%s", g_last_error.c_str());
  return GDM_OK;
}

int gdm_abi_version(void) { return GDM_HIP_ABI_VERSION; }

int gdm_get_device_count(int *n) {
  if (!n) return fail(GDM_ERR_ARG, "n is NULL");
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    return fail(GDM_ERR_HIP, hipGetErrorString(e));
  }
  return GDM_OK;
}

int gdm_op_create(const gdm_mesh_desc *mesh, int kind, const double *params, int n_params, int device,
                  gdm_op **out) {
  if (!mesh || !out) return fail(GDM_ERR_ARG, "mesh/out is NULL");
  *out = nullptr;
  const int dim = mesh->dim, p = mesh->fe_degree;
  if (dim < 1 || dim > 3) return fail(GDM_ERR_ARG, "dim must be 1, 2 or 3");
  if (p < 1 || p > 9 || p % 2 == 0)
    return fail(GDM_ERR_UNSUPPORTED, "fe_degree must be odd in [1, 9] (fe.h:321-323 tabulates odd p only)");
  if (kind < GDM_OP_MASS || kind > GDM_OP_CONVECTIVE) return fail(GDM_ERR_ARG, "unknown operator kind");
  for (int d = 0; d < dim; ++d) {
    if (mesh->n_subdivisions[d] < p)
      return fail(GDM_ERR_ARG, "n_subdivisions must be >= fe_degree in every direction");
    if (!(mesh->hi[d] > mesh->lo[d])) return fail(GDM_ERR_ARG, "empty box");
  }
  if (mesh->n_ranks < 1 || mesh->rank < 0 || mesh->rank >= mesh->n_ranks) return fail(GDM_ERR_ARG, "bad rank");
  if (mesh->periodic & ~((1 << dim) - 1)) return fail(GDM_ERR_ARG, "periodic bit beyond dim");
  if (mesh->periodic) {
    if (mesh->n_ranks != 1) return fail(GDM_ERR_UNSUPPORTED, "periodic constraints: single rank only");
    if (kind == GDM_OP_ADVECTION)
      return fail(GDM_ERR_UNSUPPORTED,
                  "periodic constraints with the advection face terms (use the convective form of "
                  "prototypes/advection_01_gdm.cc)");
    if (kind == GDM_OP_WAVE && n_params > 0 && params && params[0] > 0.0)
      return fail(GDM_ERR_UNSUPPORTED, "periodic constraints with box Nitsche terms");
  }
  if ((kind == GDM_OP_ADVECTION || kind == GDM_OP_CONVECTIVE) && (n_params < dim || !params))
    return fail(GDM_ERR_ARG, "advection needs the constant field a (dim values)");
  gdm_op *op = new (std::nothrow) gdm_op();
  if (!op) return fail(GDM_ERR_NOMEM, "out of host memory");
  GDM_GUARD_BEGIN
  op->device = device;
  op->mesh = *mesh;
  op->kind = kind;
  op->p = p;
  op->dim = dim;
  for (int d = 0; d < dim; ++d) op->N[d] = mesh->n_subdivisions[d] + 1;
  if (kind == GDM_OP_ADVECTION || kind == GDM_OP_CONVECTIVE)
    for (int d = 0; d < dim; ++d) op->a[d] = params[d];
  if (kind == GDM_OP_WAVE && n_params >= 1 && params) op->nitsche = params[0];
  // kernel axes: 3D (x, y, z) partition z; 2D (x, y, -) partition y; 1D (-, -, x) partition z
  if (dim == 3) {
    op->kdir[0] = 0; op->kdir[1] = 1; op->kdir[2] = 2; op->part_axis = 2;
  } else if (dim == 2) {
    op->kdir[0] = 0; op->kdir[1] = 1; op->kdir[2] = -1; op->part_axis = 1;
  } else {
    op->kdir[0] = -1; op->kdir[1] = -1; op->kdir[2] = 0; op->part_axis = 2;
  }
  for (int ax = 0; ax < 3; ++ax) op->K[ax] = op->kdir[ax] < 0 ? 1 : op->N[op->kdir[ax]];
  hip_check(hipSetDevice(device), "hipSetDevice");
  hip_check(hipStreamCreateWithFlags(&op->own_stream, hipStreamNonBlocking), "hipStreamCreate");
  op->stream = op->own_stream;
  hip_check(hipMalloc(&op->tail_counter, sizeof(unsigned long long)), "hipMalloc");
  keep(op, op->tail_counter);
  hip_check(hipMemset(op->tail_counter, 0, sizeof(unsigned long long)), "hipMemset");
  build_layout(op);
  build_tables(op);
  build_faces(op);
  op->zchunk = choose_zchunk(op);
  hip_check(hipMalloc(&op->dot_partial, sizeof(double) * op->n_dot_partial), "hipMalloc");
  keep(op, op->dot_partial);
  hip_check(hipMalloc(&op->dot_out, sizeof(double)), "hipMalloc");
  keep(op, op->dot_out);
  {
    std::vector<double> w;
    gdm::gauss_unit(p + 1, op->xq, w);
  }
  *out = op;
  return GDM_OK;
  }
  catch (const HipError &e) { free_op(op); return fail(GDM_ERR_HIP, e.what()); }
  catch (const std::bad_alloc &) { free_op(op); return fail(GDM_ERR_NOMEM, "out of host memory"); }
  catch (const std::invalid_argument &e) { free_op(op); return fail(GDM_ERR_ARG, e.what()); }
  catch (const std::exception &e) { free_op(op); return fail(GDM_ERR_STATE, e.what()); }
}

int gdm_op_destroy(gdm_op *op) {
  if (!op) return GDM_OK;
  (void)hipSetDevice(op->device);
  if (op->own_stream) (void)hipStreamSynchronize(op->own_stream);
  free_op(op);
  return GDM_OK;
}

int gdm_halo_plan(const gdm_mesh_desc *mesh, gdm_halo *out) {
  if (!mesh || !out) return fail(GDM_ERR_ARG, "NULL argument");
  const int dim = mesh->dim, p = mesh->fe_degree;
  if (dim < 1 || dim > 3 || p < 1) return fail(GDM_ERR_ARG, "bad mesh");
  if (mesh->n_ranks < 1 || mesh->rank < 0 || mesh->rank >= mesh->n_ranks) return fail(GDM_ERR_ARG, "bad rank");
  const int q = dim - 1;
  const unsigned ncq = (unsigned)mesh->n_subdivisions[q];
  const int nq = (int)ncq + 1;
  int64_t plane = 1;
  for (int d = 0; d < q; ++d) plane *= mesh->n_subdivisions[d] + 1;
  auto lay = [&](int r, int &pb, int &pe, int &gb, int &ga) {
    const gdm::Slab s = gdm::slab_partition(ncq, (unsigned)mesh->n_ranks, (unsigned)r);
    pb = (int)s.plane_begin;
    pe = std::max(pb, (int)s.plane_end);
    gb = pe > pb ? std::min(p, pb) : 0;
    ga = pe > pb ? std::min(p, nq - pe) : 0;
  };
  const int r = mesh->rank;
  int pb, pe, gb, ga;
  lay(r, pb, pe, gb, ga);
  gdm_halo h{};
  h.rank_below = (r > 0 && pe > pb) ? r - 1 : -1;
  h.rank_above = (r + 1 < mesh->n_ranks && pe > pb) ? r + 1 : -1;
  h.owned_offset = (int64_t)gb * plane;
  if (h.rank_below >= 0) {
    int nb, ne, ngb, nga;
    lay(r - 1, nb, ne, ngb, nga);
    if (nga > pe - pb) return fail(GDM_ERR_UNSUPPORTED, "slab thinner than the halo");
    h.send_below_offset = (int64_t)gb * plane;
    h.send_below_count = (int64_t)nga * plane;
    h.recv_below_offset = 0;
    h.recv_below_count = (int64_t)gb * plane;
  }
  if (h.rank_above >= 0) {
    int nb, ne, ngb, nga;
    lay(r + 1, nb, ne, ngb, nga);
    if (ngb > pe - pb) return fail(GDM_ERR_UNSUPPORTED, "slab thinner than the halo");
    h.send_above_offset = (int64_t)(gb + (pe - pb) - ngb) * plane;
    h.send_above_count = (int64_t)ngb * plane;
    h.recv_above_offset = (int64_t)(gb + (pe - pb)) * plane;
    h.recv_above_count = (int64_t)ga * plane;
  }
  // the reference's ghost layer: DoF boxes of the cells next to the owned
  // cell slab (one ghost cell layer, system.h:767-771) minus the owned planes
  {
    const gdm::Slab s = gdm::slab_partition(ncq, (unsigned)mesh->n_ranks, (unsigned)r);
    int lo = pb, hi = pe;
    if (s.cell_end > s.cell_begin) {
      const unsigned c0 = s.cell_begin > 0 ? s.cell_begin - 1 : 0;
      const unsigned c1 = std::min(ncq, s.cell_end + 1);
      for (unsigned c = c0; c < c1; ++c) {
        const int off = (int)gdm::box_offset(c, (unsigned)p, ncq);
        lo = std::min(lo, off);
        hi = std::max(hi, off + p + 1);
      }
    }
    h.dealii_ghost_planes_below = pb - lo;
    h.dealii_ghost_planes_above = hi - pe;
  }
  *out = h;
  return GDM_OK;
}

int gdm_mass_diagonal(gdm_op *op, double *diag_owned) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && !diag_owned) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const std::vector<double> d = mass_diagonal_owned(op);
  if (!d.empty())
    hip_check(hipMemcpyAsync(diag_owned, d.data(), sizeof(double) * d.size(), hipMemcpyHostToDevice, op->stream),
              "copy");
  hip_check(hipStreamSynchronize(op->stream), "sync");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_vec_pointwise_mult(gdm_op *op, int64_t n, const double *w, const double *x, double *y) {
  if (!op || (n > 0 && (!w || !x || !y))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(gdmk_launch_vmul(n, w, x, y, op->stream), "vmul");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_memcpy_d2d(gdm_op *op, void *dst, const void *src, size_t bytes) {
  if (!op || (bytes && (!dst || !src))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  if (bytes) hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, op->stream), "copy");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_op_layout(const gdm_op *op, gdm_layout *out) {
  if (!op || !out) return fail(GDM_ERR_ARG, "op/out is NULL");
  *out = op->layout;
  return GDM_OK;
}

int gdm_op_set_stream(gdm_op *op, void *hip_stream) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  op->stream = (hipStream_t)hip_stream;
  return GDM_OK;
}

int gdm_op_get_stream(const gdm_op *op, void **hip_stream) {
  if (!op || !hip_stream) return fail(GDM_ERR_ARG, "NULL argument");
  *hip_stream = (void *)op->stream;
  return GDM_OK;
}

int gdm_op_use_own_stream(gdm_op *op) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  op->stream = op->own_stream;
  return GDM_OK;
}

namespace {

// constraints.distribute(src) into a scratch copy, the operator, then the
// condensation of distribute_local_to_global (system.h:427-463 constraints:
// x_{last} = x_{first} per periodic direction; rows of constrained DoFs zero)
void periodic_stencil(gdm_op *op, bool mass, const double *src, double *dst) {
  const int64_t n = op->layout.n_local;
  if (!op->pscratch) op->pscratch = keep(op, dev_upload(std::vector<double>((size_t)std::max<int64_t>(n, 1), 0.0)));
  hip_check(hipMemcpyAsync(op->pscratch, src, sizeof(double) * n, hipMemcpyDeviceToDevice, op->stream), "copy");
  const int64_t N[3] = {op->N[0], op->N[1], op->N[2]};
  for (int d = 0; d < op->dim; ++d)
    if (op->mesh.periodic & (1 << d)) hip_check(gdmk_launch_periodic(op->pscratch, N, d, 0, op->stream), "distribute");
  hip_check(launch_stencil(op, mass, op->pscratch, dst), "stencil launch");
  for (int d = op->dim - 1; d >= 0; --d)
    if (op->mesh.periodic & (1 << d)) hip_check(gdmk_launch_periodic(dst, N, d, 1, op->stream), "condense");
}

void any_stencil(gdm_op *op, bool mass, const double *src, double *dst) {
  if (op->mesh.periodic)
    periodic_stencil(op, mass, src, dst);
  else
    hip_check(launch_stencil(op, mass, src, dst), "stencil launch");
}

}  // namespace

int gdm_apply(gdm_op *op, const double *src_local, double *dst_owned, const double *bc_values) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && (!src_local || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  if (op->concurrent && !op->mesh.periodic) {
    apply_with_faces(op, op->kind == GDM_OP_MASS, src_local, dst_owned, bc_values);
  } else {
    any_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned);
    if (bc_values) launch_boundary_data(op, bc_values, dst_owned);
  }
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_apply_planes(gdm_op *op, const double *src_local, double *dst_owned, int plane_begin, int plane_end) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && (!src_local || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  if (op->part_axis != 2 && (plane_begin > op->layout.owned_plane_begin || plane_end < op->layout.owned_plane_end))
    return fail(GDM_ERR_UNSUPPORTED, "gdm_apply_planes: plane sub-ranges need a 3D mesh");
  if (op->mesh.periodic) return fail(GDM_ERR_UNSUPPORTED, "gdm_apply_planes: periodic constraints");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, plane_begin, plane_end),
            "stencil launch");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_apply_planes2(gdm_op *op, const double *src_local, double *dst_owned, int b0, int e0, int b1, int e1) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && (!src_local || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  if (op->part_axis != 2) return fail(GDM_ERR_UNSUPPORTED, "gdm_apply_planes2: plane ranges need a 3D mesh");
  if (op->mesh.periodic) return fail(GDM_ERR_UNSUPPORTED, "gdm_apply_planes2: periodic constraints");
  // clip both ranges to the owned planes first (a first range in
  // the ghost planes must not drop the second), then test overlap and emptiness
  {
    const int ob = op->layout.owned_plane_begin, oe = op->layout.owned_plane_end;
    b0 = std::max(b0, ob);
    e0 = std::min(e0, oe);
    b1 = std::max(b1, ob);
    e1 = std::min(e1, oe);
  }
  if (e0 > b0 && e1 > b1 && b1 < e0 && b0 < e1) return fail(GDM_ERR_ARG, "gdm_apply_planes2: overlapping ranges");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  if (e0 <= b0) {  // one range: the plain launch
    hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, b1, e1), "stencil launch");
    return GDM_OK;
  }
  if (e1 <= b1) {
    hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, b0, e0), "stencil launch");
    return GDM_OK;
  }
  // the v7 path (small meshes) takes one range per launch
  int ty8 = 32, wgs8 = 1;
  gdmk_stencil8_geom(op->p, &ty8, &wgs8);
  if (!(op->K[1] >= ty8 + 2 * op->p + 2 && op->K[0] >= 64 + 2 * op->p + 2)) {
    hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, b0, e0), "stencil launch");
    hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, b1, e1), "stencil launch");
    return GDM_OK;
  }
  hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, b0, e0, nullptr, 0, nullptr, b1, e1),
            "stencil launch");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_add_boundary_data(gdm_op *op, const double *bc_values, double *dst_owned) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_bc_points > 0 && (!bc_values || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  launch_boundary_data(op, bc_values, dst_owned);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_apply(gdm_op *op, const double *src_local, double *dst_owned) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && (!src_local || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  any_stencil(op, true, src_local, dst_owned);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_solve(gdm_op *op, const double *rhs_owned, double *x_owned) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.n_ranks != 1)
    return fail(GDM_ERR_UNSUPPORTED,
                "gdm_mass_solve: single rank; multi-rank: gdm_mass_solve_slab + ghost exchange + gdm_mass_solve_interface");
  if (op->mesh.periodic)
    return fail(GDM_ERR_UNSUPPORTED, "gdm_mass_solve: periodic constraints couple the line ends; use gdm_mass_solve_cg");
  if (!rhs_owned || !x_owned) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  mass_solve_passes(op, rhs_owned, x_owned, nullptr);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_solve_rk(gdm_op *op, double *rhs_owned, double beta, const double *acc_in, double *acc_out,
                      double alpha, const double *y, double *Y) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.n_ranks != 1) return fail(GDM_ERR_UNSUPPORTED, "gdm_mass_solve_rk: single rank");
  if (op->mesh.periodic) return fail(GDM_ERR_UNSUPPORTED, "gdm_mass_solve_rk: periodic constraints");
  if (!rhs_owned || !acc_in || !acc_out || (Y && !y)) return fail(GDM_ERR_ARG, "NULL vector");
  {
    // the fused x pass reads rhs one chunk ahead of the stores to acc_out / Y,
    // and the separate update reads every input element before writing it:
    // both give the same result only under these aliasing rules
    const int64_t n = op->layout.n_owned;
    auto overlap = [n](const double *a, const double *b) { return a && b && a < b + n && b < a + n; };
    auto partial = [&](const double *a, const double *b) { return overlap(a, b) && a != b; };
    if (overlap(rhs_owned, acc_in) || overlap(rhs_owned, acc_out) || overlap(rhs_owned, y) || overlap(rhs_owned, Y))
      return fail(GDM_ERR_ARG, "gdm_mass_solve_rk: rhs_owned overlaps acc_in / acc_out / y / Y");
    if (overlap(acc_out, Y) || partial(acc_out, acc_in) || partial(acc_out, y) || partial(Y, acc_in) ||
        partial(Y, y))
      return fail(GDM_ERR_ARG, "gdm_mass_solve_rk: acc_out / Y must be distinct, or equal (not partially "
                               "overlapping) to an input");
  }
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const gdmk::RkOut rk{acc_in, acc_out, y, Y, beta, alpha};
  if (!mass_solve_passes(op, rhs_owned, rhs_owned, nullptr, &rk))
    hip_check(gdmk_launch_rk_update(op->layout.n_owned, beta, rhs_owned, acc_in, acc_out, alpha, Y ? y : nullptr, Y,
                                    op->stream),
              "rk_update");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_spike_eps(const gdm_mesh_desc *mesh, double *eps_host) {
  if (!mesh || !eps_host) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  if (mesh->dim < 1 || mesh->dim > 3 || mesh->fe_degree < 1 || mesh->n_ranks < 1)
    return fail(GDM_ERR_ARG, "bad mesh description");
  const int q = mesh->dim - 1;
  const unsigned nc = (unsigned)mesh->n_subdivisions[q];
  const gdm::Band M = gdm::assemble_1d(mesh->fe_degree, nc, (mesh->hi[q] - mesh->lo[q]) / nc).M;
  *eps_host = spike_eps(M, mesh->fe_degree, nc, (unsigned)mesh->n_ranks);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_spike_rounds(const gdm_mesh_desc *mesh, int *rounds) {
  if (!mesh || !rounds) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  if (mesh->dim < 1 || mesh->dim > 3 || mesh->fe_degree < 1 || mesh->n_ranks < 1)
    return fail(GDM_ERR_ARG, "bad mesh description");
  const int q = mesh->dim - 1;
  const unsigned nc = (unsigned)mesh->n_subdivisions[q];
  const gdm::Band M = gdm::assemble_1d(mesh->fe_degree, nc, (mesh->hi[q] - mesh->lo[q]) / nc).M;
  int min_planes = 0;
  const double eps = spike_eps(M, mesh->fe_degree, nc, (unsigned)mesh->n_ranks, &min_planes);
  *rounds = spike_rounds(eps, min_planes, mesh->fe_degree);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_solve_slab(gdm_op *op, const double *rhs_owned, double *x_owned) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.periodic) return fail(GDM_ERR_UNSUPPORTED, "gdm_mass_solve_slab: periodic mesh");
  if (op->layout.n_owned > 0 && (!rhs_owned || !x_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  if (op->mesh.n_ranks == 1) {
    mass_solve_passes(op, rhs_owned, x_owned, nullptr);
    return GDM_OK;
  }
  if (!op->spike.built) build_spike(op);
  if (op->spike.rounds < 0) {
    char msg[256];
    std::snprintf(msg, sizeof msg,
                  "gdm_mass_solve_slab: slabs too thin for the interface systems (dropped coupling %.3g, %d "
                  "refinement rounds do not reach %.1g or a slab has < 2p planes); use gdm_mass_solve_cg or fewer "
                  "ranks",
                  op->spike.eps, kSpikeMaxRounds, kSpikeTol);
    return fail(GDM_ERR_UNSUPPORTED, msg);
  }
  op->spike.next_round = -1;
  mass_solve_passes(op, rhs_owned, x_owned, &op->spike.slab);
  op->spike.next_round = 0;
  return GDM_OK;
  GDM_GUARD_END
}

static int mass_solve_interface_impl(gdm_op *op, double *x_local, bool ghosts);

int gdm_mass_solve_interface(gdm_op *op, double *x_local) { return mass_solve_interface_impl(op, x_local, false); }

int gdm_mass_solve_interface_ghosts(gdm_op *op, double *x_local) { return mass_solve_interface_impl(op, x_local, true); }

int gdm_mass_solve_interface_rk(gdm_op *op, const double *x_local, double beta, const double *acc_in, double *acc_out,
                                double alpha, const double *y, double *Y) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.n_ranks == 1)
    return fail(GDM_ERR_UNSUPPORTED, "gdm_mass_solve_interface_rk: multi-rank only (one rank: gdm_mass_solve_rk)");
  if (!op->spike.built || op->spike.rounds < 0 || op->spike.next_round < 0)
    return fail(GDM_ERR_STATE, "gdm_mass_solve_interface_rk: call gdm_mass_solve_slab first");
  if (op->spike.next_round != op->spike.rounds)
    return fail(GDM_ERR_STATE, "gdm_mass_solve_interface_rk: not every refinement round ran since gdm_mass_solve_slab");
  if (op->layout.n_owned > 0 && (!x_local || !acc_in || !acc_out || (Y && !y)))
    return fail(GDM_ERR_ARG, "NULL vector");
  {
    const int64_t n = op->layout.n_local;
    auto overlap = [n](const void *a, const void *b) {
      const double *p = (const double *)a, *q = (const double *)b;
      return p && q && p < q + n && q < p + n;
    };
    if (overlap(x_local, acc_out) || overlap(x_local, Y) || (Y && overlap(acc_out, Y)) ||
        (Y && overlap(Y, acc_in)) || (Y && overlap(Y, y) && Y != y) || (overlap(acc_out, y) && acc_out != y) ||
        (overlap(acc_out, acc_in) && acc_out != acc_in))
      return fail(GDM_ERR_ARG, "gdm_mass_solve_interface_rk: x_local must not overlap the outputs; acc_out / Y may "
                               "only equal (not partially overlap) an input");
  }
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  op->spike.next_round = -1;
  const SpikeTables &S = op->spike;
  const gdm_layout &L = op->layout;
  const gdmk::RkOut rk{acc_in, acc_out, y, Y, beta, alpha};
  hip_check(gdmk_launch_spike_rk(op->p, x_local, L.plane_size, L.ghost_planes_below, L.ghost_planes_above,
                                 S.n_planes, S.has_lo, S.has_hi, S.VW, S.S, S.k_begin, S.k_end,
                                 S.rounds > 0 ? S.G0 : nullptr, rk, op->stream),
            "spike_rk");
  return GDM_OK;
  GDM_GUARD_END
}

static int mass_solve_interface_impl(gdm_op *op, double *x_local, bool ghosts) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.n_ranks == 1) return GDM_OK;
  if (!op->spike.built || op->spike.rounds < 0 || op->spike.next_round < 0)
    return fail(GDM_ERR_STATE, "gdm_mass_solve_interface: call gdm_mass_solve_slab first");
  if (op->spike.next_round != op->spike.rounds) {
    char msg[160];
    std::snprintf(msg, sizeof msg,
                  "gdm_mass_solve_interface: %d of %d refinement rounds ran since gdm_mass_solve_slab "
                  "(gdm_mass_solve_interface_round)",
                  op->spike.next_round, op->spike.rounds);
    return fail(GDM_ERR_STATE, msg);
  }
  if (op->layout.n_owned > 0 && !x_local) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  op->spike.next_round = -1;
  const SpikeTables &S = op->spike;
  if ((S.k_end > S.k_begin || S.rounds > 0 || ghosts) && (S.has_lo || S.has_hi))
    hip_check(gdmk_launch_spike(op->p, x_local, op->layout.plane_size,
                                (int64_t)op->layout.ghost_planes_below * op->layout.plane_size, S.n_planes, S.has_lo,
                                S.has_hi, S.VW, S.S, S.k_begin, S.k_end, ghosts ? 2 : 0, 0,
                                S.rounds > 0 ? S.G0 : nullptr, op->stream),
              "spike");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_solve_interface_round(gdm_op *op, double *x_local, int round) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.n_ranks == 1) return fail(GDM_ERR_STATE, "gdm_mass_solve_interface_round: one rank needs no rounds");
  if (!op->spike.built || op->spike.rounds < 0)
    return fail(GDM_ERR_STATE, "gdm_mass_solve_interface_round: call gdm_mass_solve_slab first");
  if (round < 0 || round >= op->spike.rounds) return fail(GDM_ERR_ARG, "round out of range [0, rounds)");
  if (op->spike.next_round < 0)
    return fail(GDM_ERR_STATE, "gdm_mass_solve_interface_round: call gdm_mass_solve_slab first");
  if (round != op->spike.next_round) return fail(GDM_ERR_STATE, "gdm_mass_solve_interface_round: rounds run in order");
  if (op->layout.n_owned > 0 && !x_local) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const SpikeTables &S = op->spike;
  // the round counts as done only once its launch succeeded; a failed launch
  // voids the whole solve (a later interface call then refuses it)
  const hipError_t e = gdmk_launch_spike(op->p, x_local, op->layout.plane_size,
                                         (int64_t)op->layout.ghost_planes_below * op->layout.plane_size, S.n_planes,
                                         S.has_lo, S.has_hi, S.VW, S.S, S.k_begin, S.k_end, 1, round, S.G0, op->stream);
  if (e != hipSuccess) op->spike.next_round = -1;
  hip_check(e, "spike round");
  ++op->spike.next_round;
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_solve_cg(gdm_op *op, const double *rhs_owned, double *x_owned, double rel_tol, double abs_tol,
                      int max_it, int precond, int *its_host, double *res_host) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->mesh.n_ranks != 1) return fail(GDM_ERR_UNSUPPORTED, "gdm_mass_solve_cg: single rank in this version");
  if (!rhs_owned || !x_owned || rhs_owned == x_owned) return fail(GDM_ERR_ARG, "rhs and x: distinct device vectors");
  if (precond != 0 && precond != 1) return fail(GDM_ERR_ARG, "precond: 0 identity, 1 Jacobi");
  if (max_it < 0) return fail(GDM_ERR_ARG, "max_it < 0");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const int64_t n = op->layout.n_owned;
  auto vec = [&](double *&v) {
    if (!v) v = keep(op, dev_upload(std::vector<double>((size_t)std::max<int64_t>(n, 1), 0.0)));
  };
  vec(op->cg_r);
  vec(op->cg_p);
  vec(op->cg_Ap);
  vec(op->cg_z);
  if (precond == 1 && !op->cg_invdiag) {
    std::vector<double> inv = mass_diagonal_owned(op);
    for (double &v : inv) v = 1.0 / v;
    op->cg_invdiag = keep(op, dev_upload(inv));
  }
  auto dot = [&](const double *a, const double *b) {
    double r = 0.0;
    if (gdm_vec_dot(op, n, a, b, &r) != GDM_OK) throw std::runtime_error("dot");
    return r;
  };
  auto precondition = [&](const double *r, double *z) {
    if (precond == 1)
      hip_check(gdmk_launch_vmul(n, op->cg_invdiag, r, z, op->stream), "jacobi");
    else
      hip_check(hipMemcpyAsync(z, r, sizeof(double) * n, hipMemcpyDeviceToDevice, op->stream), "copy");
  };
  // SolverCG with ReductionControl(max_it, abs_tol, rel_tol): r = b - A x
  any_stencil(op, true, x_owned, op->cg_r);
  hip_check(gdmk_launch_axpby(n, 1.0, rhs_owned, -1.0, op->cg_r, op->stream), "axpby");
  double res = std::sqrt(dot(op->cg_r, op->cg_r));
  const double tol = std::max(abs_tol, rel_tol * res);
  int it = 0;
  if (res > tol) {
    precondition(op->cg_r, op->cg_z);
    hip_check(hipMemcpyAsync(op->cg_p, op->cg_z, sizeof(double) * n, hipMemcpyDeviceToDevice, op->stream), "copy");
    double rz = dot(op->cg_r, op->cg_z);
    while (true) {
      if (it >= max_it) {
        if (its_host) *its_host = it;
        if (res_host) *res_host = res;
        return fail(GDM_ERR_STATE, "gdm_mass_solve_cg: max_it reached (SolverControl::NoConvergence)");
      }
      ++it;
      any_stencil(op, true, op->cg_p, op->cg_Ap);
      const double alpha = rz / dot(op->cg_p, op->cg_Ap);
      hip_check(gdmk_launch_axpby(n, alpha, op->cg_p, 1.0, x_owned, op->stream), "axpby");
      hip_check(gdmk_launch_axpby(n, -alpha, op->cg_Ap, 1.0, op->cg_r, op->stream), "axpby");
      res = std::sqrt(dot(op->cg_r, op->cg_r));
      if (res <= tol) break;
      precondition(op->cg_r, op->cg_z);
      const double rz_new = dot(op->cg_r, op->cg_z);
      hip_check(gdmk_launch_axpby(n, 1.0, op->cg_z, rz_new / rz, op->cg_p, op->stream), "axpby");
      rz = rz_new;
    }
  }
  if (its_host) *its_host = it;
  if (res_host) *res_host = res;
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_constraints_distribute(gdm_op *op, double *v_owned) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (!op->mesh.periodic) return GDM_OK;
  if (!v_owned) return fail(GDM_ERR_ARG, "NULL vector");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const int64_t N[3] = {op->N[0], op->N[1], op->N[2]};
  for (int d = 0; d < op->dim; ++d)
    if (op->mesh.periodic & (1 << d)) hip_check(gdmk_launch_periodic(v_owned, N, d, 0, op->stream), "distribute");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_mass_solve_lines(gdm_op *op, int axis, double *v, int64_t n_lines, int64_t stride, int64_t A, int64_t B,
                         int64_t C) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (axis < 0 || axis >= op->dim) return fail(GDM_ERR_ARG, "axis out of range");
  if (n_lines < 0 || stride <= 0 || A <= 0) return fail(GDM_ERR_ARG, "bad line geometry");
  if (n_lines > 0 && !v) return fail(GDM_ERR_ARG, "NULL vector");
  int kax = -1;
  for (int ax = 0; ax < 3; ++ax)
    if (op->kdir[ax] == axis) kax = ax;
  if (kax < 0 || !op->lrow[kax]) return n_lines == 0 || op->N[axis] <= 1 ? GDM_OK : fail(GDM_ERR_STATE, "no factor");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(gdmk_launch_chol_lines(op->p, v, op->N[axis], stride, n_lines, A, B, C, op->lrow[kax], op->invd[kax],
                                   op->stream),
            "chol lines");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_vec_axpby(gdm_op *op, int64_t n, double a, const double *x, double b, double *y) {
  if (!op || (n > 0 && (!x || !y))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(gdmk_launch_axpby(n, a, x, b, y, op->stream), "axpby");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_vec_rk_update(gdm_op *op, int64_t n, double beta, const double *k, const double *acc_in, double *acc_out,
                      double alpha, const double *y, double *Y) {
  if (!op || (n > 0 && (!k || !acc_in || !acc_out || (Y && !y)))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(gdmk_launch_rk_update(n, beta, k, acc_in, acc_out, alpha, y, Y, op->stream), "rk_update");
  return GDM_OK;
  GDM_GUARD_END
}

}  // extern "C"

namespace {

// argument checks of the built-in boundary functions (gdm_fn_kind); 0 = ok
int check_bc_fn(gdm_op *op, int fn_kind, const double *params, int n_params) {
  const int need[3] = {1, 1 + op->dim, 9};
  if (fn_kind < 0 || fn_kind > 2) return fail(GDM_ERR_ARG, "unknown gdm_fn_kind");
  if (n_params < need[fn_kind] || (n_params > 0 && !params)) return fail(GDM_ERR_ARG, "too few function parameters");
  if (op->faces.size() > (size_t)gdmk::BcStage::kMaxFaces || op->p + 1 > 10)
    return fail(GDM_ERR_UNSUPPORTED, "boundary geometry");
  return GDM_OK;
}

// the boundary-point geometry (device block(0) order) and the function
void build_bc_fn(gdm_op *op, int fn_kind, const double *params, int n_params, gdmk::BcGeom &g, gdmk::BcFn &fn,
                 int &ld) {
  g = gdmk::BcGeom{};
  g.dim = op->dim;
  g.p = op->p;
  g.n_faces = (int)op->faces.size();
  g.n_points = op->layout.n_bc_points;
  for (int d = 0; d < 3; ++d) {
    g.n_sub[d] = op->mesh.n_subdivisions[d];
    g.lo[d] = op->mesh.lo[d];
    g.hi[d] = op->mesh.hi[d];
  }
  for (int q = 0; q <= op->p; ++q) g.xq[q] = op->xq[q];
  for (size_t f = 0; f < op->faces.size(); ++f) {
    const Face &F = op->faces[f];
    gdmk::BcFace &B = g.face[f];
    B.offset = F.offset;
    B.d = F.d;
    B.side = F.side;
    const FaceDir *T[2] = {&F.t0, &F.t1};
    for (int k = 0; k < 2; ++k) {
      B.Q[k] = T[k]->Q;
      B.dim_index[k] = T[k]->dim_index;
      B.cell_begin[k] = T[k]->cell_begin;
    }
  }
  fn = gdmk::BcFn{};
  fn.kind = fn_kind;
  fn.dim = op->dim;
  for (int i = 0; i < n_params && i < 12; ++i) fn.prm[i] = params[i];
  ld = 1;
  for (const Face &F : op->faces) ld = std::max({ld, F.t0.Q, F.t1.Q});
}

}  // namespace

extern "C" {

int gdm_eval_boundary(gdm_op *op, int fn_kind, const double *params, int n_params, double t, int derivative,
                      double *bc_values) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_bc_points > 0 && !bc_values) return fail(GDM_ERR_ARG, "NULL bc_values");
  if (int rc = check_bc_fn(op, fn_kind, params, n_params)) return rc;
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  gdmk::BcGeom g;
  gdmk::BcFn fn;
  int ld = 1;
  build_bc_fn(op, fn_kind, params, n_params, g, fn, ld);
  if (!op->bc_tab || op->bc_tab_ld < ld) {
    std::vector<double> zero((size_t)6 * 3 * ld * 2, 0.0);
    op->bc_tab = keep(op, dev_upload(zero));
    op->bc_tab_ld = ld;
  }
  hip_check(gdmk_launch_bc_eval(g, fn, t, derivative ? 1 : 0, bc_values, op->bc_tab, op->bc_tab_ld, op->stream),
            "bc_eval");
  return GDM_OK;
  GDM_GUARD_END
}

}  // extern "C"

namespace {

// the stage boundary values g(t_g) + alpha dg/dt(t_k) of a built-in function
// into the operator's block(0)-sized scratch (tables + one fill launch on
// `st`); returns the scratch (NULL without boundary points)
const double *fill_stage_boundary(gdm_op *op, int fn_kind, const double *params, int n_params, double t_g,
                                  double alpha, double t_k, hipStream_t st) {
  if (op->layout.n_bc_points <= 0) return nullptr;
  gdmk::BcStage stage{};
  int ld = 1;
  build_bc_fn(op, fn_kind, params, n_params, stage.g, stage.f, ld);
  if (!op->bc_stage_tab || op->bc_stage_ld < ld) {
    std::vector<double> zero((size_t)2 * gdmk::BcStage::kMaxFaces * 3 * ld * 2, 0.0);
    op->bc_stage_tab = keep(op, dev_upload(zero));
    op->bc_stage_ld = ld;
  }
  if (!op->bc_stage_vals) {
    hip_check(hipMalloc(&op->bc_stage_vals, sizeof(double) * op->layout.n_bc_points), "hipMalloc");
    keep(op, op->bc_stage_vals);
  }
  stage.tab = op->bc_stage_tab;
  stage.ld = op->bc_stage_ld;
  stage.alpha = alpha;
  hip_check(gdmk_launch_bc_tables(stage.g, stage.f, t_g, t_k, alpha != 0.0 ? 1 : 0, op->bc_stage_tab, stage.ld, st),
            "bc tables");
  // only the inflow faces: the others' values are never read (scale 0)
  int faces[gdmk::BcStage::kMaxFaces], n = 0;
  for (size_t fi = 0; fi < op->faces.size(); ++fi)
    if (op->faces[fi].scale != 0.0) faces[n++] = (int)fi;
  hip_check(gdmk_launch_bc_stage_fill(stage, faces, n, op->bc_stage_vals, st), "bc stage fill");
  return op->bc_stage_vals;
}

}  // namespace

extern "C" {

int gdm_apply_bc_fn(gdm_op *op, const double *src_local, double *dst_owned, int fn_kind, const double *params,
                    int n_params, double t_g, double alpha, double t_k) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && (!src_local || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  if (op->kind != GDM_OP_ADVECTION) return fail(GDM_ERR_UNSUPPORTED, "gdm_apply_bc_fn: advection operators only");
  if (int rc = check_bc_fn(op, fn_kind, params, n_params)) return rc;
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  // the stage values first, on the op stream (~28 M points at C3: one write
  // pass), then gdm_apply with them; a side-stream launch would wait for the
  // interior launch's workgroups (one per CU, all of its LDS) to drain
  const double *bc = fill_stage_boundary(op, fn_kind, params, n_params, t_g, alpha, t_k, op->stream);
  if (op->concurrent && !op->mesh.periodic) {
    apply_with_faces(op, false, src_local, dst_owned, bc);
  } else {
    any_stencil(op, false, src_local, dst_owned);
    if (bc) launch_boundary_data(op, bc, dst_owned);
  }
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_add_boundary_fn(gdm_op *op, double *dst_owned, int fn_kind, const double *params, int n_params, double t_g,
                        double alpha, double t_k) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_bc_points > 0 && !dst_owned) return fail(GDM_ERR_ARG, "NULL vector");
  if (op->kind != GDM_OP_ADVECTION) return fail(GDM_ERR_UNSUPPORTED, "gdm_add_boundary_fn: advection operators only");
  if (int rc = check_bc_fn(op, fn_kind, params, n_params)) return rc;
  if (op->layout.n_bc_points == 0) return GDM_OK;
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const double *bc = fill_stage_boundary(op, fn_kind, params, n_params, t_g, alpha, t_k, op->stream);
  launch_boundary_data(op, bc, dst_owned);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_error_norms(gdm_op *op, const double *u_local, int fn_kind, const double *params, int n_params, double t,
                    double *cell_errors, double *norms_host) {
  if (!op || !norms_host) return fail(GDM_ERR_ARG, "NULL argument");
  if (op->layout.n_local > 0 && !u_local) return fail(GDM_ERR_ARG, "NULL u_local");
  const int need[3] = {1, 1 + op->dim, 9};
  if (fn_kind < 0 || fn_kind > 2) return fail(GDM_ERR_ARG, "unknown gdm_fn_kind");
  if (n_params < need[fn_kind] || (n_params > 0 && !params)) return fail(GDM_ERR_ARG, "too few function parameters");
  if (op->p + 1 > 10) return fail(GDM_ERR_UNSUPPORTED, "fe_degree > 9");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  const int p = op->p, n1 = p + 1, q = op->dim - 1;
  const gdm_layout &L = op->layout;
  gdmk::ErrGeom g{};
  g.dim = op->dim;
  g.p = p;
  std::vector<double> xq, wq;
  gdm::gauss_unit(n1, xq, wq);
  g.jxw = 1.0;
  for (int d = 0; d < 3; ++d) {
    const bool on = d < op->dim;
    g.ncell[d] = on ? op->mesh.n_subdivisions[d] : 1;
    g.cb[d] = 0;
    g.ce[d] = g.ncell[d];
    g.nb[d] = g.nq[d] = on ? n1 : 1;
    g.lo[d] = on ? op->mesh.lo[d] : 0.0;
    g.h[d] = on ? (op->mesh.hi[d] - op->mesh.lo[d]) / op->mesh.n_subdivisions[d] : 1.0;
    if (on) g.jxw *= g.h[d];
  }
  g.cb[q] = L.cell_plane_begin;
  g.ce[q] = L.cell_plane_end;
  for (int k = 0; k < n1; ++k) {
    g.xq[k] = xq[k];
    g.wq[k] = wq[k];
  }
  g.N0 = op->N[0];
  g.N1 = op->dim > 1 ? op->N[1] : 1;
  g.base = (int64_t)(L.owned_plane_begin - L.ghost_planes_below) * L.plane_size;
  gdmk::BcFn fn{};
  fn.kind = fn_kind;
  fn.dim = op->dim;
  for (int i = 0; i < n_params && i < 12; ++i) fn.prm[i] = params[i];
  if (!op->err_S) {
    const int ncat = std::max(1, p);
    std::vector<double> S((size_t)ncat * n1 * n1);
    for (int c = 0; c < ncat; ++c)
      for (int i = 0; i < n1; ++i)
        for (int k = 0; k < n1; ++k) S[((size_t)c * n1 + i) * n1 + k] = gdm::shape_1d(p, c, i, xq[k], 0);
    op->err_S = keep(op, dev_upload(S));
    op->err_partial = keep(op, dev_upload(std::vector<double>((size_t)3 * op->n_err_partial + 3, 0.0)));
  }
  double out[3] = {0.0, 0.0, 0.0};
  if (g.ce[q] > g.cb[q]) {
    double *res = op->err_partial + 3 * op->n_err_partial;
    hip_check(gdmk_launch_error_norms(g, fn, t, op->err_S, u_local, cell_errors, op->err_partial, op->n_err_partial,
                                      res, op->stream),
              "error_norms");
    hip_check(hipMemcpyAsync(out, res, sizeof(out), hipMemcpyDeviceToHost, op->stream), "d2h");
    hip_check(hipStreamSynchronize(op->stream), "sync");
  }
  norms_host[0] = out[0];
  norms_host[1] = out[1];
  norms_host[2] = std::sqrt(out[2]);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_vec_dot(gdm_op *op, int64_t n, const double *x, const double *y, double *result_host) {
  if (!op || !result_host || (n > 0 && (!x || !y))) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  if (n <= 0) {
    *result_host = 0.0;
    return GDM_OK;
  }
  const int np = (int)std::min<int64_t>(op->n_dot_partial, std::max<int64_t>(1, (n + 255) / 256));
  hip_check(gdmk_launch_dot(n, x, y, op->dot_partial, np, op->dot_out, op->stream), "dot");
  hip_check(hipMemcpyAsync(result_host, op->dot_out, sizeof(double), hipMemcpyDeviceToHost, op->stream), "d2h");
  hip_check(hipStreamSynchronize(op->stream), "sync");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_synchronize(gdm_op *op) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  hipError_t e = hipStreamSynchronize(op->stream);
  if (e != hipSuccess) return fail(GDM_ERR_HIP, hipGetErrorString(e));
  return GDM_OK;
}

int gdm_malloc(gdm_op *op, size_t bytes, void **ptr) {
  if (!op || !ptr) return fail(GDM_ERR_ARG, "NULL argument");
  (void)hipSetDevice(op->device);
  hipError_t e = hipMalloc(ptr, std::max<size_t>(bytes, 1));
  if (e != hipSuccess) return fail(GDM_ERR_NOMEM, hipGetErrorString(e));
  return GDM_OK;
}

int gdm_free(gdm_op *op, void *ptr) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  (void)hipSetDevice(op->device);
  hipError_t e = hipFree(ptr);
  if (e != hipSuccess) return fail(GDM_ERR_HIP, hipGetErrorString(e));
  return GDM_OK;
}

int gdm_memcpy_h2d(gdm_op *op, void *dst, const void *src_host, size_t bytes) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  hipError_t e = hipMemcpyAsync(dst, src_host, bytes, hipMemcpyHostToDevice, op->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(op->stream);
  if (e != hipSuccess) return fail(GDM_ERR_HIP, hipGetErrorString(e));
  return GDM_OK;
}

int gdm_memcpy_d2h(gdm_op *op, void *dst_host, const void *src, size_t bytes) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  hipError_t e = hipMemcpyAsync(dst_host, src, bytes, hipMemcpyDeviceToHost, op->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(op->stream);
  if (e != hipSuccess) return fail(GDM_ERR_HIP, hipGetErrorString(e));
  return GDM_OK;
}

int gdm_bc_points(const gdm_op *op, double *xyz_host) {
  if (!op || !xyz_host) return fail(GDM_ERR_ARG, "NULL argument");
  const int n1 = op->p + 1;
  for (const Face &F : op->faces) {
    const FaceDir *T[2] = {&F.t0, &F.t1};
    for (int64_t i1 = 0; i1 < F.t1.Q; ++i1)
      for (int64_t i0 = 0; i0 < F.t0.Q; ++i0) {
        double *pt = xyz_host + 3 * (F.offset + i1 * F.t0.Q + i0);
        pt[0] = pt[1] = pt[2] = 0.0;
        pt[F.d] = F.side ? op->mesh.hi[F.d] : op->mesh.lo[F.d];
        const int64_t qi[2] = {i0, i1};
        for (int k = 0; k < 2; ++k) {
          const int e = T[k]->dim_index;
          if (e < 0) continue;
          const int c = T[k]->cell_begin + (int)(qi[k] / n1), qq = (int)(qi[k] % n1);
          const double h = (op->mesh.hi[e] - op->mesh.lo[e]) / op->mesh.n_subdivisions[e];
          pt[e] = op->mesh.lo[e] + (c + op->xq[qq]) * h;
        }
      }
  }
  return GDM_OK;
}

int gdm_bc_reference_order(const gdm_op *op, int64_t *ref_to_dev_host) {
  if (!op || !ref_to_dev_host) return fail(GDM_ERR_ARG, "NULL argument");
  // reference order: owned cells lexicographic, faces 0..2dim-1 at the box,
  // face points in deal.II QProjector order (stiffness.h:97-157)
  const int dim = op->dim, n1 = op->p + 1, q = dim - 1;
  const gdm_layout &L = op->layout;
  int nc[3] = {1, 1, 1};
  for (int d = 0; d < dim; ++d) nc[d] = op->mesh.n_subdivisions[d];
  int cb[3] = {0, 0, 0}, ce[3] = {nc[0], nc[1], nc[2]};
  cb[q] = L.cell_plane_begin;
  ce[q] = L.cell_plane_end;
  const int nfq = dim == 1 ? 1 : (dim == 2 ? n1 : n1 * n1);
  int64_t k = 0;
  for (int c2 = cb[2]; c2 < ce[2]; ++c2)
    for (int c1 = cb[1]; c1 < ce[1]; ++c1)
      for (int c0 = cb[0]; c0 < ce[0]; ++c0) {
        const int c[3] = {c0, c1, c2};
        for (int f = 0; f < 2 * dim; ++f) {
          const int d = f / 2, side = f % 2;
          if (!(side ? c[d] == nc[d] - 1 : c[d] == 0)) continue;
          const Face *F = nullptr;
          for (const Face &G : op->faces)
            if (G.d == d && G.side == side) F = &G;
          if (!F) return fail(GDM_ERR_STATE, "face missing");
          for (int qi = 0; qi < nfq; ++qi, ++k) {
            const int aa = qi % n1, bb = qi / n1;
            int qt0 = 0, qt1 = 0;  // quadrature index along t0 / t1
            if (dim == 2) {
              qt0 = aa;
            } else if (dim == 3) {
              if (d == 0) { qt0 = aa; qt1 = bb; }       // (0, q0, q1): y <- a, z <- b
              else if (d == 1) { qt0 = bb; qt1 = aa; }  // (q1, 0, q0): x <- b, z <- a
              else { qt0 = aa; qt1 = bb; }              // (q0, q1, 0): x <- a, y <- b
            }
            int64_t Q0 = 0, Q1 = 0;
            if (F->t0.dim_index >= 0) Q0 = (int64_t)(c[F->t0.dim_index] - F->t0.cell_begin) * n1 + qt0;
            if (F->t1.dim_index >= 0) Q1 = (int64_t)(c[F->t1.dim_index] - F->t1.cell_begin) * n1 + qt1;
            ref_to_dev_host[k] = F->offset + Q1 * F->t0.Q + Q0;
          }
        }
      }
  if (k != L.n_bc_points_ref) return fail(GDM_ERR_STATE, "boundary point count mismatch");
  return GDM_OK;
}

int gdm_time_op(gdm_op *op, int which, const double *src, double *dst, const double *bc_values, int n_iter,
                double *avg_ms_host) {
  if (!op || !avg_ms_host || n_iter <= 0) return fail(GDM_ERR_ARG, "bad argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hipEvent_t e0, e1;
  hip_check(hipEventCreate(&e0), "event");
  hip_check(hipEventCreate(&e1), "event");
  hip_check(hipEventRecord(e0, op->stream), "record");
  int rc = GDM_OK;
  for (int i = 0; i < n_iter && rc == GDM_OK; ++i) {
    if (which == 0) rc = gdm_apply(op, src, dst, bc_values);
    else if (which == 1) rc = gdm_mass_apply(op, src, dst);
    else rc = gdm_mass_solve(op, src, dst);
  }
  hip_check(hipEventRecord(e1, op->stream), "record");
  hip_check(hipEventSynchronize(e1), "sync");
  float ms = 0.f;
  hip_check(hipEventElapsedTime(&ms, e0, e1), "elapsed");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc != GDM_OK) return rc;
  *avg_ms_host = ms / n_iter;
  return GDM_OK;
  GDM_GUARD_END
}

// ---- cut-cell systems (host assembly in gdm_cut.cpp) ----------------------
struct gdm_cut_system;
int gdmh_cut_poisson_create(int p, int n_sub, double lo, double hi, const double *center, double radius,
                            int ghost_penalty, double rhs_value, double bc_value, gdm_cut_system **out, char *err,
                            size_t err_len);
void gdmh_cut_info(const gdm_cut_system *S, int64_t *n_rows, int64_t *nnz, int64_t *n_inside, int64_t *n_intersected);
void gdmh_cut_arrays(const gdm_cut_system *S, const int64_t **row_ptr, const uint32_t **cols, const double **vals,
                     const double **rhs);
double gdmh_cut_l2_error(const gdm_cut_system *S, const double *u);
void gdmh_cut_destroy(gdm_cut_system *S);

int gdm_cut_poisson_create(int p, int n_sub, double lo, double hi, const double *center, double radius,
                           int ghost_penalty, double rhs_value, double bc_value, gdm_cut_system **out) {
  if (!out) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  char err[256] = {0};
  if (gdmh_cut_poisson_create(p, n_sub, lo, hi, center, radius, ghost_penalty, rhs_value, bc_value, out, err,
                              sizeof(err)) != 0)
    return fail(std::strstr(err, "not implemented") ? GDM_ERR_UNSUPPORTED : GDM_ERR_ARG, err);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_poisson_info(const gdm_cut_system *S, int64_t *n_rows, int64_t *nnz, int64_t *n_inside_cells,
                         int64_t *n_intersected_cells) {
  if (!S || !n_rows || !nnz || !n_inside_cells || !n_intersected_cells) return fail(GDM_ERR_ARG, "NULL argument");
  gdmh_cut_info(S, n_rows, nnz, n_inside_cells, n_intersected_cells);
  return GDM_OK;
}

int gdm_cut_poisson_matrix(const gdm_cut_system *S, int device, gdm_csr **A) {
  if (!S || !A) return fail(GDM_ERR_ARG, "NULL argument");
  int64_t n, nnz, a, b;
  gdmh_cut_info(S, &n, &nnz, &a, &b);
  const int64_t *rp;
  const uint32_t *ci;
  const double *v, *r;
  gdmh_cut_arrays(S, &rp, &ci, &v, &r);
  return gdm_csr_create(device, n, n, nnz, rp, ci, v, 0, A);
}

int gdm_cut_poisson_csr(const gdm_cut_system *S, int64_t *row_ptr_host, uint32_t *cols_host, double *vals_host) {
  if (!S || !row_ptr_host || !cols_host || !vals_host) return fail(GDM_ERR_ARG, "NULL argument");
  int64_t n, nnz, a, b;
  gdmh_cut_info(S, &n, &nnz, &a, &b);
  const int64_t *rp;
  const uint32_t *ci;
  const double *v, *r;
  gdmh_cut_arrays(S, &rp, &ci, &v, &r);
  std::memcpy(row_ptr_host, rp, sizeof(int64_t) * (n + 1));
  std::memcpy(cols_host, ci, sizeof(uint32_t) * nnz);
  std::memcpy(vals_host, v, sizeof(double) * nnz);
  return GDM_OK;
}

int gdm_cut_poisson_rhs(const gdm_cut_system *S, double *rhs_host) {
  if (!S || !rhs_host) return fail(GDM_ERR_ARG, "NULL argument");
  int64_t n, nnz, a, b;
  gdmh_cut_info(S, &n, &nnz, &a, &b);
  const int64_t *rp;
  const uint32_t *ci;
  const double *v, *r;
  gdmh_cut_arrays(S, &rp, &ci, &v, &r);
  std::memcpy(rhs_host, r, sizeof(double) * n);
  return GDM_OK;
}

int gdm_cut_poisson_solve(const gdm_cut_system *S, gdm_csr *A, double rel_tol, double abs_tol, int max_it,
                          double *u_host, int *its_host, double *res_host) {
  if (!S || !A || !u_host) return fail(GDM_ERR_ARG, "NULL argument");
  int64_t n, nnz, a, b, m, mc, mz;
  gdmh_cut_info(S, &n, &nnz, &a, &b);
  if (gdm_csr_info(A, &m, &mc, &mz) != GDM_OK || m != n || mc != n) return fail(GDM_ERR_ARG, "matrix does not match the system");
  GDM_GUARD_BEGIN
  const int64_t *rp;
  const uint32_t *ci;
  const double *v, *r;
  gdmh_cut_arrays(S, &rp, &ci, &v, &r);
  double *bd = nullptr, *xd = nullptr;
  hip_check(hipMalloc(&bd, sizeof(double) * std::max<int64_t>(n, 1)), "hipMalloc rhs");
  if (hipMalloc(&xd, sizeof(double) * std::max<int64_t>(n, 1)) != hipSuccess) {
    (void)hipFree(bd);
    throw HipError("hipMalloc solution");
  }
  int rc = GDM_OK;
  try {
    hip_check(hipMemcpy(bd, r, sizeof(double) * n, hipMemcpyHostToDevice), "h2d rhs");
    hip_check(hipMemset(xd, 0, sizeof(double) * n), "memset");
    hip_check(hipDeviceSynchronize(), "sync");
    rc = gdm_csr_cg(A, bd, xd, 0, max_it, abs_tol, rel_tol, its_host, res_host);
    hip_check(hipDeviceSynchronize(), "sync");
    hip_check(hipMemcpy(u_host, xd, sizeof(double) * n, hipMemcpyDeviceToHost), "d2h solution");
  } catch (...) {
    (void)hipFree(bd);
    (void)hipFree(xd);
    throw;
  }
  (void)hipFree(bd);
  (void)hipFree(xd);
  return rc;
  GDM_GUARD_END
}

int gdm_cut_poisson_l2_error(const gdm_cut_system *S, const double *u_host, double *err) {
  if (!S || !u_host || !err) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  *err = gdmh_cut_l2_error(S, u_host);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_poisson_destroy(gdm_cut_system *S) {
  gdmh_cut_destroy(S);
  return GDM_OK;
}

// ---------------------------------------------------------------------------
// Cut-cell advection (include/gdm_hip.h): host assembly of the corrections
// (gdm_cut_advection.cpp), the uncut stencil of the box, device CSR products
// and the banded mass solve (gdm_band.hip).
// ---------------------------------------------------------------------------
struct gdm_cut_adv_system;
int gdmh_cut_adv_create(int p, int n_sub, double lo, double hi, const double *level_set, const double *advection,
                        double gamma_A, double gamma_M, int composite, gdm_cut_adv_system **out, char *err,
                        size_t err_len);
void gdmh_cut_adv_coupling(const gdm_cut_adv_system *S, const int64_t **rp, const uint32_t **ci, const double **v,
                           int64_t *nnz);
void gdmh_cut_adv_info(const gdm_cut_adv_system *S, int64_t *n_dofs, int64_t *n_bc, int64_t *cells,
                       int64_t *bandwidth);
void gdmh_cut_adv_arrays(const gdm_cut_adv_system *S, const int64_t **c_rp, const uint32_t **c_ci,
                         const double **c_v, const int64_t **f_rp, const uint32_t **f_ci, const double **f_v,
                         const double **bc_xy, const double **lband);
void gdmh_cut_adv_zero_rows(const gdm_cut_adv_system *S, const int64_t **rows, int64_t *n);
void gdmh_cut_adv_destroy(gdm_cut_adv_system *S);
hipError_t gdmk_launch_zero_rows(int64_t n, const int64_t *rows, double *y, hipStream_t st);
hipError_t gdmk_launch_csr_accum(int64_t n_rows, const int64_t *rp, const uint32_t *ci, const double *v,
                                 const double *x, double *y, hipStream_t st);
hipError_t gdmk_launch_band_solve(int64_t n, int64_t bw, const double *L, double *x, hipStream_t st);

}  // extern "C"

struct gdm_cut_advection {
  gdm_cut_adv_system *host = nullptr;
  gdm_op *op = nullptr;
  int64_t n_dofs = 0, n_bc = 0, bw = 0, cells[3] = {0, 0, 0};
  int64_t *c_rp = nullptr, *f_rp = nullptr, *zrows = nullptr, n_zrows = 0;
  uint32_t *c_ci = nullptr, *f_ci = nullptr;
  double *c_v = nullptr, *f_v = nullptr, *lband = nullptr;
  int composite = 0;  // GDM_CUT_ADV_COMPOSITE: (II)'s inflow couples to the partner field (p_*)
  int64_t *p_rp = nullptr;
  uint32_t *p_ci = nullptr;
  double *p_v = nullptr;
  std::vector<double> bc_xy;
  void release() {
    for (void *q : {(void *)c_rp, (void *)f_rp, (void *)c_ci, (void *)f_ci, (void *)c_v, (void *)f_v, (void *)lband,
                    (void *)zrows, (void *)p_rp, (void *)p_ci, (void *)p_v})
      if (q) (void)hipFree(q);
    p_rp = nullptr;
    p_ci = nullptr;
    p_v = nullptr;
    zrows = nullptr;
    c_rp = f_rp = nullptr;
    c_ci = f_ci = nullptr;
    c_v = f_v = lband = nullptr;
    if (op) gdm_op_destroy(op);
    op = nullptr;
    if (host) gdmh_cut_adv_destroy(host);
    host = nullptr;
  }
};

extern "C" {

int gdm_cut_advection_create(int fe_degree, int n_subdivisions, double left, double right, const double *level_set,
                             const double *advection, double ghost_parameter_A, double ghost_parameter_M,
                             int device, gdm_cut_advection **out) {
  return gdm_cut_advection_create2(fe_degree, n_subdivisions, left, right, level_set, advection, ghost_parameter_A,
                                   ghost_parameter_M, GDM_CUT_INSIDE, 0, device, out);
}

int gdm_cut_advection_create2(int fe_degree, int n_subdivisions, double left, double right, const double *level_set,
                              const double *advection, double ghost_parameter_A, double ghost_parameter_M,
                              int location, int flags, int device, gdm_cut_advection **out) {
  if (!out || !level_set || !advection) return fail(GDM_ERR_ARG, "NULL argument");
  *out = nullptr;
  if (location != GDM_CUT_INSIDE && location != GDM_CUT_OUTSIDE)
    return fail(GDM_ERR_ARG, "location: GDM_CUT_INSIDE or GDM_CUT_OUTSIDE");
  if (flags & ~GDM_CUT_ADV_COMPOSITE) return fail(GDM_ERR_ARG, "flags: GDM_CUT_ADV_COMPOSITE only");
  GDM_GUARD_BEGIN
  auto *c = new gdm_cut_advection();
  try {
    char err[256] = {0};
    // the outside field = the same assembly on the negated level set (its inside is the outside region;
    // MeshClassifier, face parts, surface normal and ghost-penalty faces follow the sign)
    const size_t nv = n_subdivisions >= 0 ? (size_t)(n_subdivisions + 1) * (size_t)(n_subdivisions + 1) : 0;
    std::vector<double> ls(level_set, level_set + nv);
    if (location == GDM_CUT_OUTSIDE)
      for (double &v : ls) v = -v;
    c->composite = (flags & GDM_CUT_ADV_COMPOSITE) != 0;
    if (gdmh_cut_adv_create(fe_degree, n_subdivisions, left, right, ls.data(), advection, ghost_parameter_A,
                            ghost_parameter_M, c->composite, &c->host, err, sizeof(err)) != 0) {
      delete c;
      return fail(GDM_ERR_ARG, err);
    }
    // the uncut box operator S: 2D advection with the same a (stencil + outflow traces)
    gdm_mesh_desc m{};
    m.dim = 2;
    m.fe_degree = fe_degree;
    m.n_subdivisions[0] = m.n_subdivisions[1] = n_subdivisions;
    m.n_subdivisions[2] = 1;
    m.lo[0] = m.lo[1] = left;
    m.hi[0] = m.hi[1] = right;
    m.hi[2] = 1.0;
    m.n_ranks = 1;
    m.rank = 0;
    const int rc = gdm_op_create(&m, GDM_OP_ADVECTION, advection, 2, device, &c->op);
    if (rc != GDM_OK) {
      c->release();
      delete c;
      return rc;
    }
    gdmh_cut_adv_info(c->host, &c->n_dofs, &c->n_bc, c->cells, &c->bw);
    const int64_t *crp, *frp;
    const uint32_t *cci, *fci;
    const double *cv, *fv, *xy, *lb;
    gdmh_cut_adv_arrays(c->host, &crp, &cci, &cv, &frp, &fci, &fv, &xy, &lb);
    const int64_t N = c->n_dofs;
    hip_check(hipSetDevice(device), "hipSetDevice");
    c->c_rp = dev_upload(std::vector<int64_t>(crp, crp + N + 1));
    c->c_ci = dev_upload(std::vector<uint32_t>(cci, cci + crp[N]));
    c->c_v = dev_upload(std::vector<double>(cv, cv + crp[N]));
    c->f_rp = dev_upload(std::vector<int64_t>(frp, frp + N + 1));
    c->f_ci = dev_upload(std::vector<uint32_t>(fci, fci + frp[N]));
    c->f_v = dev_upload(std::vector<double>(fv, fv + frp[N]));
    c->lband = dev_upload(std::vector<double>(lb, lb + N * (c->bw + 1)));
    const int64_t *zr;
    gdmh_cut_adv_zero_rows(c->host, &zr, &c->n_zrows);
    if (c->n_zrows > 0) c->zrows = dev_upload(std::vector<int64_t>(zr, zr + c->n_zrows));
    c->bc_xy.assign(xy, xy + 2 * c->n_bc);
    if (c->composite) {
      const int64_t *prp;
      const uint32_t *pci;
      const double *pv;
      int64_t pnnz = 0;
      gdmh_cut_adv_coupling(c->host, &prp, &pci, &pv, &pnnz);
      // (a field the flow only leaves through the surface has no coupling entries: pci / pv may be NULL)
      std::vector<uint32_t> ci(std::max<int64_t>(pnnz, 1), 0u);
      std::vector<double> cv(std::max<int64_t>(pnnz, 1), 0.0);
      if (pnnz > 0) {
        std::copy(pci, pci + pnnz, ci.begin());
        std::copy(pv, pv + pnnz, cv.begin());
      }
      c->p_rp = dev_upload(std::vector<int64_t>(prp, prp + N + 1));
      c->p_ci = dev_upload(ci);
      c->p_v = dev_upload(cv);
    }
  } catch (...) {
    c->release();
    delete c;
    throw;
  }
  *out = c;
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_advection_info(const gdm_cut_advection *c, int64_t *n_dofs, int64_t *n_bc_points, int64_t *cells,
                           int64_t *mass_bandwidth) {
  if (!c || !n_dofs || !n_bc_points || !cells || !mass_bandwidth) return fail(GDM_ERR_ARG, "NULL argument");
  *n_dofs = c->n_dofs;
  *n_bc_points = c->n_bc;
  for (int k = 0; k < 3; ++k) cells[k] = c->cells[k];
  *mass_bandwidth = c->bw;
  return GDM_OK;
}

int gdm_cut_advection_bc_points(const gdm_cut_advection *c, double *xy_host) {
  if (!c || (c->n_bc > 0 && !xy_host)) return fail(GDM_ERR_ARG, "NULL argument");
  std::copy(c->bc_xy.begin(), c->bc_xy.end(), xy_host);
  return GDM_OK;
}

int gdm_cut_advection_op(gdm_cut_advection *c, gdm_op **op) {
  if (!c || !op) return fail(GDM_ERR_ARG, "NULL argument");
  *op = c->op;
  return GDM_OK;
}

int gdm_cut_advection_compute_rhs(gdm_cut_advection *c, const double *u, const double *bc, double *rhs) {
  if (!c || !u || !rhs || (c->n_bc > 0 && !bc)) return fail(GDM_ERR_ARG, "NULL argument");
  if (u == rhs) return fail(GDM_ERR_ARG, "u and rhs must be distinct");
  const int rc = gdm_apply(c->op, u, rhs, nullptr);  // S u (no inflow data)
  if (rc != GDM_OK) return rc;
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  hip_check(gdmk_launch_zero_rows(c->n_zrows, c->zrows, rhs, c->op->stream), "cut rows");
  hip_check(gdmk_launch_csr_accum(c->n_dofs, c->c_rp, c->c_ci, c->c_v, u, rhs, c->op->stream), "cut correction");
  if (c->n_bc > 0)
    hip_check(gdmk_launch_csr_accum(c->n_dofs, c->f_rp, c->f_ci, c->f_v, bc, rhs, c->op->stream), "inflow data");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_advection_couple(gdm_cut_advection *c, const double *u_partner, double *rhs) {
  if (!c || !u_partner || !rhs) return fail(GDM_ERR_ARG, "NULL argument");
  if (!c->composite) return fail(GDM_ERR_STATE, "gdm_cut_advection_couple: created without GDM_CUT_ADV_COMPOSITE");
  if (u_partner == rhs) return fail(GDM_ERR_ARG, "u_partner and rhs must be distinct");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  hip_check(gdmk_launch_csr_accum(c->n_dofs, c->p_rp, c->p_ci, c->p_v, u_partner, rhs, c->op->stream), "coupling");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_advection_mass_solve(gdm_cut_advection *c, const double *rhs, double *x) {
  if (!c || !rhs || !x) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  if (x != rhs)
    hip_check(hipMemcpyAsync(x, rhs, sizeof(double) * c->n_dofs, hipMemcpyDeviceToDevice, c->op->stream), "copy");
  hip_check(gdmk_launch_band_solve(c->n_dofs, c->bw, c->lband, x, c->op->stream), "band solve");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_advection_destroy(gdm_cut_advection *c) {
  if (!c) return GDM_OK;
  c->release();
  delete c;
  return GDM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Cut-cell wave / heat (1D and 2D; host assembly csrc/gdm_cut_wave.cpp)
// ---------------------------------------------------------------------------
struct gdm_cut_wave_system;
extern "C" {
int gdmh_cut_wave_create(int dim, int p, int n_sub, double lo, double hi, int ls_degree, const double *ls_values,
                         int location, int flags, double gamma_M, double gamma_A, double nitsche,
                         gdm_cut_wave_system **out, char *err, size_t err_len);
void gdmh_cut_wave_info(const gdm_cut_wave_system *S, int64_t *n_dofs, int64_t *n_quad, int64_t *n_surface,
                        int64_t *cells);
void gdmh_cut_wave_csr(const gdm_cut_wave_system *S, int which, const int64_t **rp, const uint32_t **ci,
                       const double **v);
void gdmh_cut_wave_points(const gdm_cut_wave_system *S, const double **qx, const double **qw, const double **sx,
                          const double **sn, const int64_t **zero_rows, int64_t *n_zero);
void gdmh_cut_wave_destroy(gdm_cut_wave_system *S);
int gdmh_cut_wave_splits(const gdm_cut_wave_system *S);
int64_t gdmh_band_cholesky(int64_t n, const int64_t *rp, const uint32_t *ci, const double *v, double alpha,
                           const int64_t *rp2, const uint32_t *ci2, const double *v2, std::vector<double> &lband);
}

// message for a failed gdmh_band_cholesky (-1: not positive definite, -2: too large)
static std::string band_error(int64_t code, const char *what) {
  return std::string("cut wave: ") + what +
         (code == -2 ? ": banded factor larger than 2^28 entries (mesh too large for the dense-band solve)"
                     : " not positive definite");
}


namespace {
struct DevCsr {
  int64_t rows = 0;
  int64_t *rp = nullptr;
  uint32_t *ci = nullptr;
  double *v = nullptr;
  void upload(const gdm_cut_wave_system *S, int which, int64_t n_rows) {
    const int64_t *hrp;
    const uint32_t *hci;
    const double *hv;
    gdmh_cut_wave_csr(S, which, &hrp, &hci, &hv);
    rows = n_rows;
    rp = dev_upload(std::vector<int64_t>(hrp, hrp + n_rows + 1));
    const int64_t nnz = hrp[n_rows];
    std::vector<uint32_t> c1(std::max<int64_t>(nnz, 1), 0);  // one padding entry for an empty matrix
    std::vector<double> v1(c1.size(), 0.0);
    if (nnz > 0) {
      std::copy(hci, hci + nnz, c1.begin());
      std::copy(hv, hv + nnz, v1.begin());
    }
    ci = dev_upload(c1);
    v = dev_upload(v1);
  }
  void release() {
    for (void *q : {(void *)rp, (void *)ci, (void *)v})
      if (q) (void)hipFree(q);
    rp = nullptr;
    ci = nullptr;
    v = nullptr;
  }
  void accum(const double *x, double *y, hipStream_t st) const {
    hip_check(gdmk_launch_csr_accum(rows, rp, ci, v, x, y, st), "csr accumulate");
  }
};
}  // namespace

struct gdm_cut_wave {
  gdm_cut_wave_system *host = nullptr;
  gdm_op *op = nullptr;
  int dim = 1;
  int64_t n_dofs = 0, n_quad = 0, n_surf = 0, cells[3] = {0, 0, 0};
  DevCsr C, Ff, Fg, E, M, X;
  bool coupled = false;
  int64_t *zrows = nullptr, n_zrows = 0;
  int64_t bw_m = -1, bw_a = -1, bw_k = -1;  // -1: no factor (no mass matrix when gamma_M < 0)
  double *lband_m = nullptr, *lband_a = nullptr, *lband_k = nullptr, dt_a = 0.0;
  void release() {
    for (DevCsr *q : {&C, &Ff, &Fg, &E, &M, &X}) q->release();
    for (void *q : {(void *)zrows, (void *)lband_m, (void *)lband_a, (void *)lband_k})
      if (q) (void)hipFree(q);
    zrows = nullptr;
    lband_m = lband_a = lband_k = nullptr;
    if (op) gdm_op_destroy(op);
    op = nullptr;
    if (host) gdmh_cut_wave_destroy(host);
    host = nullptr;
  }
};

extern "C" {

int gdm_cut_wave_create(int dim, int fe_degree, int n_subdivisions, double left, double right, int ls_degree,
                        const double *ls_values, int location, int flags, double gamma_M, double gamma_A,
                        double nitsche, int device, gdm_cut_wave **out) {
  if (!out || !ls_values) return fail(GDM_ERR_ARG, "NULL argument");
  *out = nullptr;
  GDM_GUARD_BEGIN
  auto *c = new gdm_cut_wave();
  try {
    char err[256] = {0};
    if (gdmh_cut_wave_create(dim, fe_degree, n_subdivisions, left, right, ls_degree, ls_values, location, flags,
                             gamma_M, gamma_A, nitsche, &c->host, err, sizeof(err)) != 0) {
      delete c;
      return fail(GDM_ERR_ARG, err);
    }
    // the uncut box operator S: wave -(grad v, grad u) of the box (no box Nitsche)
    c->dim = dim;
    gdm_mesh_desc m{};
    m.dim = dim;
    m.fe_degree = fe_degree;
    for (int d = 0; d < 3; ++d) {
      m.n_subdivisions[d] = d < dim ? n_subdivisions : 1;
      m.lo[d] = d < dim ? left : 0.0;
      m.hi[d] = d < dim ? right : 1.0;
    }
    m.n_ranks = 1;
    m.rank = 0;
    const int rc = gdm_op_create(&m, GDM_OP_WAVE, nullptr, 0, device, &c->op);
    if (rc != GDM_OK) {
      c->release();
      delete c;
      return rc;
    }
    gdmh_cut_wave_info(c->host, &c->n_dofs, &c->n_quad, &c->n_surf, c->cells);
    gdm_layout L{};
    if (gdm_op_layout(c->op, &L) != GDM_OK || L.n_local != c->n_dofs || L.n_owned != c->n_dofs)
      throw std::runtime_error("cut wave: the box operator's layout is not the cut system's DoF range");
    hip_check(hipSetDevice(device), "hipSetDevice");
    c->C.upload(c->host, 0, c->n_dofs);
    c->Ff.upload(c->host, 1, c->n_dofs);
    c->Fg.upload(c->host, 2, c->n_dofs);
    c->E.upload(c->host, 3, c->n_quad);
    c->M.upload(c->host, 4, c->n_dofs);
    c->coupled = (flags & GDM_CUT_WAVE_COUPLED) != 0;
    if (c->coupled) c->X.upload(c->host, 6, c->n_dofs);
    const double *qx, *qw, *sx, *sn;
    const int64_t *zr;
    gdmh_cut_wave_points(c->host, &qx, &qw, &sx, &sn, &zr, &c->n_zrows);
    if (c->n_zrows > 0) c->zrows = dev_upload(std::vector<int64_t>(zr, zr + c->n_zrows));
    const int64_t *rp;
    const uint32_t *ci;
    const double *v;
    if (gamma_M >= 0.0) {
      gdmh_cut_wave_csr(c->host, 4, &rp, &ci, &v);
      std::vector<double> lb;
      c->bw_m = gdmh_band_cholesky(c->n_dofs, rp, ci, v, 0.0, nullptr, nullptr, nullptr, lb);
      if (c->bw_m < 0) throw std::runtime_error(band_error(c->bw_m, "mass matrix"));
      c->lband_m = dev_upload(lb);
    }
  } catch (...) {
    c->release();
    delete c;
    throw;
  }
  *out = c;
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_info(const gdm_cut_wave *c, int64_t *n_dofs, int64_t *n_quad, int64_t *n_surface, int64_t *cells) {
  if (!c || !n_dofs || !n_quad || !n_surface || !cells) return fail(GDM_ERR_ARG, "NULL argument");
  *n_dofs = c->n_dofs;
  *n_quad = c->n_quad;
  *n_surface = c->n_surf;
  for (int k = 0; k < 3; ++k) cells[k] = c->cells[k];
  return GDM_OK;
}

int gdm_cut_wave_points(const gdm_cut_wave *c, double *qx, double *qw, double *sx, double *sn) {
  if (!c) return fail(GDM_ERR_ARG, "NULL argument");
  const double *hqx, *hqw, *hsx, *hsn;
  const int64_t *zr;
  int64_t nz;
  gdmh_cut_wave_points(c->host, &hqx, &hqw, &hsx, &hsn, &zr, &nz);
  if (qx) std::copy(hqx, hqx + c->n_quad * c->dim, qx);
  if (qw) std::copy(hqw, hqw + c->n_quad, qw);
  if (sx) std::copy(hsx, hsx + c->n_surf * c->dim, sx);
  if (sn) std::copy(hsn, hsn + c->n_surf * c->dim, sn);
  return GDM_OK;
}

int gdm_cut_wave_op(gdm_cut_wave *c, gdm_op **op) {
  if (!c || !op) return fail(GDM_ERR_ARG, "NULL argument");
  *op = c->op;
  return GDM_OK;
}

int gdm_cut_wave_compute_rhs(gdm_cut_wave *c, const double *u, const double *fq, const double *gs, double *rhs) {
  if (!c || !rhs) return fail(GDM_ERR_ARG, "NULL argument");
  if (u == rhs) return fail(GDM_ERR_ARG, "u and rhs must be distinct");
  if (u) {
    const int rc = gdm_apply(c->op, u, rhs, nullptr);  // S u
    if (rc != GDM_OK) return rc;
  }
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  hipStream_t st = c->op->stream;
  if (u) {
    hip_check(gdmk_launch_zero_rows(c->n_zrows, c->zrows, rhs, st), "cut rows");
    c->C.accum(u, rhs, st);
  } else {
    hip_check(gdmk_launch_zero(c->n_dofs, rhs, st), "zero");
  }
  if (fq && c->n_quad > 0) c->Ff.accum(fq, rhs, st);
  if (gs && c->n_surf > 0) c->Fg.accum(gs, rhs, st);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_couple(gdm_cut_wave *c, const double *u_other, double *rhs) {
  if (!c || !u_other || !rhs) return fail(GDM_ERR_ARG, "NULL argument");
  if (!c->coupled) return fail(GDM_ERR_ARG, "gdm_cut_wave_couple: created without GDM_CUT_WAVE_COUPLED");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  c->X.accum(u_other, rhs, c->op->stream);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_mass_apply(gdm_cut_wave *c, const double *u, double *out) {
  if (!c || !u || !out || u == out) return fail(GDM_ERR_ARG, "NULL or aliased argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  hip_check(gdmk_launch_zero(c->n_dofs, out, c->op->stream), "zero");
  c->M.accum(u, out, c->op->stream);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_mass_solve(gdm_cut_wave *c, const double *rhs, double *x) {
  if (!c || !rhs || !x) return fail(GDM_ERR_ARG, "NULL argument");
  if (c->bw_m < 0) return fail(GDM_ERR_ARG, "gdm_cut_wave_mass_solve: no mass matrix (gamma_M < 0)");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  if (x != rhs)
    hip_check(hipMemcpyAsync(x, rhs, sizeof(double) * c->n_dofs, hipMemcpyDeviceToDevice, c->op->stream), "copy");
  hip_check(gdmk_launch_band_solve(c->n_dofs, c->bw_m, c->lband_m, x, c->op->stream), "band solve");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_system_solve(gdm_cut_wave *c, double dt, const double *rhs, double *x) {
  if (!c || !rhs || !x) return fail(GDM_ERR_ARG, "NULL argument");
  if (!(dt > 0.0)) return fail(GDM_ERR_ARG, "gdm_cut_wave_system_solve: dt must be positive");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  if (c->bw_a < 0 || dt != c->dt_a) {
    const int64_t *rp, *rp2;
    const uint32_t *ci, *ci2;
    const double *v, *v2;
    gdmh_cut_wave_csr(c->host, 4, &rp, &ci, &v);
    gdmh_cut_wave_csr(c->host, 5, &rp2, &ci2, &v2);
    std::vector<double> lb;
    const int64_t bw = gdmh_band_cholesky(c->n_dofs, rp, ci, v, dt, rp2, ci2, v2, lb);
    if (bw < 0) throw std::runtime_error(band_error(bw, "M + dt K"));
    // the previous factor may still be read by queued solves
    hip_check(hipStreamSynchronize(c->op->stream), "hipStreamSynchronize");
    if (c->lband_a) (void)hipFree(c->lband_a);
    c->lband_a = dev_upload(lb);
    c->bw_a = bw;
    c->dt_a = dt;
  }
  if (x != rhs)
    hip_check(hipMemcpyAsync(x, rhs, sizeof(double) * c->n_dofs, hipMemcpyDeviceToDevice, c->op->stream), "copy");
  hip_check(gdmk_launch_band_solve(c->n_dofs, c->bw_a, c->lband_a, x, c->op->stream), "band solve");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_stiffness_solve(gdm_cut_wave *c, const double *rhs, double *x) {
  if (!c || !rhs || !x) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  if (c->bw_k < 0) {
    const int64_t *rp;
    const uint32_t *ci;
    const double *v;
    gdmh_cut_wave_csr(c->host, 5, &rp, &ci, &v);
    std::vector<double> lb;
    const int64_t bw = gdmh_band_cholesky(c->n_dofs, rp, ci, v, 0.0, nullptr, nullptr, nullptr, lb);
    if (bw < 0) throw std::runtime_error(band_error(bw, "stiffness matrix"));
    c->lband_k = dev_upload(lb);
    c->bw_k = bw;
  }
  if (x != rhs)
    hip_check(hipMemcpyAsync(x, rhs, sizeof(double) * c->n_dofs, hipMemcpyDeviceToDevice, c->op->stream), "copy");
  hip_check(gdmk_launch_band_solve(c->n_dofs, c->bw_k, c->lband_k, x, c->op->stream), "band solve");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_eval(gdm_cut_wave *c, const double *u, double *vals) {
  if (!c || !u || !vals) return fail(GDM_ERR_ARG, "NULL argument");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(c->op->device), "hipSetDevice");
  hip_check(gdmk_launch_zero(c->n_quad, vals, c->op->stream), "zero");
  c->E.accum(u, vals, c->op->stream);
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_cut_wave_destroy(gdm_cut_wave *c) {
  if (!c) return GDM_OK;
  c->release();
  delete c;
  return GDM_OK;
}

}  // extern "C"
