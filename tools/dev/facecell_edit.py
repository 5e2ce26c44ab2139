R = '/root/repo/dealii-galerkin-difference-methods_amd/csrc/'
h = open(R + 'gdm_kernels.h').read()
old = "  double *T;  // scratch Q1 x (i0_end - i0_begin)"
new = """  // cell form of step 1 (t0 non-trivial and its local cells fit LDS): Phi0 =
  // [category][l][q] values phi_l(x_q) w_q h of t0, crange0[2 i] / [2 i + 1] =
  // first / last local cell of node i
  const double *phi0;
  const int *crange0;
  int p, ncell0_total, cell0_begin;
  double *T;  // scratch Q1 x (i0_end - i0_begin)"""
assert old in h; h = h.replace(old, new)
open(R + 'gdm_kernels.h', 'w').write(h)

k = open(R + 'gdm_kernels.hip').read()
anchor = "// dst(i0, i1) += scale"
if anchor not in k:
    anchor = "__global__ void __launch_bounds__(256) face_step2_kernel("
new_kernel = '''// Step 1 in cell form: for one row q1 of the face, every local cell c reduces
// its p + 1 contiguous boundary values with its category's (p+1) x (p+1) table
// (S_c[l] = sum_q Phi[cat(c)][l][q] U[q1][c (p+1) + q], one contiguous read per
// cell, no per-node weight rows), then every owned node gathers the S_c of the
// cells whose DoF boxes contain it (system.h:195-246 box offsets).
__device__ __forceinline__ int face_category(int c, int p, int n) {
  const int half = p / 2;
  return c < half ? c : (c < n - half ? half : p + c - n);
}
__device__ __forceinline__ int face_box_offset(int c, int p, int n) {
  const int half = p / 2;
  return c < half ? 0 : min(n, c + half + 1) - p;
}

template <int P>
__global__ void __launch_bounds__(512) face_cell_step1_kernel(const double *__restrict__ U, int Q0, int Q1, int rpb,
                                                               int i0_begin, int n0, const int *__restrict__ crange,
                                                               const double *__restrict__ phi, int ncell_total,
                                                               int cell_begin, double *__restrict__ T) {
  constexpr int N1 = P + 1;
  extern __shared__ double sh[];  // [P][N1][N1] Phi, then [ncells][N1] S
  double *sphi = sh, *S = sh + P * N1 * N1;
  const int ncells = Q0 / N1;
  for (int e = threadIdx.x; e < P * N1 * N1; e += blockDim.x) sphi[e] = phi[e];
  const int r0 = blockIdx.x * rpb, r1 = min(Q1, r0 + rpb);
  for (int row = r0; row < r1; ++row) {
    __syncthreads();  // Phi ready / previous row's gather done
    const double *u = U + (int64_t)row * Q0;
    for (int c = threadIdx.x; c < ncells; c += blockDim.x) {
      const int cat = face_category(cell_begin + c, P, ncell_total);
      double v[N1];
#pragma unroll
      for (int q = 0; q < N1; ++q) v[q] = u[c * N1 + q];
      const double *ph = sphi + cat * N1 * N1;
#pragma unroll
      for (int l = 0; l < N1; ++l) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < N1; ++q) s = fma(ph[l * N1 + q], v[q], s);
        S[c * N1 + l] = s;
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n0; t += blockDim.x) {
      const int i0 = i0_begin + t;
      const int cf = crange[2 * i0], cl = crange[2 * i0 + 1];
      double acc = 0.0;
      for (int c = cf; c <= cl; ++c) acc += S[c * N1 + (i0 - face_box_offset(cell_begin + c, P, ncell_total))];
      T[(int64_t)row * n0 + t] = acc;
    }
  }
}

'''
k = k.replace(anchor, new_kernel + anchor, 1)
old = """  const int n0 = f.i0_end - f.i0_begin;
  if (n0 <= 0 || f.Q1 <= 0 || f.i1_end <= f.i1_begin) return hipSuccess;"""
new = """  const int n0 = f.i0_end - f.i0_begin;
  if (n0 <= 0 || f.Q1 <= 0 || f.i1_end <= f.i1_begin) return hipSuccess;
  const size_t cell_lds = sizeof(double) * ((size_t)f.p * (f.p + 1) * (f.p + 1) + (size_t)f.Q0);
  if (f.phi0 && cell_lds <= 48 * 1024 && !std::getenv("GDM_FACE_NODE")) {
    // cell form of step 1, then the usual step 2
    const int rpb = 4;
    dim3 g1c((f.Q1 + rpb - 1) / rpb);
    switch (f.p) {
#define GDM_FACE_CELL(PP)                                                                                            \\
  case PP:                                                                                                         \\
    hipLaunchKernelGGL(face_cell_step1_kernel<PP>, g1c, dim3(512), cell_lds, st, f.U, f.Q0, f.Q1, rpb, f.i0_begin, \\
                       n0, f.crange0, f.phi0, f.ncell0_total, f.cell0_begin, f.T);                                 \\
    break;
      GDM_FACE_CELL(1) GDM_FACE_CELL(3) GDM_FACE_CELL(5) GDM_FACE_CELL(7) GDM_FACE_CELL(9)
#undef GDM_FACE_CELL
      default: return hipErrorInvalidValue;
    }
    dim3 g2((n0 + 255) / 256, f.i1_end - f.i1_begin);
    hipLaunchKernelGGL(face_step2_kernel, g2, dim3(256), 0, st, f.T, n0, f.i1_begin, f.i1_end, f.qs1, f.qc1, f.w1,
                       f.wmax1, f.dst, f.base, f.stride0, f.stride1, f.scale);
    return hipGetLastError();
  }"""
assert old in k; k = k.replace(old, new)
open(R + 'gdm_kernels.hip', 'w').write(k)

c = open(R + 'gdm_capi.cpp').read()
old = """  double *w = nullptr;    // [n_nodes][wmax]
  double *wT = nullptr;   // [wmax][n_nodes]
};"""
new = """  double *w = nullptr;    // [n_nodes][wmax]
  double *wT = nullptr;   // [wmax][n_nodes]
  double *phi = nullptr;  // [p][p+1][p+1] cell tables (cell form of the face step 1)
  int *crange = nullptr;  // [n_nodes][2] first / last local cell of each node
  int ncell_total = 0;
};"""
assert old in c; c = c.replace(old, new)
old = """      t.qs = keep(op, dev_upload(ft.qstart));
      t.qc = keep(op, dev_upload(ft.qcount));
      t.w = keep(op, dev_upload(ft.w));"""
new = """      t.qs = keep(op, dev_upload(ft.qstart));
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
      }"""
assert old in c; c = c.replace(old, new)
old = """      fa.T = op->face_tmp;
      fa.dst = dst_owned;"""
new = """      fa.phi0 = F.t0.phi;
      fa.crange0 = F.t0.crange;
      fa.p = op->p;
      fa.ncell0_total = F.t0.ncell_total;
      fa.cell0_begin = F.t0.cell_begin;
      fa.T = op->face_tmp;
      fa.dst = dst_owned;"""
assert old in c; c = c.replace(old, new)
open(R + 'gdm_capi.cpp', 'w').write(c)
print("ok")
