s = open('gdm_kernels.hip').read()
i = s.index("template <int ROWS>\n__global__ void __launch_bounds__(FACE_CHUNK) face_step1_kernel(")
j = s.index("// ---------------------------------------------------------------------------\n// BLAS-1")
s = s[:i] + '''template <int ROWS>
__global__ void __launch_bounds__(FACE_THREADS) face_step1_kernel(const double *__restrict__ U, int Q0, int Q1,
                                                                   int i0_begin, int n0,
                                                                   const int *__restrict__ qs0,
                                                                   const double *__restrict__ w0T, int wmax0,
                                                                   int ldw0, int qmax, double *__restrict__ T) {
  // block: FACE_CHUNK nodes x ROWS rows of U; thread (node t, slice s) owns
  // rows s, s + NS, ... of its node
  constexpr int NS = FACE_THREADS / FACE_CHUNK, RPT = ROWS / NS;
  extern __shared__ double sh[];  // [ROWS][qmax]
  const int c0 = blockIdx.x * FACE_CHUNK;
  const int q1b = blockIdx.y * ROWS;
  const int nc = min(FACE_CHUNK, n0 - c0);
  const int ia = i0_begin + c0;
  const int qa = qs0[ia];
  const int nq = min(Q0, qs0[ia + nc - 1] + wmax0) - qa;  // <= qmax (host-checked)
  const int nrows = min(ROWS, Q1 - q1b);
  for (int e = threadIdx.x; e < nrows * nq; e += FACE_THREADS) {
    const int r = e / nq, c = e - r * nq;
    sh[r * qmax + c] = U[(int64_t)(q1b + r) * Q0 + qa + c];
  }
  __syncthreads();
  const int t = threadIdx.x % FACE_CHUNK, sl = threadIdx.x / FACE_CHUNK;
  if (t >= nc) return;
  const int i0 = ia + t;
  const int b = qs0[i0] - qa;
  const int mend = min(wmax0, nq - b);  // weights past the node's own count are 0
  double acc[RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) acc[r] = 0.0;
  for (int m = 0; m < mend; ++m) {
    const double w = w0T[(int64_t)m * ldw0 + i0];
#pragma unroll
    for (int r = 0; r < RPT; ++r) acc[r] = fma(w, sh[(sl + r * NS) * qmax + b + m], acc[r]);
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int row = sl + r * NS;
    if (row < nrows) T[(int64_t)(q1b + row) * n0 + c0 + t] = acc[r];
  }
}

// dst(i0, i1) += scale sum_m w1[i1][m] T[qs1(i1) + m][i0] for NI1 consecutive
// i1 per block: every T row of the block's range is read once (rows of
// neighbouring i1 overlap p-fold); w1, qs1, qc1 are wave-uniform
template <int NI1>
__global__ void __launch_bounds__(64) face_step2_kernel(const double *__restrict__ T, int n0, int i1_begin,
                                                         int i1_end, const int *__restrict__ qs1,
                                                         const int *__restrict__ qc1,
                                                         const double *__restrict__ w1, int wmax1,
                                                         double *__restrict__ dst, int64_t base, int64_t stride0,
                                                         int64_t stride1, double scale) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  const int ib = i1_begin + (int)blockIdx.y * NI1, ie = min(ib + NI1, i1_end);
  if (t >= n0 || ib >= ie) return;
  const int r0 = qs1[ib], r1 = qs1[ie - 1] + qc1[ie - 1];
  double acc[NI1];
#pragma unroll
  for (int j = 0; j < NI1; ++j) acc[j] = 0.0;
  for (int r = r0; r < r1; ++r) {
    const double v = T[(int64_t)r * n0 + t];
#pragma unroll
    for (int j = 0; j < NI1; ++j) {
      const int i1 = ib + j;
      if (i1 < ie) {
        const int m = r - qs1[i1];
        if (m >= 0 && m < qc1[i1]) acc[j] = fma(w1[(int64_t)i1 * wmax1 + m], v, acc[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NI1; ++j)
    if (ib + j < ie) {
      double *d = dst + base + (int64_t)t * stride0 + (int64_t)(ib + j - i1_begin) * stride1;
      *d += scale * acc[j];
    }
}

''' + s[j:]
i = s.index("  dim3 b(256);\n  // rows per workgroup")
j = s.index("  return hipGetLastError();\n}\n\nextern \"C\" hipError_t gdmk_launch_axpby")
s = s[:i] + '''  // rows per workgroup: as many as fit 64 KiB of LDS (16, 8 or 4)
  const size_t row_bytes = sizeof(double) * (size_t)f.qmax0;
  const int rows = row_bytes * 16 <= 64 * 1024 ? 16 : (row_bytes * 8 <= 64 * 1024 ? 8 : 4);
  if (row_bytes * 4 > 64 * 1024) return hipErrorInvalidValue;  // (FACE_CHUNK + 2p) (p + 1) doubles in practice
  dim3 g1((n0 + FACE_CHUNK - 1) / FACE_CHUNK, (f.Q1 + rows - 1) / rows);
  const size_t lds = row_bytes * rows;
  static bool attr = false;
  if (!attr) {
    for (const void *k : {(const void *)face_step1_kernel<16>, (const void *)face_step1_kernel<8>,
                          (const void *)face_step1_kernel<4>}) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  if (rows == 16)
    hipLaunchKernelGGL(face_step1_kernel<16>, g1, dim3(FACE_THREADS), lds, st, f.U, f.Q0, f.Q1, f.i0_begin, n0,
                       f.qs0, f.w0T, f.wmax0, f.ldw0, f.qmax0, f.T);
  else if (rows == 8)
    hipLaunchKernelGGL(face_step1_kernel<8>, g1, dim3(FACE_THREADS), lds, st, f.U, f.Q0, f.Q1, f.i0_begin, n0,
                       f.qs0, f.w0T, f.wmax0, f.ldw0, f.qmax0, f.T);
  else
    hipLaunchKernelGGL(face_step1_kernel<4>, g1, dim3(FACE_THREADS), lds, st, f.U, f.Q0, f.Q1, f.i0_begin, n0,
                       f.qs0, f.w0T, f.wmax0, f.ldw0, f.qmax0, f.T);
  constexpr int NI1 = 8;
  dim3 g2((n0 + 63) / 64, (f.i1_end - f.i1_begin + NI1 - 1) / NI1);
  hipLaunchKernelGGL(face_step2_kernel<NI1>, g2, dim3(64), 0, st, f.T, n0, f.i1_begin, f.i1_end, f.qs1, f.qc1,
                     f.w1, f.wmax1, f.dst, f.base, f.stride0, f.stride1, f.scale);
''' + s[j:]
open('gdm_kernels.hip', 'w').write(s)
h = open('gdm_kernels.h').read()
old = "constexpr int FACE_CHUNK = 256;  // t0 nodes per workgroup of the face row kernel"
assert old in h
h = h.replace(old, "constexpr int FACE_CHUNK = 64;     // t0 nodes per workgroup of the face row kernel\nconstexpr int FACE_THREADS = 256;  // 4 row slices of FACE_CHUNK nodes")
open('gdm_kernels.h', 'w').write(h)
print("ok")
