"""Assembled sparse matrices on the device over the C ABI (include/gdm_hip.h,
"Assembled sparse matrices").

`SparseMatrix` mirrors the part of `dealii::SparseMatrix<double>` the
reference's cut-cell Poisson prototype uses (`reinit` + assembled values,
`vmult`, `m`, `n`, `n_nonzero_elements`; prototypes/cut_poisson_01_gdm.cc:
148-163, 327-336), and `solve_cg` is `SolverCG<>(ReductionControl(max_it,
abs_tol, rel_tol)).solve(A, x, b, P)` with P = PreconditionIdentity or
PreconditionJacobi (cut_poisson_01_gdm.cc:332-335).  The triplet files of
applications/wave/wave-ev.cc:93-127 are read and written by `from_triplets` /
`write_triplets`.  Every computation runs in libgdm_hip.so; there is no CPU
path.
"""
import ctypes

import numpy as np

from . import _capi
from ._capi import GdmError, check

PRECONDITIONERS = {"identity": 0, "jacobi": 1}


def _dev(t):
    import torch

    if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
        raise GdmError("contiguous device fp64 tensor expected")
    return ctypes.c_void_p(t.data_ptr())


class SparseMatrix:
    """CSR matrix resident in HBM (int64 row pointers, uint32 columns, fp64 values)."""

    def __init__(self, row_ptr, cols, vals, n_cols=None, device=0, _handle=None):
        self._lib = _capi.load()
        self._h = ctypes.c_void_p()
        self.device = device
        if _handle is not None:
            self._h = _handle
            return
        import torch

        on_device = all(isinstance(a, torch.Tensor) and a.is_cuda for a in (row_ptr, cols, vals))
        if on_device:
            rp = row_ptr.to(torch.int64).contiguous()
            ci = cols.to(torch.int32).contiguous()  # reinterpreted as uint32 by the library
            v = vals.to(torch.float64).contiguous()
            keep = (rp, ci, v)
            ptrs = [ctypes.c_void_p(a.data_ptr()) for a in keep]
        else:
            rp = np.ascontiguousarray(np.asarray(row_ptr), dtype=np.int64)
            ci = np.ascontiguousarray(np.asarray(cols), dtype=np.uint32)
            v = np.ascontiguousarray(np.asarray(vals), dtype=np.float64)
            keep = (rp, ci, v)
            ptrs = [a.ctypes.data_as(ctypes.c_void_p) for a in keep]
        n_rows = int(rp.shape[0]) - 1
        nnz = int(v.shape[0])
        if n_cols is None:
            n_cols = n_rows
        check(self._lib.gdm_csr_create(device, n_rows, int(n_cols), nnz, ptrs[0], ptrs[1], ptrs[2],
                                       1 if on_device else 0, ctypes.byref(self._h)), "gdm_csr_create")
        del keep
        # order every launch after torch's own work on its tensors (fills, copies)
        self.use_torch_stream()

    @classmethod
    def from_scipy(cls, A, device=0):
        A = A.tocsr()
        A.sort_indices()
        return cls(A.indptr.astype(np.int64), A.indices.astype(np.uint32), A.data.astype(np.float64),
                   n_cols=A.shape[1], device=device)

    @classmethod
    def from_triplets(cls, path, binary=True, device=0):
        h = ctypes.c_void_p()
        check(_capi.load().gdm_csr_read_triplets(device, str(path).encode(), 1 if binary else 0, ctypes.byref(h)),
              "gdm_csr_read_triplets")
        A = cls(None, None, None, device=device, _handle=h)
        A.use_torch_stream()
        return A

    def write_triplets(self, path, binary=True):
        check(self._lib.gdm_csr_write_triplets(self._h, str(path).encode(), 1 if binary else 0),
              "gdm_csr_write_triplets")

    def close(self):
        if self._h:
            self._lib.gdm_csr_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _info(self):
        m, n, z = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self._lib.gdm_csr_info(self._h, ctypes.byref(m), ctypes.byref(n), ctypes.byref(z)), "gdm_csr_info")
        return m.value, n.value, z.value

    def m(self):
        return self._info()[0]

    def n(self):
        return self._info()[1]

    def n_nonzero_elements(self):
        return self._info()[2]

    def to_host(self):
        """(row_ptr int64, cols uint32, vals fp64) as numpy arrays."""
        m, _, z = self._info()
        rp = np.zeros(m + 1, dtype=np.int64)
        ci = np.zeros(max(z, 1), dtype=np.uint32)
        v = np.zeros(max(z, 1), dtype=np.float64)
        check(self._lib.gdm_csr_download(self._h, rp.ctypes.data_as(ctypes.c_void_p),
                                         ci.ctypes.data_as(ctypes.c_void_p), v.ctypes.data_as(ctypes.c_void_p)),
              "gdm_csr_download")
        return rp, ci[:z], v[:z]

    def use_torch_stream(self):
        import torch

        check(self._lib.gdm_csr_set_stream(self._h, ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
              "gdm_csr_set_stream")

    def vmult(self, dst, src):
        """dst = A src (device fp64 tensors; deal.II argument order)."""
        m, n, _ = self._info()
        if dst.numel() != m or src.numel() != n:
            raise GdmError("vmult: sizes %d x %d vs dst %d, src %d" % (m, n, dst.numel(), src.numel()))
        check(self._lib.gdm_csr_vmult(self._h, _dev(src), _dev(dst)), "gdm_csr_vmult")

    def time_vmult(self, dst, src, n_iter=10):
        ms = ctypes.c_double()
        check(self._lib.gdm_csr_time_vmult(self._h, _dev(src), _dev(dst), n_iter, ctypes.byref(ms)),
              "gdm_csr_time_vmult")
        return ms.value


def solve_cg(A, x, b, preconditioner="identity", max_it=1000, abs_tol=1e-20, rel_tol=1e-14):
    """SolverCG with ReductionControl(max_it, abs_tol, rel_tol); x holds the
    initial guess and receives the solution.  Returns (iterations, residual).
    Raises GdmError (like SolverControl::NoConvergence) when max_it is hit."""
    m = A.m()
    if x.numel() != m or b.numel() != m:
        raise GdmError("solve_cg: vector sizes do not match the matrix")
    its, res = ctypes.c_int(), ctypes.c_double()
    check(A._lib.gdm_csr_cg(A._h, _dev(b), _dev(x), PRECONDITIONERS[preconditioner], int(max_it), float(abs_tol),
                            float(rel_tol), ctypes.byref(its), ctypes.byref(res)), "gdm_csr_cg")
    return its.value, res.value


def stencil_csr_2d(n, p, terms, device=0, rows_per_chunk=1 << 20):
    """Device-built CSR of a 2D Kronecker-sum operator sum_t Y_t (x) X_t on an
    n x n vertex grid with the full structural (2p+1)^2 stencil of
    System::create_sparsity_pattern (system.h:586-599; every DoF pair sharing a
    cell, i.e. |i_d - j_d| <= p).  terms: list of (y_band, x_band), each a
    length-(2p+1) Toeplitz band (offsets -p..p).  Columns ascending in a row.
    Returns (row_ptr int64, cols int32, vals fp64) device tensors -- the input
    of SparseMatrix for the cut-Poisson matvec benchmark (config 5)."""
    import torch

    dev = torch.device("cuda", device)
    i = torch.arange(n, device=dev)
    cnt1 = torch.minimum(i + p, torch.full_like(i, n - 1)) - torch.clamp(i - p, min=0) + 1
    row_nnz = (cnt1[:, None] * cnt1[None, :]).reshape(-1)
    row_ptr = torch.zeros(n * n + 1, dtype=torch.int64, device=dev)
    row_ptr[1:] = torch.cumsum(row_nnz, 0)
    nnz = int(row_ptr[-1])
    cols = torch.empty(nnz, dtype=torch.int32, device=dev)
    vals = torch.empty(nnz, dtype=torch.float64, device=dev)
    off = torch.arange(-p, p + 1, device=dev)
    dy = off.repeat_interleave(2 * p + 1)  # slot order (dy, dx) -> ascending columns
    dx = off.repeat(2 * p + 1)
    w = torch.zeros(2 * p + 1, 2 * p + 1, dtype=torch.float64, device=dev)
    for yb, xb in terms:
        w += torch.as_tensor(yb, dtype=torch.float64, device=dev)[:, None] * \
            torch.as_tensor(xb, dtype=torch.float64, device=dev)[None, :]
    w = w.reshape(-1)
    for r0 in range(0, n * n, rows_per_chunk):
        r = torch.arange(r0, min(r0 + rows_per_chunk, n * n), device=dev)
        yy = (r // n)[:, None] + dy[None, :]
        xx = (r % n)[:, None] + dx[None, :]
        ok = (yy >= 0) & (yy < n) & (xx >= 0) & (xx < n)
        c = (yy * n + xx)[ok]
        vv = w[None, :].expand_as(ok)[ok]
        s, e = int(row_ptr[r0]), int(row_ptr[r[-1] + 1])
        cols[s:e] = c.to(torch.int32)
        vals[s:e] = vv
    return row_ptr, cols, vals


class CutPoisson:
    """The 2D cut-cell Poisson system of prototypes/cut_poisson_01_gdm.cc
    (`test<2>(ghost_penalty)`, :57-405): assembled on the host by
    libgdm_hip.so (csrc/gdm_cut.cpp: MeshClassifier of the FE_Q(1) level set
    of |x - center| - radius, the deal.II QuadratureGenerator (Saye) on every
    intersected cell, (grad v, grad u)_inside + Nitsche + ghost penalty),
    solved on the device:

        S = CutPoisson(p=3, n_sub=64, ghost_penalty=True)
        A = S.matrix()                      # SparseMatrix in HBM
        x = torch.zeros(S.n_rows, ...); its, res = solve_cg(A, x, S.rhs_tensor(), "identity",
                                                           S.n_rows, 1e-10, 1e-6)
        S.l2_error(x)                       # the prototype's error line
    """

    def __init__(self, p=3, n_sub=64, lo=-1.21, hi=1.21, center=(0.0, 0.0), radius=1.0, ghost_penalty=False,
                 rhs_value=4.0, bc_value=1.0):
        self._lib = _capi.load()
        self._h = ctypes.c_void_p()
        c = (ctypes.c_double * 2)(*center)
        check(self._lib.gdm_cut_poisson_create(int(p), int(n_sub), float(lo), float(hi), c, float(radius),
                                               1 if ghost_penalty else 0, float(rhs_value), float(bc_value),
                                               ctypes.byref(self._h)), "gdm_cut_poisson_create")
        n, z, a, b = (ctypes.c_int64() for _ in range(4))
        check(self._lib.gdm_cut_poisson_info(self._h, ctypes.byref(n), ctypes.byref(z), ctypes.byref(a),
                                             ctypes.byref(b)), "gdm_cut_poisson_info")
        self.n_rows, self.nnz, self.n_inside_cells, self.n_intersected_cells = n.value, z.value, a.value, b.value
        self.h = (hi - lo) / n_sub

    def close(self):
        if self._h:
            self._lib.gdm_cut_poisson_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def matrix(self, device=0):
        """the system matrix as a device CSR (SparseMatrix)"""
        h = ctypes.c_void_p()
        check(self._lib.gdm_cut_poisson_matrix(self._h, int(device), ctypes.byref(h)), "gdm_cut_poisson_matrix")
        A = SparseMatrix(None, None, None, device=device, _handle=h)
        A.use_torch_stream()
        return A

    def csr(self):
        """host copy (row_ptr int64, cols uint32, vals fp64) of the system matrix"""
        rp = np.zeros(self.n_rows + 1, dtype=np.int64)
        ci = np.zeros(self.nnz, dtype=np.uint32)
        v = np.zeros(self.nnz)
        check(self._lib.gdm_cut_poisson_csr(self._h, rp.ctypes.data_as(ctypes.c_void_p),
                                            ci.ctypes.data_as(ctypes.c_void_p), v.ctypes.data_as(ctypes.c_void_p)),
              "gdm_cut_poisson_csr")
        return rp, ci, v

    def rhs(self):
        """right-hand side (host numpy array, global DoF order)"""
        r = np.zeros(self.n_rows)
        check(self._lib.gdm_cut_poisson_rhs(self._h, r.ctypes.data_as(ctypes.c_void_p)), "gdm_cut_poisson_rhs")
        return r

    def l2_error(self, u):
        """L2 error of u (host array or device tensor) on the inside quadrature (:349-405)"""
        if hasattr(u, "cpu"):
            u = u.detach().cpu().numpy()
        u = np.ascontiguousarray(u, dtype=np.float64)
        if u.size != self.n_rows:
            raise GdmError("l2_error: %d values for %d DoFs" % (u.size, self.n_rows))
        e = ctypes.c_double()
        check(self._lib.gdm_cut_poisson_l2_error(self._h, u.ctypes.data_as(ctypes.c_void_p), ctypes.byref(e)),
              "gdm_cut_poisson_l2_error")
        return e.value
