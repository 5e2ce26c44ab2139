"""oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper over the CPU restatement in oracle/gdm_oracle.c (reference-
faithful cell loops) and oracle/gdm_oracle_kron.c (Kronecker cross-check).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline -- never
as part of the product path.

Reference anchors are listed in the C sources' headers.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libgdm_oracle.so")

_lib = None


def build(force=False):
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        d, i, u, i64 = ctypes.c_double, ctypes.c_int, ctypes.c_uint, ctypes.c_int64
        P = ctypes.c_void_p
        L.gdmo_basis_derivative.restype = d
        L.gdmo_basis_derivative.argtypes = [i, i, i, d, i]
        L.gdmo_basis_coefficients.argtypes = [i, i, i, P]
        L.gdmo_gauss.argtypes = [i, P, P]
        L.gdmo_category.restype = u
        L.gdmo_category.argtypes = [u, u, u]
        L.gdmo_offset.restype = u
        L.gdmo_offset.argtypes = [u, u, u]
        L.gdmo_cell_dof_indices.argtypes = [i, i, P, u, P]
        L.gdmo_fe_index.restype = u
        L.gdmo_fe_index.argtypes = [i, i, P, u]
        L.gdmo_partition.argtypes = [u, u, u, P]
        L.gdmo_n_boundary_points.restype = ctypes.c_uint64
        L.gdmo_n_boundary_points.argtypes = [i, i, P, u, u]
        L.gdmo_boundary_points.argtypes = [i, i, P, P, P, u, u, P]
        L.gdmo_advection_rhs.argtypes = [i, i, P, P, P, P, P, P, P, u, u]
        L.gdmo_advection_inflow.argtypes = [i, i, P, P, P, P, P, P]
        L.gdmo_convective_rhs.argtypes = [i, i, P, P, P, P, P, P]
        L.gdmo_wave_rhs.argtypes = [i, i, P, P, P, P, i, P, d, P, P, u, u]
        L.gdmo_matrix_csr.restype = i64
        L.gdmo_matrix_csr.argtypes = [i, i, P, P, P, i, P, P, P]
        L.gdmo_csr_vmult.argtypes = [i64, P, P, P, P, P]
        L.gdmo_cg.restype = i
        L.gdmo_cg.argtypes = [i64, P, P, P, P, P, i, i, d, d]
        L.gdmo_cg_history.restype = i
        L.gdmo_cg_history.argtypes = [i64, P, P, P, P, P, i, i, d, d, P, P]
        L.gdmo_l2_error.restype = d
        L.gdmo_l2_error.argtypes = [i, i, P, P, P, P, P]
        L.gdmo_error_norms.argtypes = [i, i, P, P, P, P, P, P, P]
        L.gdmo_cell_qpoints.argtypes = [i, i, P, P, P, P]
        L.gdmo_matrices_1d.argtypes = [i, u, d, P, P, P]
        L.gdmo_kron_apply.argtypes = [P, i, i, P, P, P]
        L.gdmo_kron_mass_inverse.argtypes = [P, i, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u3(v, dim):
    a = np.ones(3, dtype=np.uint32)
    a[:dim] = v[:dim] if hasattr(v, "__len__") else v
    return a


def _d3(v, dim, fill=0.0):
    a = np.full(3, fill, dtype=np.float64)
    if hasattr(v, "__len__"):
        a[:dim] = v[:dim]
    else:
        a[:dim] = v
    return a


class Mesh:
    """Uniform Cartesian GDM mesh: dim, degree p, n_sub per direction, box."""

    def __init__(self, dim, p, n_sub, lo=0.0, hi=1.0):
        self.dim, self.p = dim, p
        self.nsub = _u3(n_sub, dim)
        if dim < 3:
            self.nsub[dim:] = 1
        self.lo = _d3(lo, dim)
        self.hi = _d3(hi, dim, 1.0)
        self.N = [int(self.nsub[d]) + 1 if d < dim else 1 for d in range(3)]
        self.n_dofs = int(np.prod(self.N))
        self.n_cells = int(np.prod([int(self.nsub[d]) for d in range(dim)]))
        self.h = [(self.hi[d] - self.lo[d]) / self.nsub[d] for d in range(dim)]

    # -- indexing --------------------------------------------------------
    def cell_dofs(self, cell):
        out = np.zeros((self.p + 1) ** self.dim, dtype=np.uint64)
        lib().gdmo_cell_dof_indices(self.dim, self.p, _p(self.nsub), cell, _p(out))
        return out

    def fe_index(self, cell):
        return lib().gdmo_fe_index(self.dim, self.p, _p(self.nsub), cell)

    def partition(self, n_procs, rank):
        out = np.zeros(4, dtype=np.uint32)
        lib().gdmo_partition(int(self.nsub[self.dim - 1]), n_procs, rank, _p(out))
        return tuple(int(x) for x in out)

    def vertex_coords(self):
        axes = [self.lo[d] + np.arange(self.N[d]) * self.h[d] for d in range(self.dim)]
        grids = np.meshgrid(*axes[::-1], indexing="ij")[::-1]
        return [g.reshape(-1) for g in grids]

    def cell_qpoints(self):
        nq = (self.p + 1) ** self.dim
        xyz = np.zeros((self.n_cells * nq, 3))
        lib().gdmo_cell_qpoints(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(xyz))
        return xyz

    def n_boundary_points(self, cb=0, ce=None):
        ce = int(self.nsub[self.dim - 1]) if ce is None else ce
        return int(lib().gdmo_n_boundary_points(self.dim, self.p, _p(self.nsub), cb, ce))

    def boundary_points(self, cb=0, ce=None):
        ce = int(self.nsub[self.dim - 1]) if ce is None else ce
        n = self.n_boundary_points(cb, ce)
        xyz = np.zeros((n, 3))
        lib().gdmo_boundary_points(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), cb, ce, _p(xyz))
        return xyz

    # -- cell-loop operators (reference-faithful) -------------------------
    def advection_rhs(self, a, u, stage_bc=None, cb=0, ce=None, rhs=None):
        ce = int(self.nsub[self.dim - 1]) if ce is None else ce
        a3 = _d3(a, self.dim)
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(self.n_dofs) if rhs is None else rhs
        bc = None if stage_bc is None else np.ascontiguousarray(stage_bc, dtype=np.float64)
        lib().gdmo_advection_rhs(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(a3), _p(u),
                                 _p(bc) if bc is not None else None, _p(out), cb, ce)
        return out

    def advection_inflow(self, a, stage_bc):
        """The inflow-data part of advection_rhs alone (u = 0), visiting only
        the boundary cells: gdmo_advection_inflow"""
        a3 = _d3(a, self.dim)
        bc = np.ascontiguousarray(stage_bc, dtype=np.float64)
        assert bc.size == self.n_boundary_points()
        out = np.zeros(self.n_dofs)
        lib().gdmo_advection_inflow(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(a3), _p(bc),
                                    _p(out))
        return out

    def convective_rhs(self, a, u):
        a3 = _d3(a, self.dim)
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(self.n_dofs)
        lib().gdmo_convective_rhs(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(a3), _p(u), _p(out))
        return out

    def wave_rhs(self, u, impl=True, fq=None, nitsche=0.0, gbc=None, cb=0, ce=None):
        ce = int(self.nsub[self.dim - 1]) if ce is None else ce
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(self.n_dofs)
        fq = None if fq is None else np.ascontiguousarray(fq, dtype=np.float64)
        gbc = None if gbc is None else np.ascontiguousarray(gbc, dtype=np.float64)
        lib().gdmo_wave_rhs(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(u), int(impl),
                            _p(fq) if fq is not None else None, float(nitsche),
                            _p(gbc) if gbc is not None else None, _p(out), cb, ce)
        return out

    def matrix_csr(self, kind=0):
        """kind 0 = mass, 1 = Laplace.  Returns (rowptr, cols, vals)."""
        n = self.n_dofs
        rowptr = np.zeros(n + 1, dtype=np.int64)
        nnz = lib().gdmo_matrix_csr(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), kind, _p(rowptr),
                                    None, None)
        cols = np.zeros(nnz, dtype=np.int64)
        vals = np.zeros(nnz)
        lib().gdmo_matrix_csr(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), kind, _p(rowptr), _p(cols),
                              _p(vals))
        return rowptr, cols, vals

    def l2_error(self, u, exact_q):
        u = np.ascontiguousarray(u, dtype=np.float64)
        e = np.ascontiguousarray(exact_q, dtype=np.float64)
        return lib().gdmo_l2_error(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(u), _p(e))

    def error_norms(self, u, exact_q, cells=False):
        """(Linf, L1, L2) of u - exact over QGauss(p+1) (advection/problem.h:
        330-425 volume part); cells=True also returns integrate_difference's
        per-cell L2 errors (vector_tools.h:25-86)."""
        u = np.ascontiguousarray(u, dtype=np.float64)
        e = np.ascontiguousarray(exact_q, dtype=np.float64)
        out = np.zeros(3)
        cl = np.zeros(self.n_cells) if cells else None
        lib().gdmo_error_norms(self.dim, self.p, _p(self.nsub), _p(self.lo), _p(self.hi), _p(u), _p(e), _p(out),
                               _p(cl) if cells else None)
        return (tuple(out), cl) if cells else tuple(out)

    # -- Kronecker cross-check ---------------------------------------------
    def matrices_1d(self, d):
        N = self.N[d]
        W = 2 * self.p + 1
        M, C, L = (np.zeros(N * W) for _ in range(3))
        lib().gdmo_matrices_1d(self.p, int(self.nsub[d]), float(self.h[d]), _p(M), _p(C), _p(L))
        return M.reshape(N, W), C.reshape(N, W), L.reshape(N, W)

    def kron_apply(self, terms, u):
        """terms: list of 3-tuples (op_x, op_y, op_z) of band matrices or None."""
        u = np.ascontiguousarray(u, dtype=np.float64)
        keep = []
        ptrs = (ctypes.c_void_p * (3 * len(terms)))()
        for t, ops in enumerate(terms):
            for d in range(3):
                A = ops[d] if d < len(ops) else None
                if A is None:
                    ptrs[3 * t + d] = None
                else:
                    A = np.ascontiguousarray(A, dtype=np.float64)
                    keep.append(A)
                    ptrs[3 * t + d] = A.ctypes.data
        N = np.array(self.N, dtype=np.uint32)
        y = np.zeros(self.n_dofs)
        lib().gdmo_kron_apply(_p(N), self.p, len(terms), ctypes.cast(ptrs, ctypes.c_void_p), _p(u), _p(y))
        return y

    def kron_mass_inverse(self, r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        keep = []
        ptrs = (ctypes.c_void_p * 3)()
        for d in range(3):
            if d < self.dim:
                M = np.ascontiguousarray(self.matrices_1d(d)[0])
                keep.append(M)
                ptrs[d] = M.ctypes.data
            else:
                ptrs[d] = None
        N = np.array(self.N, dtype=np.uint32)
        x = np.zeros(self.n_dofs)
        lib().gdmo_kron_mass_inverse(_p(N), self.p, ctypes.cast(ptrs, ctypes.c_void_p), _p(r), _p(x))
        return x

    def advection_outflow_B(self, d, a_d):
        """B_d = a_d C_d - outflow traces (face term (III) with a.n >= 0)."""
        M, C, L = self.matrices_1d(d)
        B = a_d * C.copy()
        p = self.p
        n = self.N[d] - 1
        if a_d >= 0.0:  # x = right face is outflow (a.n = a_d >= 0)
            B[n, p] -= a_d
        if -a_d >= 0.0:  # x = left face: a.n = -a_d >= 0
            B[0, p] += a_d
        return B


def cg(rowptr, cols, vals, b, x=None, precond=0, max_it=1000, abs_tol=1e-20, rel_tol=1e-14):
    n = len(rowptr) - 1
    x = np.zeros(n) if x is None else np.ascontiguousarray(x, dtype=np.float64).copy()
    b = np.ascontiguousarray(b, dtype=np.float64)
    its = lib().gdmo_cg(n, _p(rowptr), _p(cols), _p(vals), _p(b), _p(x), precond, max_it, abs_tol, rel_tol)
    return x, its


def cg_history(rowptr, cols, vals, b, precond=0, max_it=1000, abs_tol=1e-20, rel_tol=1e-14):
    """cg() from a zero start that also returns the residual norm history
    (hist[0] before iteration 1, hist[k] after iteration k) and the stopping
    threshold max(abs_tol, rel_tol |r_0|) of deal.II's ReductionControl."""
    n = len(rowptr) - 1
    x = np.zeros(n)
    b = np.ascontiguousarray(b, dtype=np.float64)
    hist = np.full(max_it + 1, np.nan)
    tol = np.zeros(1)
    its = lib().gdmo_cg_history(n, _p(rowptr), _p(cols), _p(vals), _p(b), _p(x), precond, max_it, abs_tol,
                                rel_tol, _p(hist), _p(tol))
    last = its if its >= 0 else max_it
    return x, its, hist[:last + 1], float(tol[0])


def csr_vmult(rowptr, cols, vals, x):
    n = len(rowptr) - 1
    y = np.zeros(n)
    x = np.ascontiguousarray(x, dtype=np.float64)
    lib().gdmo_csr_vmult(n, _p(rowptr), _p(cols), _p(vals), _p(x), _p(y))
    return y


def basis_value(p, cat, i, x, order=0):
    return lib().gdmo_basis_derivative(p, cat, i, float(x), order)


def basis_coefficients(p, cat, i):
    c = np.zeros(p + 1)
    lib().gdmo_basis_coefficients(p, cat, i, _p(c))
    return c


def gauss(n):
    x, w = np.zeros(n), np.zeros(n)
    lib().gdmo_gauss(n, _p(x), _p(w))
    return x, w
