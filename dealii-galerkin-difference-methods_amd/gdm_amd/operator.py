"""Device operator handle over the C ABI (include/gdm_hip.h).

`GdmOperator` owns one `gdm_op`: the uncut structured-mesh GDM operator of
one rank (mass, advection, wave or convective) with its slab layout.  Vectors
are torch CUDA tensors (fp64); torch is only the allocator / stream provider.
"""
import ctypes

import numpy as np

from . import _capi
from ._capi import GdmError, check

KINDS = {
    "mass": _capi.GDM_OP_MASS,
    "advection": _capi.GDM_OP_ADVECTION,
    "wave": _capi.GDM_OP_WAVE,
    "convective": _capi.GDM_OP_CONVECTIVE,
}


def _ptr(t):
    if t is None:
        return None
    import torch

    if not t.is_cuda or t.dtype != torch.float64:
        raise GdmError("device fp64 tensor expected")
    if not t.is_contiguous():
        raise GdmError("contiguous tensor expected")
    return ctypes.c_void_p(t.data_ptr())


class GdmOperator:
    """One rank's operator.  Local vectors are laid out
    [ghost planes below | owned planes | ghost planes above] along the last
    coordinate, each plane in the reference's lexicographic DoF order."""

    def __init__(self, dim, fe_degree, n_subdivisions, lo, hi, kind, params=(), rank=0, n_ranks=1, device=0,
                 periodic=0):
        import torch

        self._torch = torch
        self.lib = _capi.load()
        if not torch.cuda.is_available():
            raise GdmError("no GPU visible: the GDM operator engine has no CPU path")
        m = _capi.MeshDesc()
        m.dim = dim
        m.fe_degree = fe_degree
        ns = list(n_subdivisions) if hasattr(n_subdivisions, "__len__") else [n_subdivisions] * dim
        los = list(lo) if hasattr(lo, "__len__") else [lo] * dim
        his = list(hi) if hasattr(hi, "__len__") else [hi] * dim
        for d in range(3):
            m.n_subdivisions[d] = int(ns[d]) if d < dim else 1
            m.lo[d] = float(los[d]) if d < dim else 0.0
            m.hi[d] = float(his[d]) if d < dim else 1.0
        m.n_ranks, m.rank, m.periodic = n_ranks, rank, periodic
        self.mesh = m
        self.dim, self.p = dim, fe_degree
        self.kind = KINDS[kind] if isinstance(kind, str) else kind
        self.device = device
        arr = (ctypes.c_double * max(1, len(params)))(*params) if len(params) else None
        h = ctypes.c_void_p()
        torch.cuda.set_device(device)
        check(self.lib.gdm_op_create(ctypes.byref(m), self.kind, arr, len(params), device, ctypes.byref(h)),
              "gdm_op_create")
        self.h = h
        lay = _capi.Layout()
        check(self.lib.gdm_op_layout(self.h, ctypes.byref(lay)), "gdm_op_layout")
        self.layout = lay.as_dict()
        self.use_torch_stream()

    # -- lifetime -----------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.gdm_op_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def use_torch_stream(self):
        """Order the operator's launches on torch's current stream."""
        s = self._torch.cuda.current_stream(self.device).cuda_stream
        check(self.lib.gdm_op_set_stream(self.h, ctypes.c_void_p(s)), "gdm_op_set_stream")

    # -- layout helpers --------------------------------------------------------
    @property
    def n_local(self):
        return self.layout["n_local"]

    @property
    def n_owned(self):
        return self.layout["n_owned"]

    @property
    def n_bc_points(self):
        return self.layout["n_bc_points"]

    def owned_view(self, local):
        lay = self.layout
        b = lay["ghost_planes_below"] * lay["plane_size"]
        return local[b:b + lay["n_owned"]]

    def new_vector(self, local=True):
        n = self.n_local if local else self.n_owned
        return self._torch.zeros(n, dtype=self._torch.float64, device="cuda:%d" % self.device)

    def _check_sizes(self, src_local, dst_owned):
        if src_local is not None and src_local.numel() != self.n_local:
            raise GdmError("src has %d entries, local layout needs %d" % (src_local.numel(), self.n_local))
        if dst_owned is not None and dst_owned.numel() != self.n_owned:
            raise GdmError("dst has %d entries, owned layout needs %d" % (dst_owned.numel(), self.n_owned))

    # -- operator applications -------------------------------------------------
    def apply(self, src_local, dst_owned, bc_values=None):
        self._check_sizes(src_local, dst_owned)
        if bc_values is not None and bc_values.numel() != self.n_bc_points:
            raise GdmError("bc_values has %d entries, expected %d" % (bc_values.numel(), self.n_bc_points))
        check(self.lib.gdm_apply(self.h, _ptr(src_local), _ptr(dst_owned), _ptr(bc_values)), "gdm_apply")
        return dst_owned

    def apply_planes(self, src_local, dst_owned, plane_begin, plane_end):
        """Volume term for the owned output planes [plane_begin, plane_end) only."""
        self._check_sizes(src_local, dst_owned)
        check(self.lib.gdm_apply_planes(self.h, _ptr(src_local), _ptr(dst_owned), int(plane_begin), int(plane_end)),
              "gdm_apply_planes")
        return dst_owned

    def apply_planes2(self, src_local, dst_owned, b0, e0, b1, e1):
        """apply_planes of two plane ranges in one launch (gdm_apply_planes2)"""
        self._check_sizes(src_local, dst_owned)
        check(self.lib.gdm_apply_planes2(self.h, _ptr(src_local), _ptr(dst_owned), int(b0), int(e0), int(b1),
                                         int(e1)), "gdm_apply_planes2")
        return dst_owned

    def add_boundary_data(self, bc_values, dst_owned):
        self._check_sizes(None, dst_owned)
        check(self.lib.gdm_add_boundary_data(self.h, _ptr(bc_values), _ptr(dst_owned)), "gdm_add_boundary_data")
        return dst_owned

    def mass_apply(self, src_local, dst_owned):
        self._check_sizes(src_local, dst_owned)
        check(self.lib.gdm_mass_apply(self.h, _ptr(src_local), _ptr(dst_owned)), "gdm_mass_apply")
        return dst_owned

    def mass_solve_rk(self, rhs_owned, beta, acc_in, acc_out, alpha=0.0, y=None, Y=None):
        """k = M^-1 rhs; acc_out = acc_in + beta k; Y = y + alpha k (when Y is
        given), with the update fused into the last line-solve pass
        (gdm_mass_solve_rk): rhs_owned is overwritten; the same bits as
        mass_solve(rhs, rhs) + rk_update"""
        n = self.n_owned
        for v in (rhs_owned, acc_in, acc_out) + ((y, Y) if Y is not None else ()):
            if v.numel() != n:
                raise GdmError("mass_solve_rk: vectors need n_owned = %d entries" % n)
        check(self.lib.gdm_mass_solve_rk(self.h, _ptr(rhs_owned), float(beta), _ptr(acc_in), _ptr(acc_out),
                                         float(alpha), _ptr(y) if Y is not None else None, _ptr(Y)),
              "gdm_mass_solve_rk")
        return acc_out

    def mass_solve(self, rhs_owned, x_owned):
        self._check_sizes(None, rhs_owned)
        self._check_sizes(None, x_owned)
        check(self.lib.gdm_mass_solve(self.h, _ptr(rhs_owned), _ptr(x_owned)), "gdm_mass_solve")
        return x_owned

    def mass_solve_cg(self, rhs_owned, x_owned, rel_tol=1e-8, abs_tol=1e-10, max_it=100, precond=1):
        """SolverCG on the matrix-free (condensed) mass: returns (iterations, residual)"""
        self._check_sizes(None, rhs_owned)
        self._check_sizes(None, x_owned)
        its, res = ctypes.c_int(0), ctypes.c_double(0.0)
        check(self.lib.gdm_mass_solve_cg(self.h, _ptr(rhs_owned), _ptr(x_owned), float(rel_tol), float(abs_tol),
                                         int(max_it), int(precond), ctypes.byref(its), ctypes.byref(res)),
              "gdm_mass_solve_cg")
        return its.value, res.value

    def distribute(self, v_owned):
        """constraints.distribute (periodicity constraints; no-op otherwise)"""
        check(self.lib.gdm_constraints_distribute(self.h, _ptr(v_owned)), "gdm_constraints_distribute")
        return v_owned

    def mass_solve_lines(self, axis, v, n_lines, stride, A, B, C):
        """In-place 1D mass solves along `axis` (gdm_mass_solve_lines)."""
        check(self.lib.gdm_mass_solve_lines(self.h, int(axis), _ptr(v), int(n_lines), int(stride), int(A), int(B),
                                            int(C)), "gdm_mass_solve_lines")
        return v

    def axpby(self, a, x, b, y):
        check(self.lib.gdm_vec_axpby(self.h, x.numel(), float(a), _ptr(x), float(b), _ptr(y)), "gdm_vec_axpby")
        return y

    def rk_update(self, beta, k, acc_in, acc_out, alpha=0.0, y=None, Y=None):
        """acc_out = acc_in + beta k; Y = y + alpha k (when Y is given), one pass"""
        n = k.numel()
        for v in (acc_in, acc_out) + ((y, Y) if Y is not None else ()):
            if v.numel() != n:
                raise GdmError("rk_update: vector sizes differ")
        check(self.lib.gdm_vec_rk_update(self.h, n, float(beta), _ptr(k), _ptr(acc_in), _ptr(acc_out), float(alpha),
                                         _ptr(y) if Y is not None else None, _ptr(Y)), "gdm_vec_rk_update")
        return acc_out

    FN_CONSTANT, FN_CONE, FN_SINE_PRODUCT = 0, 1, 2

    def eval_boundary(self, fn_kind, params, t, derivative, out):
        """out (device order, n_bc_points) = g(t) or dg/dt(t) of a built-in function"""
        if out.numel() != self.n_bc_points:
            raise GdmError("eval_boundary: out has %d entries, expected %d" % (out.numel(), self.n_bc_points))
        prm = (ctypes.c_double * max(len(params), 1))(*[float(v) for v in params])
        check(self.lib.gdm_eval_boundary(self.h, int(fn_kind), prm, len(params), float(t), int(derivative),
                                         _ptr(out)), "gdm_eval_boundary")
        return out

    def apply_bc_fn(self, src_local, dst_owned, fn_kind, params, t_g, alpha=0.0, t_k=0.0):
        """apply() with the stage boundary values g(t_g) + alpha dg/dt(t_k) of a
        built-in function computed by the engine right before the stencil (gdm_apply_bc_fn):
        the same bits as eval_boundary + rk_update + apply(bc_values)"""
        self._check_sizes(src_local, dst_owned)
        prm = (ctypes.c_double * max(len(params), 1))(*[float(v) for v in params])
        check(self.lib.gdm_apply_bc_fn(self.h, _ptr(src_local), _ptr(dst_owned), int(fn_kind), prm, len(params),
                                       float(t_g), float(alpha), float(t_k)), "gdm_apply_bc_fn")
        return dst_owned

    def add_boundary_fn(self, dst_owned, fn_kind, params, t_g, alpha=0.0, t_k=0.0):
        """add_boundary_data() with the stage boundary values of apply_bc_fn (gdm_add_boundary_fn)"""
        self._check_sizes(None, dst_owned)
        prm = (ctypes.c_double * max(len(params), 1))(*[float(v) for v in params])
        check(self.lib.gdm_add_boundary_fn(self.h, _ptr(dst_owned), int(fn_kind), prm, len(params), float(t_g),
                                           float(alpha), float(t_k)), "gdm_add_boundary_fn")
        return dst_owned

    def mass_solve_slab(self, rhs_owned, x_owned):
        """Distributed exact mass inverse, step 1: the slab-local solve
        (gdm_mass_solve_slab).  Then exchange the ghost planes of the local
        vector holding x_owned and call mass_solve_interface."""
        check(self.lib.gdm_mass_solve_slab(self.h, _ptr(rhs_owned), _ptr(x_owned)), "gdm_mass_solve_slab")
        return x_owned

    def mass_solve_interface_round(self, x_local, round_):
        """Distributed exact mass inverse, refinement round `round_` of
        gdm_mass_spike_rounds (thin slabs): the slab's edge planes become the
        next interface systems' right-hand sides; exchange the ghost planes of
        x_local again afterwards."""
        if x_local.numel() != self.n_local:
            raise GdmError("mass_solve_interface_round: x has %d entries, expected n_local %d"
                           % (x_local.numel(), self.n_local))
        check(self.lib.gdm_mass_solve_interface_round(self.h, _ptr(x_local), int(round_)),
              "gdm_mass_solve_interface_round")
        return x_local

    def mass_solve_interface(self, x_local):
        """Distributed exact mass inverse, step 2 (gdm_mass_solve_interface):
        the owned part of x_local (ghost planes = the neighbours' slab solves)
        becomes M^-1 rhs."""
        if x_local.numel() != self.n_local:
            raise GdmError("mass_solve_interface: x has %d entries, expected n_local %d" % (x_local.numel(),
                                                                                          self.n_local))
        check(self.lib.gdm_mass_solve_interface(self.h, _ptr(x_local)), "gdm_mass_solve_interface")
        return x_local

    def mass_solve_interface_ghosts(self, x_local):
        """mass_solve_interface, and the ghost planes of x_local become the
        interface solution (the neighbours' edge planes of M^-1 rhs,
        gdm_mass_solve_interface_ghosts): x_local is a valid local vector
        without another exchange"""
        if x_local.numel() != self.n_local:
            raise GdmError("mass_solve_interface_ghosts: x has %d entries, expected n_local %d"
                           % (x_local.numel(), self.n_local))
        check(self.lib.gdm_mass_solve_interface_ghosts(self.h, _ptr(x_local)), "gdm_mass_solve_interface_ghosts")
        return x_local

    def mass_solve_interface_rk(self, x_local, beta, acc_in, acc_out, alpha=0.0, y=None, Y=None):
        """mass_solve_interface_ghosts fused with rk_update over the local
        vectors (gdm_mass_solve_interface_rk): acc_out = acc_in + beta k, Y =
        y + alpha k (when Y is given) with k the interface-corrected solve of
        every local plane; x_local is only read.  The bits of
        mass_solve_interface_ghosts(x) + rk_update(beta, x, ...)."""
        n = self.n_local
        for v in (x_local, acc_in, acc_out) + ((y, Y) if Y is not None else ()):
            if v.numel() != n:
                raise GdmError("mass_solve_interface_rk: vectors need n_local = %d entries" % n)
        check(self.lib.gdm_mass_solve_interface_rk(self.h, _ptr(x_local), float(beta), _ptr(acc_in), _ptr(acc_out),
                                                   float(alpha), _ptr(y) if Y is not None else None, _ptr(Y)),
              "gdm_mass_solve_interface_rk")
        return acc_out

    def error_norms(self, u_local, fn_kind, params, t, cell_errors=None):
        """(Linf, L1, L2) of u - f(t) over QGauss(p+1) on the owned cells
        (advection/problem.h:269-425 postprocess, volume part); cell_errors
        (device, n_owned_cells) receives integrate_difference's per-cell L2
        errors (vector_tools.h:25-86).  Multi-rank callers reduce: max, sum,
        sqrt(sum of squares)."""
        if u_local.numel() != self.n_local:
            raise GdmError("error_norms: u has %d entries, expected n_local %d" % (u_local.numel(), self.n_local))
        if cell_errors is not None and cell_errors.numel() != self.n_owned_cells:
            raise GdmError("error_norms: cell_errors has %d entries, expected %d" % (cell_errors.numel(),
                                                                                     self.n_owned_cells))
        prm = (ctypes.c_double * max(len(params), 1))(*[float(v) for v in params])
        out = (ctypes.c_double * 3)()
        check(self.lib.gdm_error_norms(self.h, _ptr(u_local), int(fn_kind), prm, len(params), float(t),
                                       _ptr(cell_errors), out), "gdm_error_norms")
        return tuple(out)

    @property
    def n_owned_cells(self):
        n = max(0, self.layout["cell_plane_end"] - self.layout["cell_plane_begin"])
        for d in range(self.dim - 1):
            n *= self.mesh.n_subdivisions[d]
        return n

    def dot(self, x, y):
        r = ctypes.c_double(0.0)
        check(self.lib.gdm_vec_dot(self.h, x.numel(), _ptr(x), _ptr(y), ctypes.byref(r)), "gdm_vec_dot")
        return r.value

    def synchronize(self):
        check(self.lib.gdm_synchronize(self.h), "gdm_synchronize")

    def time_op(self, which, src, dst, bc=None, n_iter=10):
        ms = ctypes.c_double(0.0)
        check(self.lib.gdm_time_op(self.h, int(which), _ptr(src), _ptr(dst), _ptr(bc), int(n_iter), ctypes.byref(ms)),
              "gdm_time_op")
        return ms.value

    # -- boundary points -------------------------------------------------------
    def bc_points(self):
        n = self.n_bc_points
        xyz = np.zeros((max(n, 1), 3))
        check(self.lib.gdm_bc_points(self.h, xyz.ctypes.data_as(ctypes.c_void_p)), "gdm_bc_points")
        return xyz[:n]

    @property
    def n_bc_points_ref(self):
        return self.layout["n_bc_points_ref"]

    def bc_reference_order(self):
        n = self.n_bc_points_ref
        perm = np.zeros(max(n, 1), dtype=np.int64)
        check(self.lib.gdm_bc_reference_order(self.h, perm.ctypes.data_as(ctypes.c_void_p)),
              "gdm_bc_reference_order")
        return perm[:n]
