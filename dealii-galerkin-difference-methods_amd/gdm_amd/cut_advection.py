"""The cut-cell advection application on the device: the
reference's applications/advection (non-composite, alpha = 0) on a 2D GDM
mesh cut by an FE_Q(1) level set, through the C ABI "Cut-cell advection"
entry points of include/gdm_hip.h.

  CutAdvection         StiffnessMatrixOperator::compute_rhs
                       (advection/stiffness.h:196-606) = uncut fused stencil
                       of the box (cut rows zeroed) + host-assembled cut rows + inflow
                       data, and the mass solve (mass.h:47-243 +
                       problem.h:236-267) as an exact banded solve
  CutAdvectionCompositeProblem
                       AdvectionProblem::run, composite branch (problem.h:103-181,
                       advection-app.cc's preset): an inside and an outside
                       field, each with its own advection, region, ghost
                       penalty and mass; the cut-surface inflow value is the
                       partner field (stiffness.h:448-453)
  CutAdvectionProblem  AdvectionProblem::run (problem.h:31-102): DiscreteTime,
                       initialize_time_step (block(0) = g(t_n) at the stage
                       boundary points), RK_CLASSIC_FOURTH_ORDER with
                       k = (dg/dt, M^-1 compute_rhs), device-resident in the
                       low-storage form of gdm_amd.problem; the boundary data
                       are evaluated on the host from the caller's functions
                       (the reference's Function::value calls) and uploaded.

Every computation runs in libgdm_hip.so; there is no CPU path.
"""
import ctypes

import numpy as np

from . import _capi
from ._capi import GdmError, check
from .problem import RK4_A, RK4_B, RK4_C, DiscreteTime


def _ptr(t):
    import torch

    if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
        raise GdmError("contiguous device fp64 tensor expected")
    return ctypes.c_void_p(t.data_ptr())


class CutAdvection:
    """Device operator of the cut advection problem on [left, right]^2.

    level_set: callable f(x, y) (vectorised) or the (n+1)^2 vertex values
    (x fastest); its FE_Q(1) interpolant defines inside (< 0).
    location: INSIDE (the field on phi < 0) or OUTSIDE (phi > 0); composite:
    the cut-surface inflow value is a partner field (couple()) instead of stage
    boundary data (include/gdm_hip.h gdm_cut_advection_create2)."""

    INSIDE, OUTSIDE = -1, 1  # GDM_CUT_INSIDE / GDM_CUT_OUTSIDE
    COMPOSITE = 1            # GDM_CUT_ADV_COMPOSITE

    def __init__(self, fe_degree, n_subdivisions, left, right, level_set, advection, ghost_parameter_A=0.5,
                 ghost_parameter_M=0.5, device=0, location=-1, composite=False):
        self._lib = _capi.load()
        self._h = ctypes.c_void_p()
        N = n_subdivisions + 1
        self.h = (right - left) / n_subdivisions
        xv = left + np.arange(N) * self.h
        if callable(level_set):
            X, Y = np.meshgrid(xv, xv, indexing="xy")
            ls = np.asarray(level_set(X.reshape(-1), Y.reshape(-1)), dtype=np.float64)
        else:
            ls = np.ascontiguousarray(level_set, dtype=np.float64).reshape(-1)
        if ls.shape[0] != N * N:
            raise GdmError("level_set: %d vertex values expected" % (N * N))
        a = (ctypes.c_double * 2)(*[float(v) for v in advection])
        self.location, self.composite = int(location), bool(composite)
        check(self._lib.gdm_cut_advection_create2(int(fe_degree), int(n_subdivisions), float(left), float(right),
                                                  ls.ctypes.data_as(ctypes.c_void_p), a, float(ghost_parameter_A),
                                                  float(ghost_parameter_M), self.location,
                                                  self.COMPOSITE if composite else 0, int(device),
                                                  ctypes.byref(self._h)),
              "gdm_cut_advection_create2")
        nd, nb, bw = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        cells = (ctypes.c_int64 * 3)()
        check(self._lib.gdm_cut_advection_info(self._h, ctypes.byref(nd), ctypes.byref(nb), cells, ctypes.byref(bw)),
              "gdm_cut_advection_info")
        self.n_dofs, self.n_bc_points, self.mass_bandwidth = nd.value, nb.value, bw.value
        self.cells = dict(inside=cells[0], intersected=cells[1], outside=cells[2])
        op = ctypes.c_void_p()
        check(self._lib.gdm_cut_advection_op(self._h, ctypes.byref(op)), "gdm_cut_advection_op")
        self._op = op
        self.device = device
        self.vertices = xv
        # order every launch after torch's work on the caller's stream (vector
        # allocation / copies), like GdmOperator does
        import torch

        s = torch.cuda.current_stream(device).cuda_stream
        check(self._lib.gdm_op_set_stream(self._op, ctypes.c_void_p(s)), "gdm_op_set_stream")

    def close(self):
        if self._h:
            self._lib.gdm_cut_advection_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bc_points(self):
        """(n_bc_points, 2) stage boundary points in the reference's point_counter order"""
        xy = np.zeros((max(self.n_bc_points, 1), 2))
        check(self._lib.gdm_cut_advection_bc_points(self._h, xy.ctypes.data_as(ctypes.c_void_p)),
              "gdm_cut_advection_bc_points")
        return xy[:self.n_bc_points]

    def new_vector(self, n=None):
        import torch

        return torch.zeros(self.n_dofs if n is None else n, dtype=torch.float64, device="cuda:%d" % self.device)

    def compute_rhs(self, u, bc, out):
        check(self._lib.gdm_cut_advection_compute_rhs(self._h, _ptr(u), _ptr(bc) if self.n_bc_points else None,
                                                      _ptr(out)), "gdm_cut_advection_compute_rhs")
        return out

    def couple(self, u_partner, out):
        """out += P u_partner: the partner field's inflow on the cut surface (composite)"""
        check(self._lib.gdm_cut_advection_couple(self._h, _ptr(u_partner), _ptr(out)), "gdm_cut_advection_couple")
        return out

    def mass_solve(self, rhs, x):
        check(self._lib.gdm_cut_advection_mass_solve(self._h, _ptr(rhs), _ptr(x)), "gdm_cut_advection_mass_solve")
        return x

    def rk_update(self, beta, k, acc_in, acc_out, alpha=0.0, y=None, Y=None):
        n = k.numel()
        check(self._lib.gdm_vec_rk_update(self._op, n, float(beta), _ptr(k), _ptr(acc_in), _ptr(acc_out),
                                          float(alpha), _ptr(y) if Y is not None else None,
                                          _ptr(Y) if Y is not None else None), "gdm_vec_rk_update")

    def synchronize(self):
        check(self._lib.gdm_synchronize(self._op), "gdm_synchronize")


class CutAdvectionProblem:
    """AdvectionProblem::run (problem.h:31-102, non-composite) on the device.
    exact(x, y, t) / exact_dt(x, y, t): the boundary function g and dg/dt
    (vectorised numpy), evaluated at the stage boundary points on the host."""

    def __init__(self, ca, exact, exact_dt):
        import torch

        self.ca, self.g, self.dg = ca, exact, exact_dt
        self.pts = ca.bc_points()
        nb = max(ca.n_bc_points, 1)
        self.u = ca.new_vector()
        self.bc = ca.new_vector(nb)
        self._acc = [ca.new_vector(nb), ca.new_vector()]
        self._Y = [ca.new_vector(nb), ca.new_vector()]
        self._k = [ca.new_vector(nb), ca.new_vector()]
        self._torch = torch

    def _upload(self, values, dst):
        t = self._torch.from_numpy(np.ascontiguousarray(values, dtype=np.float64))
        dst[:len(values)].copy_(t)

    def set_initial_condition(self, t=0.0):
        """GDM::VectorTools::interpolate: vertex values of g(t)"""
        X, Y = np.meshgrid(self.ca.vertices, self.ca.vertices, indexing="xy")
        self._upload(self.g(X.reshape(-1), Y.reshape(-1), t), self.u)

    def step(self, t, h):
        ca = self.ca
        x, y_ = self.pts[:, 0], self.pts[:, 1]
        self._upload(self.g(x, y_, t), self.bc)  # initialize_time_step
        y = (self.bc, self.u)
        acc, Y, k = self._acc, self._Y, self._k
        stage = y
        for s in range(4):
            ts = t + RK4_C[s] * h
            self._upload(self.dg(x, y_, ts), k[0])  # block(0) = dg/dt (stiffness.h:286-289)
            ca.compute_rhs(stage[1], stage[0], k[1])
            ca.mass_solve(k[1], k[1])
            last = s == 3
            a_next = 0.0 if last else h * RK4_A[s]
            for b in (0, 1):
                ca.rk_update(h * RK4_B[s], k[b], (y if s == 0 else acc)[b], (y if last else acc)[b], a_next,
                             None if last else y[b], None if last else Y[b])
            stage = Y

    def run(self, start_t, end_t, dt):
        self.set_initial_condition(start_t)
        time = DiscreteTime(start_t, end_t, dt)
        n = 0
        while not time.is_at_end():
            self.step(time.t, time.next_step_size())
            n += 1
            time.advance()
        self.ca.synchronize()
        return n


class CutAdvectionCompositeProblem:
    """AdvectionProblem::run, composite branch (problem.h:103-181) on the
    device: BlockVector (bc_in, u_in, bc_out, u_out), f = (dg/dt,
    M_in^-1 (rhs_in(u_in, bc_in) + P_in u_out), dg/dt, M_out^-1 (rhs_out +
    P_out u_in)), RK_CLASSIC_FOURTH_ORDER in the low-storage form (deal.II's
    summation order), both fields on one stream.  exact / exact_dt: g and
    dg/dt (vectorised numpy) at the stage boundary points of each field.
    The reference prints nothing for this preset (advection-app.cc), so the
    device run is checked against oracle/cut_advection2d.py's restatement:
    parity unpinned."""

    def __init__(self, p, n_sub, left, right, level_set, advection_in, advection_out, exact, exact_dt,
                 ghost_parameter_A=0.5, ghost_parameter_M=0.5, device=0):
        import torch

        self.f = [CutAdvection(p, n_sub, left, right, level_set, adv, ghost_parameter_A, ghost_parameter_M, device,
                               location=loc, composite=True)
                  for loc, adv in ((CutAdvection.INSIDE, advection_in), (CutAdvection.OUTSIDE, advection_out))]
        # one stream for both fields (the coupling reads the partner's stage)
        s = torch.cuda.current_stream(device).cuda_stream
        for ca in self.f:
            check(ca._lib.gdm_op_set_stream(ca._op, ctypes.c_void_p(s)), "gdm_op_set_stream")
        self.g, self.dg, self._torch = exact, exact_dt, torch
        self.pts = [ca.bc_points() for ca in self.f]
        nb = [max(ca.n_bc_points, 1) for ca in self.f]
        ca = self.f[0]
        sizes = [nb[0], ca.n_dofs, nb[1], ca.n_dofs]
        self.y = [ca.new_vector(n) for n in sizes]
        self._acc = [ca.new_vector(n) for n in sizes]
        self._Y = [ca.new_vector(n) for n in sizes]
        self._k = [ca.new_vector(n) for n in sizes]

    def _upload(self, values, dst):
        dst[:len(values)].copy_(self._torch.from_numpy(np.ascontiguousarray(values, dtype=np.float64)))

    def set_initial_condition(self, t=0.0):
        X, Y = np.meshgrid(self.f[0].vertices, self.f[0].vertices, indexing="xy")
        u0 = self.g(X.reshape(-1), Y.reshape(-1), t)
        self._upload(u0, self.y[1])
        self._upload(u0, self.y[3])

    def _rhs(self, t, stage, k):
        for i, (ca, pts) in enumerate(zip(self.f, self.pts)):
            bb, ub = 2 * i, 2 * i + 1
            if ca.n_bc_points:
                self._upload(self.dg(pts[:, 0], pts[:, 1], t), k[bb])
            ca.compute_rhs(stage[ub], stage[bb], k[ub])
            ca.couple(stage[3 - 2 * i], k[ub])  # the partner field's u
            ca.mass_solve(k[ub], k[ub])

    def step(self, t, h):
        y, acc, Y, k = self.y, self._acc, self._Y, self._k
        for i, (ca, pts) in enumerate(zip(self.f, self.pts)):  # initialize_time_step
            if ca.n_bc_points:
                self._upload(self.g(pts[:, 0], pts[:, 1], t), y[2 * i])
        stage = y
        ca = self.f[0]
        for s in range(4):
            self._rhs(t + RK4_C[s] * h, stage, k)
            last = s == 3
            a_next = 0.0 if last else h * RK4_A[s]
            for b in range(4):
                ca.rk_update(h * RK4_B[s], k[b], (y if s == 0 else acc)[b], (y if last else acc)[b], a_next,
                             None if last else y[b], None if last else Y[b])
            stage = Y

    def run(self, start_t, end_t, dt, max_steps=None):
        self.set_initial_condition(start_t)
        time = DiscreteTime(start_t, end_t, dt)
        n = 0
        while not time.is_at_end() and (max_steps is None or n < max_steps):
            self.step(time.t, time.next_step_size())
            n += 1
            time.advance()
        self.f[0].synchronize()
        return n
