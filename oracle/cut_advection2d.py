"""2D cut-cell GDM advection restatement (test infrastructure: only tests/ and
tools/ may import it) of the reference's advection application as
advection-convergence.cc runs it, i.e. the case that
applications/advection/tests/test_01.output prints ("parallel-ramp-degree",
advection-convergence.cc:229-250; SURVEY §4: the file is that case, not
advection-app).

What it restates (paths relative to the reference root):

  * parameters: unit square, n = 40, p = 3 (cfl 0.4) / 5 (cfl 0.1), end_t 0.1,
    ghost parameters gamma_M = gamma_A = 0.5, max_val 2, constant advection
    a = 2 (cos(phi + phi_add), sin(phi + phi_add)), exact solution
    sin(sqrt 2 pi x^ / (1 - x_shift)), x^ = cos phi (X - x_shift) + sin phi Y at
    X = x - t a, its time derivative, FE_Q(1) level set of
    SignedDistance::Plane((x_shift, 0), (sin phi, -cos phi))
                                        advection-convergence.cc:50-195
  * mesh, categories, DoF boxes, MeshClassifier, Saye quadrature of the cut
    cells: oracle/cut2d.py (pinned by prototypes/cut_poisson_01_gdm.output)
  * compute_rhs, non-composite, alpha = 0:
      (I)   cell:       (a u, grad v)_inside
      (II)  surface:    (a.n) (-(a.n >= 0 ? u : u+)) v on the cut surface,
                        u+ = stage boundary value
      (III) box faces:  the same upwind flux on the inside part of every
                        boundary face (NonMatching::FEInterfaceValues: QGauss
                        (p+1) on each inside sub-interval of the face)
      (IV)  ghost penalty: -0.5 gamma_A h^2 [d_n v][d_n u] on every interior
                        face with an intersected cell and a non-outside
                        neighbour, visited from both cells
                                        advection/stiffness.h:215-606
      block(0) = dg/dt at the boundary points, collected in the same
      cell / surface / face order (stiffness.h:40-160, 286-289)
  * mass: (v, u)_inside + 0.5 gamma_M h^3 [d_n v][d_n u] (both visits), zero
    diagonals -> 1                      advection/mass.h:47-243
  * AdvectionProblem::run: dt = h cfl / max_val, DiscreteTime(0, end_t, dt),
    initialize_time_step (block(0) = g(t_n)), RK_CLASSIC_FOURTH_ORDER with
    k = (dg/dt, M^-1 compute_rhs) -- the reference's SolverCG + Trilinos ILU to
    rel 1e-14 (problem.h:236-267) restated by an exact sparse LU solve; the
    CG's stopping rule leaves ~1e-13 in u (a Jacobi-CG to the same 1e-14
    moves the p = 5 surface norms, ~5e-8, by up to 4e-13), which is the
    tolerance of the golden comparison beyond the printed digits -- vertex
    interpolation of the initial condition, and the last postprocess' six
    norms: L2 / L1 / Linf of u_h - u over the inside quadrature and over the
    surface quadrature
                                        advection/problem.h:31-205, 269-485

Every operator is linear in (u, block(0)), so compute_rhs is assembled once as
sparse matrices K (u) and F (boundary values): the same sums as the
reference's cell loop, in matrix form.

Pinned to applications/advection/tests/test_01.output (all 18 rows x 6
columns) by tests/test_cut_advection_golden.py.
"""
import math

import numpy as np
import scipy.sparse as sps
import scipy.sparse.linalg as spla

import cut1d
import cut2d
import oracle as O

X_SHIFT = 0.2001


class CutAdvection2D:
    def __init__(self, p, n_sub, factor, factor_rotation=0.0, cfl=None, gamma_M=0.5, gamma_A=0.5, end_t=0.1):
        increment = 5.0
        self.phi = (math.pi * increment / 180.0) * factor
        self.phi_add = (math.pi * increment / 180.0) * factor_rotation
        self.rot = (increment * factor, increment * (factor + factor_rotation))
        self.p, self.n = p, n_sub
        self.cfl = cfl if cfl is not None else (0.4 if p == 3 else 0.1)
        self.gM, self.gA = gamma_M, gamma_A
        self.end_t = end_t
        self.a = np.array([2.0 * math.cos(self.phi + self.phi_add), 2.0 * math.sin(self.phi + self.phi_add)])
        # geometry / basis / Saye quadrature from the cut-Poisson restatement on [0, 1]^2
        self.geo = g = cut2d.CutPoisson2D(p, n_sub, 0.0, 1.0)
        self.h, self.N = g.h, g.N
        nrm = (math.sin(self.phi), -math.cos(self.phi))
        xx, yy = np.meshgrid(g.xv, g.xv, indexing="xy")  # [iy, ix]
        g.ls = (xx - X_SHIFT) * nrm[0] + yy * nrm[1]     # SignedDistance::Plane at the vertices
        for cy in range(n_sub):
            for cx in range(n_sub):
                v = g.ls[cy:cy + 2, cx:cx + 2]
                g.loc[cy, cx] = (cut2d.INSIDE if np.all(v < 0) else
                                 (cut2d.OUTSIDE if np.all(v > 0) else cut2d.INTERSECTED))
        self._assemble()

    # -- exact solution (advection-convergence.cc:50-117) -------------------
    def exact(self, x, y, t):
        X, Y = x - t * self.a[0], y - t * self.a[1]
        xh = math.cos(self.phi) * (X - X_SHIFT) + math.sin(self.phi) * Y
        return np.sin(math.sqrt(2.0) * math.pi * xh / (1.0 - X_SHIFT))

    def exact_dt(self, x, y, t):
        X, Y = x - t * self.a[0], y - t * self.a[1]
        xh = math.cos(self.phi) * (X - X_SHIFT) + math.sin(self.phi) * Y
        k = math.sqrt(2.0) * math.pi / (1.0 - X_SHIFT)
        return np.cos(k * xh) * k * (math.cos(self.phi) * (-self.a[0]) + math.sin(self.phi) * (-self.a[1]))

    # -- quadrature helpers --------------------------------------------------
    def _face_quadrature(self, cx, cy, f):
        """inside part of face f (0: s=0, 1: s=1, 2: t=0, 3: t=1) of a cell:
        [(s, t, JxW)] with QGauss(p+1) on every inside sub-interval"""
        g = self.geo
        v = g.ls[cy:cy + 2, cx:cx + 2]  # v[t][s]
        if f < 2:
            f0, f1 = v[0, f], v[1, f]
        else:
            f0, f1 = v[f - 2, 0], v[f - 2, 1]
        r = cut2d._linear_root(f0, f1)
        edges = [0.0] + ([r] if r is not None else []) + [1.0]
        out = []
        for a, b in zip(edges[:-1], edges[1:]):
            L = b - a
            if L <= 0.0:
                continue
            mid = f0 + (f1 - f0) * 0.5 * (a + b)
            if not mid < 0.0:
                continue
            for x, w in zip(g.qx, g.qw):
                c = a + L * x
                st = (float(f), c) if f < 2 else (c, float(f - 2))
                out.append((st[0], st[1], w * L * self.h))
        return out

    def _has_ghost_penalty(self, cx, cy, f):
        n = self.n
        nx, ny = [(cx - 1, cy), (cx + 1, cy), (cx, cy - 1), (cx, cy + 1)][f]
        if not (0 <= nx < n and 0 <= ny < n):
            return None
        a, b = self.geo.loc[cy, cx], self.geo.loc[ny, nx]
        I, O = cut2d.INTERSECTED, cut2d.OUTSIDE
        if (a == I and b != O) or (b == I and a != O):
            return nx, ny
        return None

    def _gp_face(self, cx, cy, f, nx, ny):
        """(dof indices of both cells, [n_dofs_both, nq] normal jumps of the
        shape gradients, JxW) of the full face f (FEInterfaceValues, QGauss)"""
        g = self.geo
        q, w = g.qx, g.qw
        side = f % 2
        if f < 2:
            sc, tc, sn, tn = np.full(len(q), float(side)), q, np.full(len(q), 1.0 - side), q
            nrm = np.array([-1.0 if side == 0 else 1.0, 0.0])
        else:
            sc, tc, sn, tn = q, np.full(len(q), float(side)), q, np.full(len(q), 1.0 - side)
            nrm = np.array([0.0, -1.0 if side == 0 else 1.0])
        _, gc = g.shapes(cx, cy, sc, tc)
        _, gn = g.shapes(nx, ny, sn, tn)
        jump = np.concatenate([np.einsum("d,diq->iq", nrm, gc), -np.einsum("d,diq->iq", nrm, gn)])
        idx = np.concatenate([g.dofs(cx, cy), g.dofs(nx, ny)])
        return idx, jump, w * self.h

    # -- assembly --------------------------------------------------------------
    def _assemble(self):
        g, p, n, h = self.geo, self.p, self.n, self.h
        ND = self.N * self.N
        Kr, Kc, Kv = [], [], []
        Mr, Mc, Mv = [], [], []
        Fr, Fc, Fv = [], [], []
        Pr, Pc, Pv = [], [], []  # composite: (II)'s inflow from the partner field
        composite = getattr(self, "composite", False)
        pts = []  # boundary points (x, y) in the reference's point_counter order

        def add(R, C, V, rows, cols, mat):
            R.append(np.repeat(rows, len(cols)))
            C.append(np.tile(cols, len(rows)))
            V.append(np.asarray(mat).reshape(-1))

        def upwind(d, val, flux, w):
            """flux (a.n) (-(a.n >= 0 ? u : u+)) v: K for outflow points, F columns for inflow ones"""
            for q in range(len(w)):
                if flux[q] >= 0.0:
                    add(Kr, Kc, Kv, d, d, -flux[q] * w[q] * np.outer(val[:, q], val[:, q]))
                else:
                    col = len(pts) - len(w) + q
                    add(Fr, Fc, Fv, d, np.array([col]), (-flux[q] * w[q] * val[:, q])[:, None])

        for cy in range(n):
            for cx in range(n):
                if g.loc[cy, cx] == cut2d.OUTSIDE:
                    continue
                d = g.dofs(cx, cy)
                ins, sur = g.cell_quadrature(cx, cy)
                if ins:
                    s, t, w = (np.array(c) for c in zip(*ins))
                    val, grad = g.shapes(cx, cy, s, t)
                    # (I): (a u_q) . grad phi_i JxW  ->  K[i, j] += sum_q (a . grad phi_i) phi_j w
                    ag = np.einsum("d,diq->iq", self.a, grad)
                    add(Kr, Kc, Kv, d, d, np.einsum("iq,jq,q->ij", ag, val, w))
                    add(Mr, Mc, Mv, d, d, np.einsum("iq,jq,q->ij", val, val, w))
                if sur:  # (II) cut surface, outward normal of the inside domain
                    s = np.array([c[0] for c in sur])
                    t = np.array([c[1] for c in sur])
                    w = np.array([c[2] for c in sur])
                    nr = np.array([c[3] for c in sur])
                    val, _ = g.shapes(cx, cy, s, t)
                    if composite:
                        # u+ = the partner field at the point (stiffness.h:448-453); no stage point (:115)
                        flux = nr @ self.a
                        for q in range(len(w)):
                            if flux[q] >= 0.0:
                                add(Kr, Kc, Kv, d, d, -flux[q] * w[q] * np.outer(val[:, q], val[:, q]))
                            else:
                                add(Pr, Pc, Pv, d, d, -flux[q] * w[q] * np.outer(val[:, q], val[:, q]))
                    else:
                        for q in range(len(w)):
                            pts.append(g.real_point(cx, cy, s[q], t[q]))
                        upwind(d, val, nr @ self.a, w)
                for f in range(4):  # (III) box faces
                    at_bnd = (f == 0 and cx == 0) or (f == 1 and cx == n - 1) or (f == 2 and cy == 0) or \
                             (f == 3 and cy == n - 1)
                    if not at_bnd:
                        continue
                    fq = self._face_quadrature(cx, cy, f)
                    if not fq:
                        continue
                    s, t, w = (np.array(c) for c in zip(*fq))
                    val, _ = g.shapes(cx, cy, s, t)
                    nrm = [(-1.0, 0.0), (1.0, 0.0), (0.0, -1.0), (0.0, 1.0)][f]
                    for q in range(len(w)):
                        pts.append(g.real_point(cx, cy, s[q], t[q]))
                    upwind(d, val, np.full(len(w), nrm[0] * self.a[0] + nrm[1] * self.a[1]), w)
                for f in range(4):  # (IV) ghost penalty, stiffness (h^2) and mass (h^3)
                    nb = self._has_ghost_penalty(cx, cy, f)
                    if nb is None:
                        continue
                    idx, jump, jw = self._gp_face(cx, cy, f, *nb)
                    S = np.einsum("iq,jq,q->ij", jump, jump, jw)
                    add(Kr, Kc, Kv, idx, idx, -0.5 * self.gA * h * h * S)
                    add(Mr, Mc, Mv, idx, idx, 0.5 * self.gM * h * h * h * S)
        cat = lambda L: np.concatenate(L) if L else np.zeros(0)  # noqa: E731
        self.K = sps.csr_matrix((cat(Kv), (cat(Kr).astype(np.int64), cat(Kc).astype(np.int64))), shape=(ND, ND))
        M = sps.csr_matrix((cat(Mv), (cat(Mr).astype(np.int64), cat(Mc).astype(np.int64))), shape=(ND, ND)).tolil()
        diag = M.diagonal()
        for i in np.flatnonzero(diag == 0.0):
            M[i, i] = 1.0
        self.M = M.tocsc()
        self.points = np.array(pts) if pts else np.zeros((0, 2))
        self.F = sps.csr_matrix((cat(Fv), (cat(Fr).astype(np.int64), cat(Fc).astype(np.int64))),
                                shape=(ND, len(pts)))
        Mc = self.M.tocsr()
        Mc.sort_indices()
        self._csr = (Mc.indptr.astype(np.int64), Mc.indices.astype(np.int64), Mc.data)
        self.P = sps.csr_matrix((cat(Pv), (cat(Pr).astype(np.int64), cat(Pc).astype(np.int64))), shape=(ND, ND))

    def solve(self, b, exact=True):
        """M^-1 b by sparse LU (exact=False: SolverCG + PreconditionJacobi,
        ReductionControl(1000, 1e-20, 1e-14) from zero, for the spread study)"""
        if exact:
            if not hasattr(self, "_lu"):
                self._lu = spla.splu(self.M)
            return self._lu.solve(b)
        rp, ci, v = self._csr
        x, its = O.cg(rp, ci, v, b, precond=1, max_it=1000, abs_tol=1e-20, rel_tol=1e-14)
        if its < 0:
            raise RuntimeError("mass CG did not converge")
        return x

    # -- time loop (problem.h:40-102) ----------------------------------------
    def compute_rhs(self, u, bc):
        return self.K @ u + self.F @ bc

    def run(self, exact_solve=True):
        g, nb = self.geo, len(self.points)
        X, Y = np.meshgrid(g.xv, g.xv, indexing="xy")
        u = self.exact(X.reshape(-1), Y.reshape(-1), 0.0)  # GDM::VectorTools::interpolate at t = 0
        px, py = self.points[:, 0], self.points[:, 1]
        dt = self.h * self.cfl / 2.0
        time = cut1d.DiscreteTime(0.0, self.end_t, dt)

        def f(t, y):
            return np.concatenate([self.exact_dt(px, py, t), self.solve(self.compute_rhs(y[nb:], y[:nb]), exact_solve)])

        while not time.is_at_end():
            y = np.concatenate([self.exact(px, py, time.t), u])  # initialize_time_step
            y = cut1d.rk4_step(f, time.t, time.next_step_size(), y)
            u = y[nb:]
            t_end = time.t + time.next_step_size()
            time.advance()
        self.u, self.t_end, self.steps = u, t_end, time.step
        return self.errors(u, t_end)

    # -- postprocess (problem.h:269-485) --------------------------------------
    def errors(self, u, t):
        """(Linf, L1, L2, Linf_face, L1_face, L2_face) of u_h - u(t)"""
        g = self.geo
        e = [0.0] * 6
        for cy in range(self.n):
            for cx in range(self.n):
                if g.loc[cy, cx] == cut2d.OUTSIDE:
                    continue
                ins, sur = g.cell_quadrature(cx, cy)
                for quad, off in ((ins, 0), (sur, 3)):
                    if not quad:
                        continue
                    s = np.array([c[0] for c in quad])
                    tt = np.array([c[1] for c in quad])
                    w = np.array([c[2] for c in quad])
                    val, _ = g.shapes(cx, cy, s, tt)
                    x, y = g.real_point(cx, cy, s, tt)
                    err = u[g.dofs(cx, cy)] @ val - self.exact(x, y, t)
                    e[off] = max(e[off], float(np.max(np.abs(err))))
                    e[off + 1] += float(np.sum(np.abs(err) * w))
                    e[off + 2] += float(np.sum(err * err * w))
        e[2], e[5] = math.sqrt(e[2]), math.sqrt(e[5])
        return tuple(e)


class CutAdvectionField(CutAdvection2D):
    """One field of the composite application (advection-app.cc:99-152;
    problem.h:103-181): the same assembly on [lo, hi]^2 for the given vertex
    level set and advection.  The outside field (location outside) is this
    assembly on the negated level set: its inside is the outside region, the
    face parts and MeshClassifier follow the sign, the Saye surface points of
    a bilinear level set are the same and its normal is the flipped one of
    stiffness.h:437, the ghost-penalty faces those of the inverse location
    (stiffness.h:260-280, mass.h:67-104).  composite: (II)'s inflow is P
    u_partner."""

    def __init__(self, p, n_sub, lo, hi, ls_vertex, a, composite=True, gamma_M=0.5, gamma_A=0.5):
        self.p, self.n = p, n_sub
        self.gM, self.gA = gamma_M, gamma_A
        self.a = np.asarray(a, dtype=np.float64)
        self.composite = composite
        self.geo = g = cut2d.CutPoisson2D(p, n_sub, lo, hi)
        self.h, self.N = g.h, g.N
        g.ls = np.asarray(ls_vertex, dtype=np.float64).reshape(self.N, self.N)
        for cy in range(n_sub):
            for cx in range(n_sub):
                v = g.ls[cy:cy + 2, cx:cx + 2]
                g.loc[cy, cx] = (cut2d.INSIDE if np.all(v < 0) else
                                 (cut2d.OUTSIDE if np.all(v > 0) else cut2d.INTERSECTED))
        self._assemble()

    def exact(self, x, y, t):
        return app_exact(x, y, t)


def app_exact(x, y, t=0.0):
    """advection-app.cc:50-64: max(0, 0.3 - |p - (-0.3, -0.3)|), time independent"""
    return np.maximum(0.0, 0.3 - np.hypot(np.asarray(x) + 0.3, np.asarray(y) + 0.3))


def app_exact_dt(x, y, t=0.0):
    """advection-app.cc:66-81: 0"""
    return np.zeros_like(np.asarray(x, dtype=np.float64))


class CompositeAdvection2D:
    """AdvectionProblem::run, composite branch (problem.h:103-181) with
    advection-app.cc's preset (factor 27: phi = 135 deg, x_shift 0.25, level
    set SignedDistance::Plane((x_shift, 0), (sin phi, -cos phi)), a = (3, 1)
    inside, (1, 2) outside, p = 5, [-1, 1]^2, gamma_M = gamma_A = 0.5, cfl 0.2,
    max_val 4, end_t 0.6; n_sub = 200 in the preset, any n here).  Block vector
    (bc_in, u_in, bc_out, u_out), f = (dg/dt, M_in^-1 (K_in u_in + F_in bc_in +
    P_in u_out), dg/dt, M_out^-1 (...)), RK_CLASSIC_FOURTH_ORDER over the whole
    block vector, DiscreteTime, the loop's error[2] < 1 guard.  The mass solves
    are the reference's SolverDirect branch (sparse LU).  The reference prints
    nothing for this preset: parity unpinned beyond the non-composite pins
    of the shared assembly (test_01.output)."""

    def __init__(self, p=5, n_sub=200, end_t=0.6, cfl=0.2, factor=27.0, x_shift=0.25, a_in=(3.0, 1.0),
                 a_out=(1.0, 2.0), lo=-1.0, hi=1.0, gamma_M=0.5, gamma_A=0.5, max_val=4.0):
        phi = (math.pi * 5.0 / 180.0) * factor
        nrm = (math.sin(phi), -math.cos(phi))
        h = (hi - lo) / n_sub
        xv = lo + np.arange(n_sub + 1) * h
        xx, yy = np.meshgrid(xv, xv, indexing="xy")
        self.ls = ((xx - x_shift) * nrm[0] + yy * nrm[1]).reshape(-1)
        self.fields = [CutAdvectionField(p, n_sub, lo, hi, self.ls, a_in, True, gamma_M, gamma_A),
                       CutAdvectionField(p, n_sub, lo, hi, -self.ls, a_out, True, gamma_M, gamma_A)]
        self.dt = h * cfl / max_val
        self.end_t, self.xv = end_t, xv

    def rhs(self, t, y):
        """the field blocks of fu_rhs before the mass solves: [rhs_in, rhs_out]"""
        nb = [len(f.points) for f in self.fields]
        bc_in, u_in = y[:nb[0]], y[nb[0]:nb[0] + self.n]
        o = nb[0] + self.n
        bc_out, u_out = y[o:o + nb[1]], y[o + nb[1]:]
        fi, fo = self.fields
        return (fi.K @ u_in + fi.F @ bc_in + fi.P @ u_out, fo.K @ u_out + fo.F @ bc_out + fo.P @ u_in)

    @property
    def n(self):
        return self.fields[0].N ** 2

    def run(self, max_steps=None):
        fi, fo = self.fields
        pin, pout = fi.points, fo.points
        nb = [len(pin), len(pout)]
        X, Y = np.meshgrid(self.xv, self.xv, indexing="xy")
        u0 = app_exact(X.reshape(-1), Y.reshape(-1))
        u_in, u_out = u0.copy(), u0.copy()
        time = cut1d.DiscreteTime(0.0, self.end_t, self.dt)

        def bcs(t):
            return (app_exact(pin[:, 0], pin[:, 1], t) if nb[0] else np.zeros(0),
                    app_exact(pout[:, 0], pout[:, 1], t) if nb[1] else np.zeros(0))

        def f(t, y):
            r_in, r_out = self.rhs(t, y)
            d_in = app_exact_dt(pin[:, 0], pin[:, 1], t) if nb[0] else np.zeros(0)
            d_out = app_exact_dt(pout[:, 0], pout[:, 1], t) if nb[1] else np.zeros(0)
            return np.concatenate([d_in, fi.solve(r_in), d_out, fo.solve(r_out)])

        rows = [(0, 0.0) + self.errors(u_in, u_out, 0.0)]
        steps = 0
        # the loop guard error[2] < 1: L2 of the outside field's postprocess, row entry 2 + 6 + 2
        while not time.is_at_end() and rows[-1][10] < 1.0 and (max_steps is None or steps < max_steps):
            b_in, b_out = bcs(time.t)  # initialize_time_step
            y = np.concatenate([b_in, u_in, b_out, u_out])
            y = cut1d.rk4_step(f, time.t, time.next_step_size(), y)
            u_in = y[nb[0]:nb[0] + self.n]
            u_out = y[nb[0] + self.n + nb[1]:]
            t_end = time.t + time.next_step_size()
            time.advance()
            steps += 1
            rows.append((steps, t_end) + self.errors(u_in, u_out, t_end))
        self.u_in, self.u_out, self.steps = u_in, u_out, steps
        return rows

    def errors(self, u_in, u_out, t):
        """postprocess(inside) then postprocess(outside) (problem.h:150-175): the six norms (Linf, L1, L2,
        Linf_face, L1_face, L2_face) of each field"""
        return tuple(self.fields[0].errors(u_in, t)) + tuple(self.fields[1].errors(u_out, t))


def table_row(p, factor, n_sub=40):
    """one row of advection-convergence.cc's "parallel-ramp-degree" table:
    (fe_degree, cfl, n_subdivision, rot_0, rot_1, error_2, error_1, error_inf,
    error_2_face, error_1_face, error_inf_face)"""
    P = CutAdvection2D(p, n_sub, factor)
    linf, l1, l2, linf_f, l1_f, l2_f = P.run()
    return (p, P.cfl, n_sub, P.rot[0], P.rot[1], l2, l1, linf, l2_f, l1_f, linf_f)
