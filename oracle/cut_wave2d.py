"""2D cut-cell restatement of the reference's wave application for dim = 2
with FE_Q(k) level sets (test infrastructure: only tests/ may import it).

Restates what applications/wave computes for the presets "wave" (wave-rk)
and "step85" (poisson) at dim = 2 (paths relative to the reference root):

  * mesh + categories + DoF boxes      include/gdm/system.h:195-246, 404-424
  * level set: FE_Q(k) (Gauss-Lobatto support points) interpolant of
    SignedDistance::Sphere (|x| - 1)   applications/wave/include/gdm/wave/discretization.h:78-93
  * NonMatching::MeshClassifier: the cell's Lagrange values mapped to the
    Bernstein basis of degree k; all coefficients < 0 inside, all > 0
    outside, else intersected
  * NonMatching::FEValues: QGauss(p+1)^2 on inside cells; on intersected
    cells deal.II's QuadratureGenerator (Saye's algorithm) on the cell's
    tensor-product level-set polynomial in reference coordinates:
      - value bounds: second-order Taylor estimate at the box centre widened
        by the vertex values; gradient bounds from the Hessian at the centre;
        definite if the value bounds exclude [-1e-11, 1e-11]
      - height direction: the largest lower bound of |df/dx_i| (first of
        equal ones), used if > 1e-11; ties within 1e-12 relative (cells
        symmetric about a diagonal, where deal.II's choice is decided by
        round-off) take direction 0 unless tie_hdir overrides them;
        else the box is split in halves along its longest side (at most 4
        splits), then the midpoint rule
      - the cross-section split at the roots of the level set restricted to
        the bottom and top faces (RootFinder: sign change at the ends ->
        root; else Taylor bounds, up to 2 interval halvings), QGauss(p+1) per
        sub-interval; sub-intervals negative on both faces get QGauss(p+1) over
        the whole height, indefinite ones are lifted point by point: the line
        split at its roots, QGauss(p+1) on every negative segment, one surface
        point at the root with weight w |grad f| / |df/dx_h| and normal
        grad f / |grad f|
    (deal.II source/non_matching/{mesh_classifier,quadrature_generator}.cc;
    deal.II is not vendored in the reference: restated from its published
    algorithm, R. Saye, SIAM J. Sci. Comput. 37 (2015) A993)
  * mass (v, u)_inside + 0.5 g_M h^3 [d_n v][d_n u], zero diagonals -> 1
                                       .../wave/mass.h:47-249
  * compute_rhs: -(grad v, grad u) + (v, f) + surface Nitsche (gamma_D = 5p)
    - 0.5 g_A h [d_n v][d_n u] (h^1 in the rhs)   .../wave/stiffness.h:42-407
  * stiffness matrix: (grad v, grad u) + surface Nitsche + 0.5 g_A h^3
    [d_n v][d_n u], zero diagonals -> 1    .../wave/stiffness.h:602-800
  * wave-rk (RK_CLASSIC_FOURTH_ORDER + DiscreteTime) and poisson (one
    stiffness solve)                   .../wave/problem.h:39-110, 283-346
  * postprocess: L2 / L1 / Linf on the inside quadrature   .../wave/problem.h:504-615
  * parameters of "wave" and "step85"  applications/wave/wave-app.cc:13-57, 215-262

Solves are exact (sparse LU) where the reference runs CG + AMG to
ReductionControl(1000, 1e-20, 1e-14) (the "[L] solved in 2-3" lines).  Roots
are bisected to machine precision where deal.II's toms748 stops at a bracket
of 1e-12 (reference coordinates).  Box splits do not occur on the presets'
meshes (counted in QGen.n_splits; the split direction rule is restated
unverified).  Pinned to applications/wave/tests/{wave_1,step85_0}.output by
tests/test_cut_wave2d_golden.py.
"""
import math

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla
import scipy.special

import oracle as O
from cut1d import DiscreteTime, gauss, gauss_lobatto, rk4_step

INSIDE, INTERSECTED, OUTSIDE = -1, 0, 1
LIMIT = 1e-11            # limit_to_be_definite, lower_bound_implicit_function
MAX_BOX_SPLITS = 4
MAX_ROOT_SPLITS = 2
ROOT_TOL = 1e-12


def lagrange_to_monomial(nodes):
    """A[a, i]: L_a(s) = sum_i A[a, i] s^i"""
    return np.linalg.inv(np.vander(nodes, increasing=True)).T


def lagrange_to_bernstein(nodes):
    """T: Bernstein coefficients = T @ Lagrange values (1D, degree len(nodes)-1)"""
    k = len(nodes) - 1
    B = np.array([[math.comb(k, i) * s ** i * (1 - s) ** (k - i) for i in range(k + 1)] for s in nodes])
    return np.linalg.inv(B)


class TensorPoly:
    """f(s, t) = sum_ij C[i, j] s^i t^j on the unit square: the FE_Q(k)
    interpolant of one cell from its values vals[a, b] at (s_a, t_b)."""

    def __init__(self, A, vals):
        self.C = A.T @ vals @ A
        self.k = self.C.shape[0] - 1

    def _pw(self, x):
        k = self.k
        p = np.array([x ** i for i in range(k + 1)])
        d = np.array([i * x ** (i - 1) if i > 0 else 0.0 for i in range(k + 1)])
        d2 = np.array([i * (i - 1) * x ** (i - 2) if i > 1 else 0.0 for i in range(k + 1)])
        return p, d, d2

    def value(self, s, t):
        ps, _, _ = self._pw(s)
        pt, _, _ = self._pw(t)
        return float(ps @ self.C @ pt)

    def grad(self, s, t):
        ps, ds, _ = self._pw(s)
        pt, dt, _ = self._pw(t)
        return np.array([ds @ self.C @ pt, ps @ self.C @ dt])

    def hess(self, s, t):
        ps, ds, d2s = self._pw(s)
        pt, dt, d2t = self._pw(t)
        return np.array([[d2s @ self.C @ pt, ds @ self.C @ dt], [ds @ self.C @ dt, ps @ self.C @ d2t]])


def _indefinite(lo, hi):
    return not (lo > 0.0 or hi < 0.0)


def _lower_abs(lo, hi):
    return min(abs(lo), abs(hi)) if (lo > 0.0 or hi < 0.0) else 0.0


def _refine_root(g, a, b, fa):
    """bisection of a sign-changing bracket to machine precision"""
    if fa == 0.0:
        return a
    for _ in range(200):
        m = 0.5 * (a + b)
        if m == a or m == b:
            break
        fm = g(m)
        if fm == 0.0:
            return m
        if (fm < 0.0) == (fa < 0.0):
            a, fa = m, fm
        else:
            b = m
    return 0.5 * (a + b)


def find_roots(g, dg, d2g, a, b, depth=0, out=None):
    """RootFinder::find_roots of one 1D function on [a, b]"""
    if out is None:
        out = []
    fa, fb = g(a), g(b)
    if np.sign(fa) != np.sign(fb):
        out.append(_refine_root(g, a, b, fa))
        return out
    c, dx = 0.5 * (a + b), 0.5 * (b - a)
    v = g(c)
    spread = abs(dg(c)) * dx + 0.5 * abs(d2g(c)) * dx * dx
    if not _indefinite(v - spread, v + spread):
        return out
    if depth < MAX_ROOT_SPLITS:
        find_roots(g, dg, d2g, a, c, depth + 1, out)
        find_roots(g, dg, d2g, c, b, depth + 1, out)
    return out


def _unique_sorted(roots):
    roots = sorted(roots)
    out = []
    for r in roots:
        if not out or abs(r - out[-1]) >= ROOT_TOL:
            out.append(r)
    return out


class QGen:
    """QuadratureGenerator<2> for one TensorPoly on a box in reference
    coordinates: inside [(s, t, w)] (f < 0), outside [(s, t, w)] (f > 0),
    surface [(s, t, w, normal)]; deal.II fills q_partitioning.negative /
    .positive in the same pass, a point whose level set is exactly 0 goes to
    neither."""

    def __init__(self, f, qx, qw, tie=0):
        self.f, self.qx, self.qw, self.tie = f, qx, qw, tie
        self.inside, self.outside, self.surface = [], [], []
        self.n_splits = 0
        self.n_midpoint = 0
        self.n_ties = 0

    def _tensor(self, lo, hi, dst):
        L0, L1 = hi[0] - lo[0], hi[1] - lo[1]
        for b, wb in zip(self.qx, self.qw):
            for a, wa in zip(self.qx, self.qw):
                dst.append((lo[0] + L0 * a, lo[1] + L1 * b, wa * wb * L0 * L1))

    def _restriction(self, hdir, hval):
        """the level set on the line x_hdir = hval as a function of the other coordinate"""
        f = self.f
        if hdir == 1:
            return (lambda c: f.value(c, hval), lambda c: f.grad(c, hval)[0], lambda c: f.hess(c, hval)[0, 0])
        return (lambda c: f.value(hval, c), lambda c: f.grad(hval, c)[1], lambda c: f.hess(hval, c)[1, 1])

    def generate(self, lo, hi, n_box_splits=0):
        f = self.f
        c = 0.5 * (np.asarray(lo) + np.asarray(hi))
        dx = 0.5 * (np.asarray(hi) - np.asarray(lo))
        val, g, H = f.value(*c), f.grad(*c), f.hess(*c)
        spread = abs(g[0]) * dx[0] + abs(g[1]) * dx[1] + 0.5 * sum(
            abs(H[i, j]) * dx[i] * dx[j] for i in range(2) for j in range(2))
        vmin, vmax = val - spread, val + spread
        for vs in (lo[0], hi[0]):
            for vt in (lo[1], hi[1]):
                fv = f.value(vs, vt)
                vmin, vmax = min(vmin, fv), max(vmax, fv)
        if vmin > LIMIT:
            self._tensor(lo, hi, self.outside)
            return
        if vmax < -LIMIT:
            self._tensor(lo, hi, self.inside)
            return
        low = []
        for i in range(2):
            dg = abs(H[i, 0]) * dx[0] + abs(H[i, 1]) * dx[1]
            low.append(_lower_abs(g[i] - dg, g[i] + dg))
        # first of equal ones; equal within 1e-12 relative (cells symmetric about a diagonal tie up to round-off)
        if abs(low[1] - low[0]) <= 1e-12 * max(low):
            hdir = self.tie
            self.n_ties += 1
        else:
            hdir = 1 if low[1] > low[0] else 0
        if low[hdir] > LIMIT:
            self._height(hdir, lo, hi)
        elif n_box_splits < MAX_BOX_SPLITS:
            self.n_splits += 1
            d = 0 if (hi[0] - lo[0]) >= (hi[1] - lo[1]) else 1
            mid = 0.5 * (lo[d] + hi[d])
            hi_l, lo_r = list(hi), list(lo)
            hi_l[d], lo_r[d] = mid, mid
            self.generate(lo, tuple(hi_l), n_box_splits + 1)
            self.generate(tuple(lo_r), hi, n_box_splits + 1)
        else:
            self.n_midpoint += 1
            fc = f.value(*c)
            if fc != 0.0:
                (self.inside if fc < 0.0 else self.outside).append((c[0], c[1], (hi[0] - lo[0]) * (hi[1] - lo[1])))

    def _height(self, hdir, lo, hi):
        f = self.f
        cdir = 1 - hdir
        c_lo, c_hi, h_lo, h_hi = lo[cdir], hi[cdir], lo[hdir], hi[hdir]

        def point(cc, hh):
            return (cc, hh) if cdir == 0 else (hh, cc)

        bottom, top = self._restriction(hdir, h_lo), self._restriction(hdir, h_hi)
        roots = []
        for r in (bottom, top):
            find_roots(*r, c_lo, c_hi, 0, roots)
        edges = [c_lo] + _unique_sorted(roots) + [c_hi]
        Lh = h_hi - h_lo
        for a, b in zip(edges[:-1], edges[1:]):
            L = b - a
            if not L > 0.0:
                continue
            m = 0.5 * (a + b)
            sb, st = bottom[0](m), top[0](m)
            for x, w in zip(self.qx, self.qw):
                cc, wc = a + L * x, w * L
                if (sb < 0.0 and st < 0.0) or (sb > 0.0 and st > 0.0):
                    dst = self.inside if sb < 0.0 else self.outside
                    for y, wy in zip(self.qx, self.qw):
                        dst.append(point(cc, h_lo + Lh * y) + (wc * wy * Lh,))
                    continue
                line = (lambda hh, cc=cc: f.value(*point(cc, hh)),
                        lambda hh, cc=cc: f.grad(*point(cc, hh))[hdir],
                        lambda hh, cc=cc: f.hess(*point(cc, hh))[hdir, hdir])
                hr = _unique_sorted(find_roots(*line, h_lo, h_hi))
                hs = [h_lo] + hr + [h_hi]
                for ha, hb in zip(hs[:-1], hs[1:]):
                    Ls = hb - ha
                    if not Ls > 0.0:
                        continue
                    fm = f.value(*point(cc, 0.5 * (ha + hb)))
                    if fm != 0.0:
                        dst = self.inside if fm < 0.0 else self.outside
                        for y, wy in zip(self.qx, self.qw):
                            dst.append(point(cc, ha + Ls * y) + (wc * wy * Ls,))
                if len(hr) == 1:
                    s, t = point(cc, hr[0])
                    gr = f.grad(s, t)
                    ng = math.hypot(gr[0], gr[1])
                    self.surface.append((s, t, wc * ng / abs(gr[hdir]), gr / ng))


class CutWave2D:
    """The wave application's discretization on [left, right]^2 (GDM degree
    p, level set FE_Q(k) of |x| - 1)."""

    def __init__(self, p=3, n=40, left=-1.21, right=1.21, k=None, level_set=None, tie_hdir=None):
        self.p, self.n = p, n
        self.k = p if k is None else k
        self.h = (right - left) / n
        self.N = n + 1
        self.left = left
        self.xv = np.array([left + i * self.h for i in range(self.N)])
        self.qx, self.qw = gauss(p + 1)
        self.level_set = level_set or (lambda x, y: math.hypot(x, y) - 1.0)
        gl = gauss_lobatto(self.k + 1)
        self.gl = gl
        A = lagrange_to_monomial(gl)
        T = lagrange_to_bernstein(gl)
        self.coef = {cat: [np.asarray(O.basis_coefficients(p, cat, i)) for i in range(p + 1)] for cat in range(p)}
        self.loc = np.zeros((n, n), dtype=int)
        self.quad = {}
        self.n_splits = self.n_midpoint = 0
        self.ties = []  # cells whose height direction was a tie
        self.ls_values = np.zeros((n, n, self.k + 1, self.k + 1))  # [cy, cx, b (t), a (s)]
        for cy in range(n):
            for cx in range(n):
                x0, y0 = self.xv[cx], self.xv[cy]
                vals = np.array([[self.level_set(x0 + s * self.h, y0 + t * self.h) for t in gl] for s in gl])  # [a, b]
                self.ls_values[cy, cx] = vals.T
                bern = T @ vals @ T.T
                if bern.max() < 0.0:
                    self.loc[cy, cx] = INSIDE
                elif bern.min() > 0.0:
                    self.loc[cy, cx] = OUTSIDE
                else:
                    self.loc[cy, cx] = INTERSECTED
                    q = QGen(TensorPoly(A, vals), self.qx, self.qw, (tie_hdir or {}).get((cx, cy), 0))
                    q.generate((0.0, 0.0), (1.0, 1.0))
                    if q.n_ties:
                        self.ties.append((cx, cy))
                    self.n_splits += q.n_splits
                    self.n_midpoint += q.n_midpoint
                    self.quad[(cx, cy)] = (q.inside, q.surface, q.outside)

    # -- GDM indexing (system.h:195-246, 404-424) --------------------------
    def category(self, c):
        p, n = self.p, self.n
        return c if c < p // 2 else (p // 2 if c < n - p // 2 else p + c - n)

    def offset(self, c):
        p, n = self.p, self.n
        return 0 if c < p // 2 else min(n, c + p // 2 + 1) - p

    def dofs(self, cx, cy):
        ox, oy = self.offset(cx), self.offset(cy)
        k = np.arange(self.p + 1)
        return ((oy + k)[:, None] * self.N + (ox + k)[None, :]).reshape(-1)

    def _basis_1d(self, cat, s, order):
        s = np.atleast_1d(np.asarray(s, dtype=float))
        out = np.zeros((self.p + 1, s.size))
        for i, c in enumerate(self.coef[cat]):
            cc = np.polynomial.polynomial.polyder(c, order) if order else c
            out[i] = np.polynomial.polynomial.polyval(s, cc)
        return out

    def shapes(self, cx, cy, s, t):
        """values [n_dofs, nq], gradients [2, n_dofs, nq] (real coordinates)"""
        cxat, cyat = self.category(cx), self.category(cy)
        vx, dx = self._basis_1d(cxat, s, 0), self._basis_1d(cxat, s, 1) / self.h
        vy, dy = self._basis_1d(cyat, t, 0), self._basis_1d(cyat, t, 1) / self.h
        val = (vy[:, None, :] * vx[None, :, :]).reshape(-1, vx.shape[1])
        gx = (vy[:, None, :] * dx[None, :, :]).reshape(-1, vx.shape[1])
        gy = (dy[:, None, :] * vx[None, :, :]).reshape(-1, vx.shape[1])
        return val, np.stack([gx, gy])

    def cell_quadrature(self, cx, cy, location=INSIDE):
        """the region's quadrature [(s, t, JxW)] and the surface [(s, t, JxW,
        level-set normal)] of one cell"""
        loc, h = self.loc[cy, cx], self.h
        if loc == -location:
            return [], []
        if loc == location:
            return [(a, b, wa * wb * h * h) for b, wb in zip(self.qx, self.qw) for a, wa in zip(self.qx, self.qw)], []
        ins, sur, out = self.quad[(cx, cy)]
        reg = ins if location == INSIDE else out
        return [(s, t, w * h * h) for s, t, w in reg], [(s, t, w * h, nn) for s, t, w, nn in sur]

    def boundary_faces(self, cx, cy, location):
        """(axis, side) of the cell's faces on the domain boundary that lie in
        the region of `location` (NonMatching::FEInterfaceValues on the face:
        MeshClassifier's face location, the Bernstein coefficients of the
        level set restricted to the face)"""
        n, k, out = self.n, self.k, []
        T = lagrange_to_bernstein(self.gl)
        for axis, side in ((0, 0), (0, 1), (1, 0), (1, 1)):
            c = (cx, cy)[axis]
            if c != (0 if side == 0 else n - 1):
                continue
            v = self.ls_values[cy, cx]  # [b (t), a (s)]
            line = v[:, 0 if side == 0 else k] if axis == 0 else v[0 if side == 0 else k, :]
            bern = T @ line
            if bern.max() < 0.0:
                where = INSIDE
            elif bern.min() > 0.0:
                where = OUTSIDE
            else:
                raise NotImplementedError("intersected domain boundary face (the level set crosses the box)")
            if where == location:
                out.append((axis, side))
        return out

    def real_point(self, cx, cy, s, t):
        return self.xv[cx] + np.asarray(s) * self.h, self.xv[cy] + np.asarray(t) * self.h

    # -- ghost-penalty faces (mass.h:86-105 / stiffness.h:80-98) ------------
    def gp_faces(self, location=INSIDE):
        """(cell, neighbour, axis, side) per visit for the field of
        `location`; each qualifying face is visited from both cells"""
        n, out, inv = self.n, [], -location
        for cy in range(n):
            for cx in range(n):
                a = self.loc[cy, cx]
                if a == inv:
                    continue
                for f, (nx, ny) in enumerate(((cx - 1, cy), (cx + 1, cy), (cx, cy - 1), (cx, cy + 1))):
                    if not (0 <= nx < n and 0 <= ny < n):
                        continue
                    b = self.loc[ny, nx]
                    if (a == INTERSECTED and b != inv) or (b == INTERSECTED and a != inv):
                        out.append(((cx, cy), (nx, ny), f // 2, f % 2))
        return out

    def _face_jump(self, c, nb, axis, side):
        """(global DoFs, [n_dofs, nq] normal-derivative jumps, JxW) on the face"""
        q = self.qx
        if axis == 0:
            sc, tc, sn, tn = np.full(q.size, float(side)), q, np.full(q.size, 1.0 - side), q
        else:
            sc, tc, sn, tn = q, np.full(q.size, float(side)), q, np.full(q.size, 1.0 - side)
        _, gc = self.shapes(*c, sc, tc)
        _, gn = self.shapes(*nb, sn, tn)
        idx = np.concatenate([self.dofs(*c), self.dofs(*nb)])
        return idx, np.concatenate([gc[axis], -gn[axis]]), self.qw * self.h

    # -- operators ------------------------------------------------------------
    def matrices(self, gamma_M, gamma_A, nitsche, location=INSIDE, interface_data=True, domain_data=False,
                 coupled=False):
        """the field of `location`: mass M (None if gamma_M < 0), stiffness K,
        impl operator A (compute_rhs(u) = -A u + data), load pieces Ff
        [N, nq] (JxW folded), Fg [N, n_data] (the Dirichlet data points: the
        surface points with interface_data (II, stiffness.h:205-259, normal
        flipped for the outside field), the Gauss points of the boundary
        faces in the region with domain_data (IV, :262-330)); with coupled the
        composite interface terms of compute_rhs(BlockVector) (:420-575): the
        own field's part in A, the partner's rhs contribution X (r += X
        u_other); evaluation E [nq, N]; the region's and data points"""
        p, h, N2 = self.p, self.h, self.N * self.N
        Mt, Kt, At, Xt, fft, fgt, et = [], [], [], [], [], [], []
        qpts, spts = [], []
        sg = 1.0 if location == INSIDE else -1.0
        tau = 0.5 * nitsche / h

        def add(T, rows, cols, V):
            T.append((np.repeat(rows, len(cols)), np.tile(cols, len(rows)), V.reshape(-1)))

        def nitsche_points(d, val, dn, w, pts):
            """Dirichlet Nitsche terms at points with normal derivatives dn"""
            S = (np.einsum("iq,jq,q->ij", -dn, val, w) + np.einsum("iq,jq,q->ij", val, -dn, w) +
                 nitsche / h * np.einsum("iq,jq,q->ij", val, val, w))
            add(Kt, d, d, S)
            add(At, d, d, S)
            s0 = len(spts)
            spts.extend(pts)
            si = np.arange(s0, s0 + len(pts))
            for a in range(len(d)):
                fgt.append((np.full(len(si), d[a]), si, (nitsche / h * val[a] - dn[a]) * w))

        for cy in range(self.n):
            for cx in range(self.n):
                if self.loc[cy, cx] == -location:
                    continue
                d = self.dofs(cx, cy)
                ins, sur = self.cell_quadrature(cx, cy, location)
                if ins:
                    s = np.array([x[0] for x in ins])
                    t = np.array([x[1] for x in ins])
                    w = np.array([x[2] for x in ins])
                    val, grad = self.shapes(cx, cy, s, t)
                    add(Mt, d, d, np.einsum("iq,jq,q->ij", val, val, w))
                    G = np.einsum("diq,djq,q->ij", grad, grad, w)
                    add(Kt, d, d, G)
                    add(At, d, d, G)
                    q0 = len(qpts)
                    x, y = self.real_point(cx, cy, s, t)
                    qpts += list(zip(x, y, w))
                    qi = np.arange(q0, q0 + len(ins))
                    for a in range(len(d)):
                        fft.append((np.full(len(qi), d[a]), qi, val[a] * w))
                        et.append((qi, np.full(len(qi), d[a]), val[a]))
                if sur and interface_data:
                    s = np.array([x[0] for x in sur])
                    t = np.array([x[1] for x in sur])
                    w = np.array([x[2] for x in sur])
                    nrm = sg * np.array([x[3] for x in sur]).T
                    val, grad = self.shapes(cx, cy, s, t)
                    x, y = self.real_point(cx, cy, s, t)
                    nitsche_points(d, val, np.einsum("diq,dq->iq", grad, nrm), w, list(zip(x, y, nrm[0], nrm[1])))
                if domain_data:
                    for axis, side in self.boundary_faces(cx, cy, location):
                        q = self.qx
                        s, t = (np.full(q.size, float(side)), q) if axis == 0 else (q, np.full(q.size, float(side)))
                        val, grad = self.shapes(cx, cy, s, t)
                        nv = 2.0 * side - 1.0
                        x, y = self.real_point(cx, cy, s, t)
                        nx_, ny_ = (nv, 0.0) if axis == 0 else (0.0, nv)
                        nitsche_points(d, val, nv * grad[axis], self.qw * h,
                                       [(a_, b_, nx_, ny_) for a_, b_ in zip(x, y)])
                if sur and coupled:
                    s = np.array([x[0] for x in sur])
                    t = np.array([x[1] for x in sur])
                    w = np.array([x[2] for x in sur])
                    nrm = np.array([x[3] for x in sur]).T  # the level-set normal (outward of the inside)
                    val, grad = self.shapes(cx, cy, s, t)
                    dn = np.einsum("diq,dq->iq", grad, nrm)
                    # r_own -= (-0.5 dn_v [u] -+ v n.{grad u} +- tau v [u]), [u] = u_in - u_out
                    VdN = np.einsum("iq,jq,q->ij", dn, val, w)
                    VnD = np.einsum("iq,jq,q->ij", val, dn, w)
                    VV = np.einsum("iq,jq,q->ij", val, val, w)
                    a_in = -0.5 * VdN - sg * 0.5 * VnD + sg * tau * VV
                    a_out = 0.5 * VdN - sg * 0.5 * VnD - sg * tau * VV
                    add(At, d, d, a_in if location == INSIDE else a_out)
                    add(Xt, d, d, -(a_out if location == INSIDE else a_in))
        for c, nb, axis, side in self.gp_faces(location):
            idx, j, w = self._face_jump(c, nb, axis, side)
            J = np.einsum("iq,jq,q->ij", j, j, w)
            if gamma_M >= 0:
                add(Mt, idx, idx, 0.5 * gamma_M * h ** 3 * J)
            add(Kt, idx, idx, 0.5 * gamma_A * h ** 3 * J)
            add(At, idx, idx, 0.5 * gamma_A * h * J)

        def build(T, shape, unit_diag):
            r = np.concatenate([x[0] for x in T]) if T else np.zeros(0, int)
            c = np.concatenate([x[1] for x in T]) if T else np.zeros(0, int)
            v = np.concatenate([x[2] for x in T]) if T else np.zeros(0)
            m = sp.csr_matrix((v, (r, c)), shape=shape)
            if unit_diag:
                dg = m.diagonal()
                m = m + sp.diags(np.where(dg == 0.0, 1.0, 0.0))
            return m.tocsr()

        nq, ns = len(qpts), len(spts)
        return dict(M=build(Mt, (N2, N2), True) if gamma_M >= 0 else None, K=build(Kt, (N2, N2), True),
                    A=build(At, (N2, N2), False), X=build(Xt, (N2, N2), False), Ff=build(fft, (N2, nq), False),
                    Fg=build(fgt, (N2, ns), False), E=build(et, (nq, N2), False), q=np.array(qpts).reshape(-1, 3),
                    s=np.array(spts).reshape(-1, 4))

    def interpolate(self, fun, t):
        """GDM::VectorTools::interpolate: vertex values (x fastest)"""
        X, Y = np.meshgrid(self.xv, self.xv, indexing="xy")
        return fun(X.reshape(-1), Y.reshape(-1), t)

    def errors(self, ops, u, exact, t):
        q = ops["q"]
        e = ops["E"] @ u - exact(q[:, 0], q[:, 1], t)
        return math.sqrt(float(np.sum(e * e * q[:, 2]))), float(np.sum(np.abs(e) * q[:, 2])), float(np.max(np.abs(e)))


# -- applications/wave/wave-app.cc parameter sets (dim = 2) -----------------
def wave_params():
    k = 3.0 * math.pi
    ex = lambda x, y, t: scipy.special.j0(k * np.hypot(x, y)) * math.cos(k * t)
    return dict(p=3, n=40, left=-1.21, right=1.21, gamma_M=0.25 * math.sqrt(3.0), gamma_A=0.5 * math.sqrt(3.0),
                nitsche=15.0, g=ex, f=None, exact=ex, start_t=0.0, end_t=2.0, cfl=0.3, cfl_pow=1.0)


def step85_params():
    ex = lambda x, y, t: 1.0 - (x * x + y * y - 1.0)
    return dict(p=3, n=40, left=-1.21, right=1.21, gamma_M=-1.0, gamma_A=0.5, nitsche=15.0,
                g=lambda x, y, t: np.ones_like(x), f=lambda x, y, t: np.full_like(x, 4.0), exact=ex)


def run(simulation, max_steps=None, model=None):
    """postprocess rows [(counter, t, L2, L1, Linf)] of WaveProblem<2>::run
    for simulation in {"wave", "step85"}; (rows, model, operators)"""
    P = wave_params() if simulation == "wave" else step85_params()
    m = model or CutWave2D(P["p"], P["n"], P["left"], P["right"])
    ops = m.matrices(P["gamma_M"], P["gamma_A"], P["nitsche"])
    q, s = ops["q"], ops["s"]

    def data(t):
        r = np.zeros(m.N * m.N)
        if P["f"] is not None and q.size:
            r += ops["Ff"] @ P["f"](q[:, 0], q[:, 1], t)
        if P["g"] is not None and s.size:
            r += ops["Fg"] @ P["g"](s[:, 0], s[:, 1], t)
        return r

    if simulation == "step85":
        u = spla.spsolve(ops["K"].tocsc(), data(0.0))
        return [(0, 0.0) + m.errors(ops, u, P["exact"], 0.0)], m, ops
    lu = spla.splu(ops["M"].tocsc())
    N = m.N * m.N
    dt = P["cfl"] * m.h ** P["cfl_pow"]
    time = DiscreteTime(P["start_t"], P["end_t"], dt)
    u = m.interpolate(P["exact"], P["start_t"])
    rows = [(0, 0.0) + m.errors(ops, u, P["exact"], 0.0)]
    y = np.concatenate([u, np.zeros_like(u)])

    def f(t, y):
        return np.concatenate([y[N:], lu.solve(-(ops["A"] @ y[:N]) + data(t))])

    n = 0
    while not time.is_at_end() and (max_steps is None or n < max_steps):
        t0, h = time.t, time.next_step_size()
        y = rk4_step(f, t0, h, y)
        n += 1
        rows.append((n, t0 + h) + m.errors(ops, y[:N], P["exact"], t0 + h))
        time.advance()
    return rows, m, ops


# -- composite presets (wave-app.cc:152-221 heat-composite, :286-347 wave-composite, dim = 2) --
def composite_params(kind):
    """an inside and an outside field coupled across the circle, domain
    Dirichlet data on the box faces (all in the outside region), no
    interface data; heat-composite on the heat-rk settings, wave-composite on
    the wave settings"""
    if kind == "heat-composite":
        ex = lambda x, y, t: x ** 9 * y ** 8 * math.exp(-t)  # noqa: E731
        f = lambda x, y, t: -x ** 7 * y ** 6 * math.exp(-t) * (x * x * y * y + 72 * y * y + 56 * x * x)  # noqa: E731
        return dict(p=3, n=40, left=-1.21, right=1.21, gamma_M=0.75, gamma_A=1.5, nitsche=15.0, g_domain=ex, f=f,
                    exact=ex, start_t=0.0, end_t=0.1, cfl=0.3 / 9.0, cfl_pow=2.0)
    P = wave_params()
    return dict(P, g_domain=P["g"], g=None)


def run_composite(simulation, max_steps=None, n=None, model=None, cfl_scale=1.0):
    """WaveProblem<2>::run for "heat-composite" / "wave-composite"
    (problem.h:128-214 heat-rk, :346-433 wave-rk on a BlockVector): rows
    [(counter, t, L2, L1, Linf)] alternating inside / outside; (rows, model,
    [operators inside, operators outside]).  At the presets' CFL the outside
    field is outside RK4's stability region (the box corners' Nitsche mode,
    tests/test_cut_wave2d_host.py): cfl_scale < 1 gives the stable runs."""
    P = composite_params(simulation)
    P["cfl"] *= cfl_scale
    m = model or CutWave2D(P["p"], P["n"] if n is None else n, P["left"], P["right"])
    ops = [m.matrices(P["gamma_M"], P["gamma_A"], P["nitsche"], location=loc, interface_data=False,
                      domain_data=True, coupled=True) for loc in (INSIDE, OUTSIDE)]
    lu = [spla.splu(o["M"].tocsc()) for o in ops]
    N = m.N * m.N

    def data(o, t):
        r = np.zeros(N)
        q, s = o["q"], o["s"]
        if P["f"] is not None and q.size:
            r += o["Ff"] @ P["f"](q[:, 0], q[:, 1], t)
        if s.size:
            r += o["Fg"] @ P["g_domain"](s[:, 0], s[:, 1], t)
        return r

    def fields(t, u0, u1):
        r0 = -(ops[0]["A"] @ u0) + ops[0]["X"] @ u1 + data(ops[0], t)
        r1 = -(ops[1]["A"] @ u1) + ops[1]["X"] @ u0 + data(ops[1], t)
        return lu[0].solve(r0), lu[1].solve(r1)

    dt = P["cfl"] * m.h ** P["cfl_pow"]
    time = DiscreteTime(P["start_t"], P["end_t"], dt)
    u = m.interpolate(P["exact"], P["start_t"])
    rows = []

    def post(t, u0, u1, counter):
        rows.append((counter, t) + m.errors(ops[0], u0, P["exact"], t))
        rows.append((counter, t) + m.errors(ops[1], u1, P["exact"], t))

    post(0.0, u, u, 0)
    if simulation == "wave-composite":
        y = np.concatenate([u, u, np.zeros(N), np.zeros(N)])

        def f(t, y):
            a0, a1 = fields(t, y[:N], y[N:2 * N])
            return np.concatenate([y[2 * N:3 * N], y[3 * N:], a0, a1])
    else:
        y = np.concatenate([u, u])

        def f(t, y):
            return np.concatenate(fields(t, y[:N], y[N:]))
    k = 0
    while not time.is_at_end() and (max_steps is None or k < max_steps):
        t0, h = time.t, time.next_step_size()
        y = rk4_step(f, t0, h, y)
        k += 1
        post(t0 + h, y[:N], y[N:2 * N], k)
        time.advance()
    return rows, m, ops
