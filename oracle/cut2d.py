"""2D cut-cell GDM restatement of prototypes/cut_poisson_01_gdm.cc (test
infrastructure: only tests/ and tools/ may import it).

What it restates (paths relative to the reference root):

  * mesh, categories, DoF boxes       include/gdm/system.h:195-246, 404-424
  * level set: FE_Q(1) interpolant of SignedDistance::Sphere (|x| - 1) on the
    vertices, NonMatching::MeshClassifier (vertex signs: inside / outside /
    intersected)                      cut_poisson_01_gdm.cc:100-120
  * NonMatching::FEValues quadrature: QGauss(p+1)^2 on inside cells; on
    intersected cells the deal.II QuadratureGenerator (Saye's algorithm) for
    the bilinear level set of the cell: Taylor bounds of the function and its
    gradient over the box, the height direction with the largest lower bound
    of |df/dx_i| (first of equal ones), the level set restricted to the bottom
    and top faces of that direction, the cross-section split at the roots of
    both restrictions with QGauss(p+1) per sub-interval, every such point
    lifted along the height direction: the line split at its root,
    QGauss(p+1) on each inside (f < 0) segment, one surface point at the root
    with weight w |grad f| / |df/dx_h| and normal grad f / |grad f|
    (deal.II source/non_matching/quadrature_generator.cc; deal.II is not
    vendored in the reference: restated from its published algorithm,
    R. Saye, SIAM J. Sci. Comput. 37 (2015) A993)
  * assembly: (grad v, grad u)_inside + Nitsche on the surface
    (gamma = 5 (p+1) p, h = minimum_vertex_distance) + ghost penalty
    0.5 * 0.5 * h [d_n v][d_n u] on every interior face with an intersected
    cell and a non-outside neighbour, visited from both cells; rhs 4 v +
    Nitsche data g = 1; zero diagonals -> 1    cut_poisson_01_gdm.cc:148-323
  * SolverCG, PreconditionIdentity, ReductionControl(n, 1e-10, 1e-6)
                                       cut_poisson_01_gdm.cc:326-335
  * L2 error against 1 - 2/dim (|x|^2 - 1) over the inside quadrature
                                       cut_poisson_01_gdm.cc:349-405

Pinned to prototypes/cut_poisson_01_gdm.output (the L2 errors of both runs,
without and with ghost penalty, to the 5 printed digits) by
tests/test_cut2d_golden.py.  Roots of the linear restrictions are computed in
closed form where deal.II's RootFinder iterates to its tolerance (1e-12 in
reference coordinates), far below the printed digits.
"""
import math

import numpy as np

import oracle as O

INSIDE, OUTSIDE, INTERSECTED = -1, 1, 0


def _gauss(n):
    x, w = O.gauss(n)
    return np.asarray(x), np.asarray(w)


class Bilinear:
    """f(s, t) = a + b s + c t + d s t on the unit square (FE_Q(1) level set
    in the reference coordinates of one cell; s = x direction)."""

    def __init__(self, v00, v10, v01, v11):
        self.a = v00
        self.b = v10 - v00
        self.c = v01 - v00
        self.d = v11 - v10 - v01 + v00

    def __call__(self, s, t):
        return self.a + self.b * s + self.c * t + self.d * s * t

    def grad(self, s, t):
        return np.array([self.b + self.d * t, self.c + self.d * s])


def _taylor_bounds(f, lo, hi):
    """deal.II taylor_estimate_function_bounds on the box [lo, hi]: value and
    gradient bounds from the first/second-order expansion at the centre."""
    cx, cy = 0.5 * (lo[0] + hi[0]), 0.5 * (lo[1] + hi[1])
    dx, dy = 0.5 * (hi[0] - lo[0]), 0.5 * (hi[1] - lo[1])
    val = f(cx, cy)
    g = f.grad(cx, cy)
    # Hessian [[0, d], [d, 0]]
    hd = abs(f.d)
    v_spread = abs(g[0]) * dx + abs(g[1]) * dy + 0.5 * (2 * hd * dx * dy)
    gb = [(g[0] - hd * dy, g[0] + hd * dy), (g[1] - hd * dx, g[1] + hd * dx)]
    return (val - v_spread, val + v_spread), gb


def _linear_root(f0, f1):
    """root in (0, 1) of the linear function with values f0 at 0 and f1 at 1 (or None)"""
    if f0 == 0.0 and f1 == 0.0:
        return None
    if (f0 < 0.0 < f1) or (f1 < 0.0 < f0):
        return f0 / (f0 - f1)
    return None


def saye_quadrature(f, nq, lo=(0.0, 0.0), hi=(1.0, 1.0)):
    """Inside (f < 0) and surface quadrature of the box [lo, hi] in reference
    coordinates: ([(s, t, w)], [(s, t, w, n)])."""
    qx, qw = _gauss(nq)
    (vmin, vmax), gb = _taylor_bounds(f, lo, hi)
    ext = (hi[0] - lo[0]) * (hi[1] - lo[1])
    if vmin > 1e-11:  # definitely outside
        return [], []
    if vmax < -1e-11:  # definitely inside
        return [(lo[0] + (hi[0] - lo[0]) * a, lo[1] + (hi[1] - lo[1]) * b, wa * wb * ext)
                for b, wb in zip(qx, qw) for a, wa in zip(qx, qw)], []
    low = []
    for (g0, g1) in gb:
        low.append(min(abs(g0), abs(g1)) if (g0 > 0 or g1 < 0) else 0.0)
    hdir = int(np.argmax(low))  # first of equal ones
    if not low[hdir] > 1e-11:
        raise NotImplementedError("box split / midpoint fallback of the quadrature generator")
    cdir = 1 - hdir
    c_lo, c_hi = lo[cdir], hi[cdir]
    h_lo, h_hi = lo[hdir], hi[hdir]

    def point(c, h):
        return (c, h) if cdir == 0 else (h, c)

    def fval(c, h):
        s, t = point(c, h)
        return f(s, t)

    # cross-section: roots of the restrictions to the bottom and top faces
    roots = []
    for hh in (h_lo, h_hi):
        r = _linear_root(fval(c_lo, hh), fval(c_hi, hh))
        if r is not None:
            roots.append(c_lo + r * (c_hi - c_lo))
    roots = sorted(roots)
    edges = [c_lo] + roots + [c_hi]
    low_q = []
    for a, b in zip(edges[:-1], edges[1:]):
        L = b - a
        if L > 0:
            low_q += [(a + L * x, w * L) for x, w in zip(qx, qw)]
    inside, surface = [], []
    for c, w in low_q:
        r = _linear_root(fval(c, h_lo), fval(c, h_hi))
        hs = [h_lo] + ([h_lo + r * (h_hi - h_lo)] if r is not None else []) + [h_hi]
        for a, b in zip(hs[:-1], hs[1:]):
            L = b - a
            if L <= 0:
                continue
            if fval(c, 0.5 * (a + b)) < 0.0:
                for x, wx in zip(qx, qw):
                    s, t = point(c, a + L * x)
                    inside.append((s, t, w * wx * L))
        if r is not None:
            hroot = h_lo + r * (h_hi - h_lo)
            s, t = point(c, hroot)
            g = f.grad(s, t)
            ng = math.hypot(g[0], g[1])
            surface.append((s, t, w * ng / abs(g[hdir]), g / ng))
    return inside, surface


class CutPoisson2D:
    """The reference's cut Poisson problem on [-1.21, 1.21]^2 (GDM degree p)."""

    def __init__(self, p=3, n_sub=64, left=-1.21, right=1.21, ghost_penalty=False):
        self.p, self.n = p, n_sub
        self.h = (right - left) / n_sub
        self.N = n_sub + 1
        self.left = left
        self.xv = np.array([left + i * self.h for i in range(self.N)])
        self.gp = ghost_penalty
        self.nq = p + 1
        self.qx, self.qw = _gauss(self.nq)
        xx, yy = np.meshgrid(self.xv, self.xv, indexing="xy")  # [iy, ix]
        self.ls = np.sqrt(xx * xx + yy * yy) - 1.0  # SignedDistance::Sphere at the vertices
        self.coef = {cat: [np.asarray(O.basis_coefficients(p, cat, i)) for i in range(p + 1)] for cat in range(p)}
        self.loc = np.zeros((n_sub, n_sub), dtype=int)
        for cy in range(n_sub):
            for cx in range(n_sub):
                v = self.ls[cy:cy + 2, cx:cx + 2]
                self.loc[cy, cx] = INSIDE if np.all(v < 0) else (OUTSIDE if np.all(v > 0) else INTERSECTED)

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
        return ((oy + k)[:, None] * self.N + (ox + k)[None, :]).reshape(-1)  # local i = ix + (p+1) iy

    def _basis_1d(self, cat, s, order):
        """[p+1, len(s)] values (order 0) or derivatives (order 1) in reference coordinates"""
        s = np.atleast_1d(np.asarray(s, dtype=float))
        out = np.zeros((self.p + 1, s.size))
        for i, c in enumerate(self.coef[cat]):
            cc = np.polynomial.polynomial.polyder(c, order) if order else c
            out[i] = np.polynomial.polynomial.polyval(s, cc)
        return out

    def shapes(self, cx, cy, s, t):
        """values [n_dofs, nq], gradients [2, n_dofs, nq] (real coordinates) at reference points (s, t)"""
        cxat, cyat = self.category(cx), self.category(cy)
        vx, dx = self._basis_1d(cxat, s, 0), self._basis_1d(cxat, s, 1) / self.h
        vy, dy = self._basis_1d(cyat, t, 0), self._basis_1d(cyat, t, 1) / self.h
        val = (vy[:, None, :] * vx[None, :, :]).reshape(-1, vx.shape[1])
        gx = (vy[:, None, :] * dx[None, :, :]).reshape(-1, vx.shape[1])
        gy = (dy[:, None, :] * vx[None, :, :]).reshape(-1, vx.shape[1])
        return val, np.stack([gx, gy])

    def cell_quadrature(self, cx, cy):
        """inside [(s, t, JxW)], surface [(s, t, JxW, normal)] of cell (cx, cy)"""
        loc = self.loc[cy, cx]
        h = self.h
        if loc == OUTSIDE:
            return [], []
        if loc == INSIDE:
            return [(a, b, wa * wb * h * h) for b, wb in zip(self.qx, self.qw) for a, wa in zip(self.qx, self.qw)], []
        v = self.ls[cy:cy + 2, cx:cx + 2]
        f = Bilinear(v[0, 0], v[0, 1], v[1, 0], v[1, 1])
        ins, sur = saye_quadrature(f, self.nq)
        return [(s, t, w * h * h) for s, t, w in ins], [(s, t, w * h, n) for s, t, w, n in sur]

    def real_point(self, cx, cy, s, t):
        return self.xv[cx] + s * self.h, self.xv[cy] + t * self.h

    # -- assembly (cut_poisson_01_gdm.cc:148-323) --------------------------
    def assemble(self):
        """(CSR row_ptr, cols, vals, rhs) of the reference's system"""
        p, n, h = self.p, self.n, self.h
        nd = (p + 1) ** 2
        gamma = 5.0 * (p + 1) * p
        entries = {}
        rhs = np.zeros(self.N * self.N)

        def add(rows, cols, M):
            for a, r in enumerate(rows):
                for b, c in enumerate(cols):
                    key = (int(r), int(c))
                    entries[key] = entries.get(key, 0.0) + M[a, b]

        # flux / cell sparsity: every coupling of a cell's (and with GP, a face
        # neighbour's) DoFs is a structural entry, zero or not
        struct = set()
        for cy in range(n):
            for cx in range(n):
                d = self.dofs(cx, cy)
                for r in d:
                    for c in d:
                        struct.add((int(r), int(c)))
                if self.gp:
                    for nx, ny in ((cx + 1, cy), (cx, cy + 1)):
                        if nx < n and ny < n:
                            e = self.dofs(nx, ny)
                            for r in d:
                                for c in e:
                                    struct.add((int(r), int(c)))
                                    struct.add((int(c), int(r)))
        for cy in range(n):
            for cx in range(n):
                if self.loc[cy, cx] == OUTSIDE:
                    continue
                d = self.dofs(cx, cy)
                K = np.zeros((nd, nd))
                F = np.zeros(nd)
                ins, sur = self.cell_quadrature(cx, cy)
                if ins:
                    s = np.array([q[0] for q in ins])
                    t = np.array([q[1] for q in ins])
                    w = np.array([q[2] for q in ins])
                    val, grad = self.shapes(cx, cy, s, t)
                    K += np.einsum("diq,djq,q->ij", grad, grad, w)
                    F += 4.0 * val @ w
                if sur:
                    s = np.array([q[0] for q in sur])
                    t = np.array([q[1] for q in sur])
                    w = np.array([q[2] for q in sur])
                    nrm = np.array([q[3] for q in sur]).T  # [2, nq]
                    val, grad = self.shapes(cx, cy, s, t)
                    dn = np.einsum("diq,dq->iq", grad, nrm)
                    K += np.einsum("iq,jq,q->ij", -dn, val, w) + np.einsum("jq,iq,q->ij", -dn, val, w) + \
                        gamma / h * np.einsum("iq,jq,q->ij", val, val, w)
                    F += (gamma / h * val - dn) @ w  # g = 1
                if self.gp:
                    for f, (nx, ny) in enumerate(((cx - 1, cy), (cx + 1, cy), (cx, cy - 1), (cx, cy + 1))):
                        if not (0 <= nx < n and 0 <= ny < n):
                            continue
                        a, b = self.loc[cy, cx], self.loc[ny, nx]
                        if not ((a == INTERSECTED and b != OUTSIDE) or (b == INTERSECTED and a != OUTSIDE)):
                            continue
                        # face quadrature QGauss(p+1), normal along the face axis
                        axis, side = (0, f % 2) if f < 2 else (1, f % 2)
                        if axis == 0:
                            sc, tc = np.full(self.nq, float(side)), self.qx
                            sn, tn = np.full(self.nq, 1.0 - side), self.qx
                        else:
                            sc, tc = self.qx, np.full(self.nq, float(side))
                            sn, tn = self.qx, np.full(self.nq, 1.0 - side)
                        _, gc = self.shapes(cx, cy, sc, tc)
                        _, gn = self.shapes(nx, ny, sn, tn)
                        jump = np.concatenate([gc[axis], -gn[axis]])  # normal . [grad phi] (sign irrelevant)
                        S = 0.5 * 0.5 * h * np.einsum("iq,jq,q->ij", jump, jump, self.qw * h)
                        idx = np.concatenate([d, self.dofs(nx, ny)])
                        add(idx, idx, S)
                add(d, d, K)
                rhs[d] += F
        for key in struct:
            entries.setdefault(key, 0.0)
        for i in range(self.N * self.N):
            if entries.get((i, i), 0.0) == 0.0:
                entries[(i, i)] = 1.0
        keys = sorted(entries)
        rows = np.array([k[0] for k in keys], dtype=np.int64)
        cols = np.array([k[1] for k in keys], dtype=np.int64)
        vals = np.array([entries[k] for k in keys])
        rp = np.zeros(self.N * self.N + 1, dtype=np.int64)
        np.add.at(rp, rows + 1, 1)
        rp = np.cumsum(rp)
        return rp, cols, vals, rhs

    def solve(self, rp, cols, vals, rhs):
        """SolverCG + PreconditionIdentity + ReductionControl(n, 1e-10, 1e-6) from zero"""
        n = len(rhs)
        return O.cg(rp, cols, vals, rhs, precond=0, max_it=n, abs_tol=1e-10, rel_tol=1e-6)

    def l2_error(self, u):
        err2 = 0.0
        for cy in range(self.n):
            for cx in range(self.n):
                if self.loc[cy, cx] == OUTSIDE:
                    continue
                ins, _ = self.cell_quadrature(cx, cy)
                if not ins:
                    continue
                s = np.array([q[0] for q in ins])
                t = np.array([q[1] for q in ins])
                w = np.array([q[2] for q in ins])
                val, _ = self.shapes(cx, cy, s, t)
                uh = u[self.dofs(cx, cy)] @ val
                x, y = self.real_point(cx, cy, s, t)
                exact = 1.0 - (x * x + y * y - 1.0)
                err2 += np.sum((uh - exact) ** 2 * w)
        return math.sqrt(err2)


def run(ghost_penalty, p=3, n_sub=64):
    """(mesh size, L2 error, CG iterations, system) of one test<2>(ghost_penalty) run"""
    P = CutPoisson2D(p, n_sub, ghost_penalty=ghost_penalty)
    rp, cols, vals, rhs = P.assemble()
    u, its = P.solve(rp, cols, vals, rhs)
    return P.h, P.l2_error(u), its, (rp, cols, vals, rhs, u)
