"""1D cut-cell GDM restatement of the reference's wave application (test
infrastructure: only tests/ may import it).

Restates, for dim = 1, what applications/wave computes (paths relative to the
reference root):

  * mesh + categories + DoF boxes      include/gdm/system.h:195-246, 404-424
  * level set: FE_Q(p) interpolant of SignedDistance::Sphere (|x| - r),
    MeshClassifier (signs of the interpolant's Bernstein coefficients:
    inside / outside / intersected)
                                       applications/wave/include/gdm/wave/discretization.h:82-99
  * NonMatching::FEValues in 1D: QGauss(p+1) on the inside part of a cut
    cell, one surface point at the root with weight 1 and the level-set
    normal
  * mass matrix  (v, u)_inside + 0.5 g_M h^3 [dv/dn][du/dn] on ghost-penalty
    faces, zero diagonals -> 1      .../wave/mass.h:47-249
  * compute_rhs: -(v', u') + (v, f) + surface Nitsche (gamma_D = 5p) +
    -0.5 g_A h [v'][u'] (GP, h^1 in the rhs)   .../wave/stiffness.h:42-407
  * stiffness matrix: (v', u') + surface Nitsche + 0.5 g_A h^3 [v'][u']
    (GP, h^3 in the matrix)          .../wave/stiffness.h:602-800
  * wave-rk, heat-rk (RK_CLASSIC_FOURTH_ORDER + DiscreteTime), heat-impl
    (u <- (M + dt S)^-1 (M u + dt f))  .../wave/problem.h:39-346
  * composite (heat-composite, wave-composite): an inside and an outside
    field, each with its region's mass / stiffness / ghost penalty, domain
    Dirichlet data by Nitsche on the boundary faces in its region (IV,
    .../wave/stiffness.h:262-330), coupled by the interface terms of
    compute_rhs(BlockVector) (:420-575)
  * postprocess: L2 / L1 / Linf error on the inside quadrature
                                       .../wave/problem.h:504-590
  * parameters of "wave", "heat-rk", "heat-impl"   applications/wave/wave-app.cc:62-285

The mass / system solves are exact (dense LU): the reference's CG with
AMG / ILU to ReductionControl(1000, 1e-20, 1e-14) converges in 1-2 steps on
these 41-DoF systems (the "[L] solved in N" lines), i.e. to the same values
within 1e-14.  Pinned to applications/wave/tests/{wave_0,heat_0,heat_1}.output
and {wave,heat}_composite_0.output (tests/test_cut1d_golden.py); the level-set root is found by bisection to
machine precision where deal.II's root finder stops at its tolerance, a
difference far below the 9 printed digits.
"""
import math

import numpy as np

import oracle as O


def gauss(n):
    """QGauss(n) on [0, 1]."""
    x, w = O.gauss(n)
    return np.asarray(x), np.asarray(w)


def gauss_lobatto(n):
    """QGaussLobatto(n) on [0, 1] (FE_Q support points)."""
    if n == 2:
        return np.array([0.0, 1.0])
    # interior points: roots of P'_{n-1}
    c = np.zeros(n)
    c[-1] = 1.0
    r = np.polynomial.legendre.legroots(np.polynomial.legendre.legder(c))
    return np.concatenate([[0.0], np.sort((r + 1.0) / 2.0), [1.0]])


class DiscreteTime:
    """deal.II DiscreteTime (base/discrete_time.cc): the next time is the
    current one plus the last step, the step recomputed as the difference of
    the two times (round-off accumulates as in the reference), snapped to the
    end time when within 5 % of a step of it."""

    def __init__(self, start, end, dt):
        self.t, self.end, self.step = float(start), float(end), 0
        self._next = self._next_time(self.t, float(dt))

    def _next_time(self, current, step):
        n = current + step
        if step > 0.0 and n > self.end - 0.05 * step:
            n = self.end
        return n

    def is_at_end(self):
        return self.t == self.end

    def next_step_size(self):
        return self._next - self.t

    def advance(self):
        step = self._next - self.t
        self.t = self._next
        self._next = self._next_time(self.t, step)
        self.step += 1

RK4 = dict(a=[[], [0.5], [0.0, 0.5], [0.0, 0.0, 1.0]], b=[1 / 6, 1 / 3, 1 / 3, 1 / 6], c=[0.0, 0.5, 0.5, 1.0])


def rk4_step(f, t, h, y):
    """TimeStepping::ExplicitRungeKutta::evolve_one_time_step with
    RK_CLASSIC_FOURTH_ORDER: k_i = f(t + c_i h, y + h sum_j a_ij k_j),
    y += h sum_i b_i k_i."""
    k = []
    for i in range(4):
        yi = y.copy()
        for j, aij in enumerate(RK4["a"][i]):
            if aij != 0.0:
                yi = yi + h * aij * k[j]
        k.append(f(t + RK4["c"][i] * h, yi))
    for i in range(4):
        y = y + h * RK4["b"][i] * k[i]
    return y


class Cut1D:
    INSIDE, OUTSIDE, INTERSECTED = -1, 1, 0

    def __init__(self, p, n_sub, left, right, level_set, ls_degree=None):
        self.p, self.n = p, n_sub
        self.left, self.right = left, right
        self.h = (right - left) / n_sub
        self.N = n_sub + 1
        self.xv = np.array([left + i * self.h for i in range(self.N)])
        self.level_set = level_set
        k = ls_degree if ls_degree is not None else p
        self.gl = gauss_lobatto(k + 1)
        self.qx, self.qw = gauss(p + 1)
        self._shape_cache = {}
        self.cells = [self._cell(c) for c in range(n_sub)]

    # -- GDM indexing (system.h:195-246, 404-424) --------------------------
    def category(self, c):
        p, n = self.p, self.n
        return c if c < p // 2 else (p // 2 if c < n - p // 2 else p + c - n)

    def offset(self, c):
        p, n = self.p, self.n
        return 0 if c < p // 2 else min(n, c + p // 2 + 1) - p

    def _cell(self, c):
        x0 = self.xv[c]
        # FE_Q(k) interpolant of the level set on the cell (Lagrange through GL points)
        vals = np.array([self.level_set(x0 + s * self.h) for s in self.gl])
        # MeshClassifier: signs of the Bernstein coefficients of the interpolant
        k = len(self.gl) - 1
        B = np.array([[math.comb(k, i) * s ** i * (1 - s) ** (k - i) for i in range(k + 1)] for s in self.gl])
        bern = np.linalg.solve(B, vals)
        if np.all(bern < 0):
            loc = self.INSIDE
        elif np.all(bern > 0):
            loc = self.OUTSIDE
        else:
            loc = self.INTERSECTED

        def phi(s):  # interpolant at reference coordinate s
            r = 0.0
            for a, sa in enumerate(self.gl):
                la = 1.0
                for b, sb in enumerate(self.gl):
                    if b != a:
                        la *= (s - sb) / (sa - sb)
                r += vals[a] * la
            return r

        cell = dict(c=c, x0=x0, cat=self.category(c), off=self.offset(c), loc=loc, surface=[])
        full = [(x0 + s * self.h, w * self.h) for s, w in zip(self.qx, self.qw)]
        if loc == self.INSIDE:
            cell["q"], cell["q_out"] = full, []
        elif loc == self.OUTSIDE:
            cell["q"], cell["q_out"] = [], full
        else:
            # roots of the interpolant in (0, 1): sign changes on a fine grid + bisection
            grid = np.linspace(0.0, 1.0, 65)
            pv = [phi(s) for s in grid]
            roots = []
            for a in range(64):
                if pv[a] == 0.0:
                    roots.append(grid[a])
                elif pv[a] * pv[a + 1] < 0:
                    lo, hi = grid[a], grid[a + 1]
                    flo = pv[a]
                    for _ in range(200):
                        mid = 0.5 * (lo + hi)
                        if mid == lo or mid == hi:
                            break
                        fm = phi(mid)
                        if (fm < 0) == (flo < 0):
                            lo, flo = mid, fm
                        else:
                            hi = mid
                    roots.append(0.5 * (lo + hi))
            pts = [0.0] + roots + [1.0]
            q, q_out = [], []
            for a, b in zip(pts[:-1], pts[1:]):
                seg = [(x0 + (a + (b - a) * s) * self.h, (b - a) * w * self.h) for s, w in zip(self.qx, self.qw)]
                if phi(0.5 * (a + b)) < 0:  # inside sub-interval
                    q += seg
                else:
                    q_out += seg
            cell["q"], cell["q_out"] = q, q_out
            for r in roots:
                # level-set normal (gradient direction) at the root, finite difference of the interpolant
                e = 1e-7
                g = phi(min(r + e, 1.0)) - phi(max(r - e, 0.0))
                cell["surface"].append((x0 + r * self.h, 1.0 if g > 0 else -1.0))
        return cell

    def shapes(self, cell, x, order):
        """values (order 0) or x-derivatives (order 1) of the p+1 local shapes at x"""
        key = (cell["c"], x, order)
        v = self._shape_cache.get(key)
        if v is None:
            s = (x - cell["x0"]) / self.h
            v = np.array([O.basis_value(self.p, cell["cat"], i, s, order) / self.h ** order
                          for i in range(self.p + 1)])
            self._shape_cache[key] = v
        return v

    def dofs(self, cell):
        return cell["off"] + np.arange(self.p + 1)

    # -- ghost-penalty faces (mass.h:86-105 / stiffness.h:80-98) ------------
    def gp_faces(self, location=-1):
        """(cell, neighbour, face point) for every (cell, face) pair the
        reference visits for the field of `location` (INSIDE / OUTSIDE); each
        interior face near a cut is visited from both sides (the 0.5 factors)."""
        inv = -location
        out = []
        for c, cell in enumerate(self.cells):
            if cell["loc"] == inv:
                continue
            for f, nb in ((0, c - 1), (1, c + 1)):
                if nb < 0 or nb >= self.n:
                    continue
                nl = self.cells[nb]["loc"]
                if (cell["loc"] == self.INTERSECTED and nl != inv) or \
                        (nl == self.INTERSECTED and cell["loc"] != inv):
                    out.append((c, nb, self.xv[c + f]))
        return out

    def region(self, cell, location):
        """the cell's quadrature of the INSIDE or OUTSIDE region"""
        return cell["q"] if location == self.INSIDE else cell["q_out"]

    def _jump_grad(self, c, nb, xf):
        """global DoF -> [dphi/dx] = (from cell c) - (from neighbour) at face xf"""
        key = ("jump", c, nb)
        if key in self._shape_cache:
            return self._shape_cache[key]
        j = {}
        for cc, sgn in ((c, 1.0), (nb, -1.0)):
            cell = self.cells[cc]
            g = self.shapes(cell, xf, 1)
            for i, d in enumerate(self.dofs(cell)):
                j[d] = j.get(d, 0.0) + sgn * g[i]
        self._shape_cache[key] = j
        return j

    # -- matrices -----------------------------------------------------------
    def mass_matrix(self, gamma_M, location=-1):
        M = np.zeros((self.N, self.N))
        for cell in self.cells:
            if cell["loc"] == -location:
                continue
            d = self.dofs(cell)
            for x, jxw in self.region(cell, location):
                v = self.shapes(cell, x, 0)
                M[np.ix_(d, d)] += np.outer(v, v) * jxw
        for c, nb, xf in self.gp_faces(location):
            j = self._jump_grad(c, nb, xf)
            keys = list(j)
            for a in keys:
                for b in keys:
                    M[a, b] += 0.5 * gamma_M * self.h ** 3 * j[a] * j[b]
        for i in range(self.N):
            if M[i, i] == 0.0:
                M[i, i] = 1.0
        return M

    def stiffness_matrix(self, gamma_A, nitsche, with_surface=True):
        S = np.zeros((self.N, self.N))
        for cell in self.cells:
            if cell["loc"] == self.OUTSIDE:
                continue
            d = self.dofs(cell)
            for x, jxw in cell["q"]:
                g = self.shapes(cell, x, 1)
                S[np.ix_(d, d)] += np.outer(g, g) * jxw
            if with_surface:
                for xs, n in cell["surface"]:
                    v, g = self.shapes(cell, xs, 0), self.shapes(cell, xs, 1)
                    S[np.ix_(d, d)] += (-n * np.outer(g, v) - n * np.outer(v, g) +
                                        nitsche / self.h * np.outer(v, v))
        for c, nb, xf in self.gp_faces():
            j = self._jump_grad(c, nb, xf)
            for a in j:
                for b in j:
                    S[a, b] += 0.5 * gamma_A * self.h ** 3 * j[a] * j[b]
        for i in range(self.N):
            if S[i, i] == 0.0:
                S[i, i] = 1.0
        return S

    def rhs(self, u, t, impl, gamma_A, nitsche, f=None, g=None, location=-1, g_domain=None):
        """StiffnessMatrixOperator::compute_rhs_internal (wave/stiffness.h:42-407)
        for the field of `location`: interface Dirichlet data g (II), domain
        Dirichlet data g_domain on the boundary faces of that region (IV)"""
        r = np.zeros(self.N)
        for cell in self.cells:
            if cell["loc"] == -location:
                continue
            d = self.dofs(cell)
            ul = u[d]
            cv = np.zeros(self.p + 1)
            for x, jxw in self.region(cell, location):
                v, gr = self.shapes(cell, x, 0), self.shapes(cell, x, 1)
                if impl:
                    cv -= gr * (gr @ ul) * jxw
                if f is not None:
                    cv += f(x, t) * v * jxw
            if g is not None:
                for xs, n in cell["surface"]:
                    n = n if location == self.INSIDE else -n
                    v, gr = self.shapes(cell, xs, 0), self.shapes(cell, xs, 1)
                    uq, duq = v @ ul, gr @ ul
                    if impl:
                        cv -= (-n * gr * uq - n * duq * v + nitsche / self.h * v * uq)
                    cv += g(xs, t) * (nitsche / self.h * v - n * gr)
            if g_domain is not None:
                for xf, n in self.domain_faces(cell, location):
                    v, gr = self.shapes(cell, xf, 0), self.shapes(cell, xf, 1)
                    uq, duq = v @ ul, gr @ ul
                    if impl:
                        cv -= (-n * gr * uq - n * duq * v + nitsche / self.h * v * uq)
                    cv += g_domain(xf, t) * (nitsche / self.h * v - n * gr)
            r[d] += cv
        if impl:
            for c, nb, xf in self.gp_faces(location):
                j = self._jump_grad(c, nb, xf)
                ju = sum(j[a] * u[a] for a in j)
                for a in j:
                    r[a] -= 0.5 * gamma_A * self.h * j[a] * ju
        return r

    def domain_faces(self, cell, location):
        """(point, outward normal) of the cell's faces on the domain boundary
        that lie in the region of `location` (NonMatching::FEInterfaceValues
        of the face: the level set's sign at the face point)"""
        out = []
        for xf, n, at in ((self.xv[0], -1.0, cell["c"] == 0), (self.xv[-1], 1.0, cell["c"] == self.n - 1)):
            if at and np.sign(self.level_set(xf)) == location:
                out.append((xf, n))
        return out

    def coupling(self, u0, u1, nitsche):
        """the composite interface terms of compute_rhs(BlockVector)
        (wave/stiffness.h:420-575): tau = nitsche / 2, [u] = u0 - u1,
        {u'} = (u0' + u1') / 2 on the surface points of intersected cells"""
        r0, r1 = np.zeros(self.N), np.zeros(self.N)
        tau = 0.5 * nitsche
        for cell in self.cells:
            if cell["loc"] != self.INTERSECTED:
                continue
            d = self.dofs(cell)
            for xs, n in cell["surface"]:
                v, gr = self.shapes(cell, xs, 0), self.shapes(cell, xs, 1)
                jump = v @ u0[d] - v @ u1[d]
                avg = 0.5 * (gr @ u0[d] + gr @ u1[d])
                r0[d] -= -0.5 * n * gr * jump - v * n * avg + tau / self.h * v * jump
                r1[d] -= -0.5 * n * gr * jump + v * n * avg - tau / self.h * v * jump
        return r0, r1

    def errors(self, u, exact, t, location=-1):
        """problem.h:504-590: (L2, L1, Linf) over the region's quadrature"""
        l2, l1, linf = 0.0, 0.0, 0.0
        for cell in self.cells:
            if cell["loc"] == -location:
                continue
            ul = u[self.dofs(cell)]
            for x, jxw in self.region(cell, location):
                e = self.shapes(cell, x, 0) @ ul - exact(x, t)
                l2 += e * e * jxw
                l1 += abs(e) * jxw
                linf = max(linf, abs(e))
        return math.sqrt(l2), l1, linf

    def interpolate(self, fun, t):
        """GDM::VectorTools::interpolate: vertex values (vector_tools.h:11-23)"""
        return np.array([fun(x, t) for x in self.xv])


# -- applications/wave/wave-app.cc parameter sets (dim = 1) -----------------
def _sphere(x):
    return abs(x) - 1.0


def wave_params():
    k = 1.5 * math.pi
    ex = lambda x, t: math.cos(k * abs(x)) * math.cos(k * t)
    return dict(p=3, n=40, left=-1.21, right=1.21, gamma_M=0.25 * math.sqrt(3.0), gamma_A=0.5 * math.sqrt(3.0),
                nitsche=15.0, g=ex, f=None, exact=ex, start_t=0.0, end_t=2.0, cfl=0.3, cfl_pow=1.0)


def heat_params(kind):
    ex = lambda x, t: x ** 9 * math.exp(-t)
    f = lambda x, t: -x ** 7 * math.exp(-t) * (x * x + 72)
    cfl, cfl_pow = (0.3 / 9.0, 2.0) if kind == "heat-rk" else (0.3, 1.0)
    return dict(p=3, n=40, left=-1.21, right=1.21, gamma_M=0.75, gamma_A=1.5, nitsche=15.0, g=ex, f=f, exact=ex,
                start_t=0.0, end_t=0.1, cfl=cfl, cfl_pow=cfl_pow)


def composite_params(kind):
    """wave-app.cc:150-214 heat-composite (heat-rk), :263-330 wave-composite
    (wave-rk): an inside and an outside field coupled across the interface,
    domain Dirichlet data on the boundary faces, no interface data"""
    if kind == "heat-composite":
        P = heat_params("heat-rk")
    else:
        P = wave_params()
    P = dict(P, g_domain=P["g"], g=None)
    return P


def run_composite(simulation, max_steps=None):
    """WaveProblem<1>::run for "heat-composite" / "wave-composite": rows
    [(counter, t, L2, L1, Linf)] alternating inside / outside
    (problem.h:128-214 heat-rk, :346-433 wave-rk)"""
    P = composite_params(simulation)
    m = Cut1D(P["p"], P["n"], P["left"], P["right"], _sphere)
    I, O_ = Cut1D.INSIDE, Cut1D.OUTSIDE
    Minv = [np.linalg.inv(m.mass_matrix(P["gamma_M"], loc)) for loc in (I, O_)]
    dt = P["cfl"] * m.h ** P["cfl_pow"]
    time = DiscreteTime(P["start_t"], P["end_t"], dt)
    N = m.N

    def fields_rhs(t, u0, u1):
        c0, c1 = m.coupling(u0, u1, P["nitsche"])
        r = [m.rhs(u, t, True, P["gamma_A"], P["nitsche"], f=P["f"], location=loc, g_domain=P["g_domain"]) + c
             for u, loc, c in ((u0, I, c0), (u1, O_, c1))]
        return Minv[0] @ r[0], Minv[1] @ r[1]

    rows = []

    def post(t, u0, u1, counter):
        rows.append((counter, t) + m.errors(u0, P["exact"], t, I))
        rows.append((counter, t) + m.errors(u1, P["exact"], t, O_))

    u = m.interpolate(P["exact"], P["start_t"])
    post(0.0, u, u, 0)
    if simulation == "wave-composite":
        y = np.concatenate([u, u, np.zeros(N), np.zeros(N)])

        def f(t, y):
            a0, a1 = fields_rhs(t, y[:N], y[N:2 * N])
            return np.concatenate([y[2 * N:3 * N], y[3 * N:], a0, a1])
    else:
        y = np.concatenate([u, u])

        def f(t, y):
            return np.concatenate(fields_rhs(t, y[:N], y[N:]))
    n = 0
    while not time.is_at_end() and (max_steps is None or n < max_steps):
        t0, h = time.t, time.next_step_size()
        y = rk4_step(f, t0, h, y)
        n += 1
        post(t0 + h, y[:N], y[N:2 * N], n)
        time.advance()
    return rows


def run(simulation, max_steps=None):
    """Returns the postprocess table [(counter, t, L2, L1, Linf)] of
    WaveProblem<1>::run for simulation in {"wave", "heat-rk", "heat-impl"}."""
    P = wave_params() if simulation == "wave" else heat_params(simulation)
    m = Cut1D(P["p"], P["n"], P["left"], P["right"], _sphere)
    M = m.mass_matrix(P["gamma_M"])
    Minv = np.linalg.inv(M)
    dt = P["cfl"] * m.h ** P["cfl_pow"]
    time = DiscreteTime(P["start_t"], P["end_t"], dt)
    rows = []

    def post(t, u, counter):
        rows.append((counter, t) + m.errors(u, P["exact"], t))

    u = m.interpolate(P["exact"], P["start_t"])
    post(0.0, u, 0)
    if simulation == "wave":
        y = np.concatenate([u, np.zeros_like(u)])
        N = m.N

        def f(t, y):
            r = m.rhs(y[:N], t, True, P["gamma_A"], P["nitsche"], f=P["f"], g=P["g"])
            return np.concatenate([y[N:], Minv @ r])
    elif simulation == "heat-rk":
        y = u

        def f(t, y):
            return Minv @ m.rhs(y, t, True, P["gamma_A"], P["nitsche"], f=P["f"], g=P["g"])
    else:
        S = m.stiffness_matrix(P["gamma_A"], P["nitsche"])
    n = 0
    while not time.is_at_end() and (max_steps is None or n < max_steps):
        t0, h = time.t, time.next_step_size()
        if simulation == "heat-impl":
            rhs = h * m.rhs(u, t0 + h, False, P["gamma_A"], P["nitsche"], f=P["f"], g=P["g"]) + M @ u
            u = np.linalg.solve(M + h * S, rhs)
        else:
            y = rk4_step(f, t0, h, y)
            u = y[:m.N]
        n += 1
        post(t0 + h, u, n)
        time.advance()
    return rows
