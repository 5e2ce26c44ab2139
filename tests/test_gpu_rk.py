"""Device-resident RK (gdm_amd/problem.py,
csrc/gdm_rk.hip) against the oracle's RK over the reference-faithful cell
loops.  The oracle side uses oracle/cut1d.py's rk4_step + DiscreteTime, the
restatement of deal.II's ExplicitRungeKutta (RK_CLASSIC_FOURTH_ORDER) and
DiscreteTime that reproduces the reference's wave_0 / heat_1 goldens
(tests/test_cut1d_golden.py) -- the RK semantics are pinned there.

Tolerances (fp64): RK state after the steps rel-L2 <= 1e-10 (mass solves
included); vector update and boundary-function evaluation <= 1e-14.
"""
import math

import numpy as np
import pytest

import cut1d
import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def test_rk_update():
    import gdm_amd

    op = gdm_amd.GdmOperator(1, 3, 40, 0.0, 1.0, "mass")
    rng = np.random.default_rng(0)
    n = 100003
    k, a, y = (rng.uniform(-1, 1, n) for _ in range(3))
    kd, ad, yd = dev(k), dev(a), dev(y)
    acc, Y = torch.zeros_like(kd), torch.zeros_like(kd)
    op.rk_update(0.37, kd, ad, acc, -1.25, yd, Y)
    np.testing.assert_allclose(host(acc), a + 0.37 * k, rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(host(Y), y - 1.25 * k, rtol=1e-14, atol=1e-15)
    op.rk_update(2.0, kd, acc, acc)  # in place, no stage vector
    np.testing.assert_allclose(host(acc), a + 0.37 * k + 2.0 * k, rtol=1e-14, atol=1e-14)


def _sine(pts, t, prm, dim, derivative):
    a, k, ph = prm[0:3], prm[3:6], prm[6:9]
    s = [np.sin(2 * np.pi * k[d] * (pts[:, d] - a[d] * t) + ph[d]) for d in range(dim)]
    c = [np.cos(2 * np.pi * k[d] * (pts[:, d] - a[d] * t) + ph[d]) for d in range(dim)]
    if not derivative:
        return np.prod(s, axis=0)
    r = np.zeros(len(pts))
    for d in range(dim):
        v = -2 * np.pi * k[d] * a[d] * c[d]
        for e in range(dim):
            if e != d:
                v = v * s[e]
        r += v
    return r


SINE = [1.0, 0.15, -0.05, 1.0, 2.0, 1.0, 0.3, 0.0, 0.7]


@pytest.mark.parametrize("dim,p,n", [(1, 3, 20), (2, 5, (30, 17)), (3, 5, (9, 11, 7)), (3, 7, 8)])
def test_eval_boundary_vs_host(dim, p, n):
    import gdm_amd

    a = (1.0, 0.15, -0.05)[:dim]
    op = gdm_amd.GdmOperator(dim, p, n, -0.5, 1.5, "advection", params=a)
    pts = op.bc_points()
    out = torch.zeros(op.n_bc_points, dtype=torch.float64, device="cuda")
    for deriv in (0, 1):
        op.eval_boundary(op.FN_SINE_PRODUCT, SINE, 0.37, deriv, out)
        np.testing.assert_allclose(host(out), _sine(pts, 0.37, SINE, dim, deriv), rtol=0, atol=1e-13)
    cone = [0.3, -0.3, -0.3, 0.1][: 1 + dim]
    op.eval_boundary(op.FN_CONE, cone, 0.0, 0, out)
    r = np.sqrt(((pts[:, :dim] - np.array(cone[1:])) ** 2).sum(axis=1))
    np.testing.assert_allclose(host(out), np.maximum(0.0, 0.3 - r), rtol=0, atol=1e-15)
    op.eval_boundary(op.FN_CONE, cone, 0.0, 1, out)
    assert not host(out).any()
    op.eval_boundary(op.FN_CONSTANT, [2.5], 1.0, 0, out)
    assert (host(out) == 2.5).all()


def _wave_oracle(m, u0, dt, steps, nitsche=0.0):
    N = m.n_dofs

    def f(t, y):
        r = m.wave_rhs(y[:N], impl=True, nitsche=nitsche)
        return np.concatenate([y[N:], m.kron_mass_inverse(r)])

    y = np.concatenate([u0, np.zeros(N)])
    time = cut1d.DiscreteTime(0.0, dt * (steps - 0.5), dt)  # the last step is shrunk
    n = 0
    while not time.is_at_end():
        y = cut1d.rk4_step(f, time.t, time.next_step_size(), y)
        time.advance()
        n += 1
    return y, n, time


@pytest.mark.parametrize("dim,p,n,nitsche", [(1, 3, 40, 0.0), (1, 7, 30, 0.0), (2, 5, (14, 11), 0.0),
                                             (3, 5, 7, 0.0), (3, 7, 8, 0.0), (2, 3, 12, 15.0)])
def test_wave_rk_vs_oracle(dim, p, n, nitsche):
    """wave-rk (wave/problem.h:280-346): du/dt = v, dv/dt = M^-1 K u, RK4 +
    DiscreteTime (last step shrunk) on the device vs the oracle."""
    import gdm_amd

    lo, hi = -1.21, 1.21
    params = (nitsche,) if nitsche > 0 else ()
    op = gdm_amd.GdmOperator(dim, p, n, lo, hi, "wave", params=params)
    m = O.Mesh(dim, p, n, lo, hi)
    X = m.vertex_coords()
    u0 = np.ones(m.n_dofs)
    for d in range(dim):
        u0 = u0 * np.cos(1.5 * np.pi * X[d] / 1.21 * 0.5 + 0.2 * d)
    h = min(m.h) * 0.05
    steps = 3
    y_ref, n_ref, time = _wave_oracle(m, u0, h, steps, nitsche)
    prob = gdm_amd.WaveProblem(op)
    prob.u.copy_(dev(u0))
    n_dev = prob.run(0.0, time.end, h)
    assert n_dev == n_ref == steps
    assert rel(host(prob.u), y_ref[:m.n_dofs]) < 1e-10
    assert rel(host(prob.v), y_ref[m.n_dofs:]) < 1e-10


def _advection_oracle(m, a, u0, prm, h, steps):
    pts = m.boundary_points()
    dim = m.dim
    u = u0.copy()
    time = cut1d.DiscreteTime(0.0, h * steps, h)
    while not time.is_at_end():
        t = time.t
        bc = _sine(pts, t, prm, dim, 0)  # initialize_time_step
        nb = len(bc)

        def f(tt, y):
            r = m.advection_rhs(a, y[nb:], y[:nb])
            return np.concatenate([_sine(pts, tt, prm, dim, 1), m.kron_mass_inverse(r)])

        y = cut1d.rk4_step(f, t, time.next_step_size(), np.concatenate([bc, u]))
        u = y[nb:]
        time.advance()
    return u


@pytest.mark.parametrize("dim,p,n", [(1, 3, 30), (2, 5, (13, 10)), (3, 5, 7)])
def test_advection_rk_device_boundary_vs_oracle(dim, p, n):
    """advection problem.h:31-102 with block(0) = g(t_n) / dg/dt evaluated on
    the device (no host evaluation, no H2D copy in the loop) vs the oracle
    RK over the cell loop with the same g."""
    import gdm_amd

    a = (1.0, 0.15, -0.05)[:dim]
    op = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "advection", params=a)
    m = O.Mesh(dim, p, n)
    X = np.stack(m.vertex_coords(), axis=1)
    u0 = _sine(np.pad(X, ((0, 0), (0, 3 - dim))), 0.0, SINE, dim, 0)
    h = min(m.h) * 0.1
    steps = 3
    ref = _advection_oracle(m, a, u0, SINE, h, steps)
    prob = gdm_amd.AdvectionProblem(op, op.FN_SINE_PRODUCT, SINE)
    prob.u.copy_(dev(u0))
    assert prob.run(0.0, h * steps, h) == steps
    assert rel(host(prob.u), ref) < 1e-10
