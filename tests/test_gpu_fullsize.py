"""Full-size checks of the BASELINE configs against the oracle's independent
Kronecker-form C code (oracle/gdm_oracle_kron.c, itself checked against the
reference-faithful cell loops in tests/test_oracle_kron.py):

  C2  2D advection p = 5, 1024^2 DoFs: compute_rhs (volume + outflow traces) and
      the exact mass inverse
  C4  3D wave p = 7, 256^3 DoFs: compute_rhs and the exact mass inverse
  C3  3D advection p = 5, 512^3 DoFs: compute_rhs and the exact mass inverse

Same seeded inputs on both sides; tolerance rel-L2 1e-12 (fp64 summation
order).  The inflow boundary data are covered at reduced size in
tests/test_gpu_parity.py (the oracle's cell loop is too slow at 512^3)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402

A2 = (2 * 0.9063077870366499, 2 * 0.42261826174069944)  # BASELINE C2 (tools/bench_ops.py)
A3 = (1.0, 0.15, -0.05)


def _gdm():
    import gdm_amd

    return gdm_amd


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _terms(m, kind, a=None):
    M = [m.matrices_1d(d)[0] for d in range(m.dim)]
    if kind == "wave":
        B = [-m.matrices_1d(d)[2] for d in range(m.dim)]
    else:
        B = [m.advection_outflow_B(d, a[d]) for d in range(m.dim)]
    if m.dim == 2:
        return [(B[0], M[1]), (M[0], B[1])]
    return [(B[0], M[1], M[2]), (M[0], B[1], M[2]), (M[0], M[1], B[2])]


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_apply_and_mass_inverse_full_size(cfg):
    g = _gdm()
    if cfg == "C2":
        dim, p, n, lo, hi, kind, prm = 2, 5, 1023, 0.0, 1.0, "advection", A2
    else:
        dim, p, n, lo, hi, kind, prm = 3, 7, 255, -1.21, 1.21, "wave", ()
    op = g.GdmOperator(dim, p, n, lo, hi, kind, params=prm)
    m = O.Mesh(dim, p, n, lo, hi)
    assert op.n_owned == m.n_dofs == (n + 1) ** dim
    u = np.random.default_rng(7).uniform(-1, 1, m.n_dofs)
    y = op.new_vector(local=False)
    op.apply(torch.from_numpy(u).cuda(), y)
    ref = m.kron_apply(_terms(m, kind, prm), u)
    assert _rel(y.cpu().numpy(), ref) < 1e-12
    x = op.new_vector(local=False)
    op.mass_solve(torch.from_numpy(ref).cuda(), x)
    assert _rel(x.cpu().numpy(), m.kron_mass_inverse(ref)) < 1e-12


def test_c3_apply_full_size():
    g = _gdm()
    op = g.GdmOperator(3, 5, 511, 0.0, 1.0, "advection", params=A3)
    m = O.Mesh(3, 5, 511, 0.0, 1.0)
    u = np.random.default_rng(8).uniform(-1, 1, m.n_dofs)
    y = op.new_vector(local=False)
    op.apply(torch.from_numpy(u).cuda(), y)
    got = y.cpu().numpy()
    del y
    assert _rel(got, m.kron_apply(_terms(m, "advection", A3), u)) < 1e-12


def test_c3_mass_inverse_full_size():
    """The headline config's per-stage solve (advection/problem.h:236-267):
    the device's exact Kronecker mass inverse at 512^3, p = 5, against the
    oracle's banded-Cholesky Kronecker inverse on the same right-hand side."""
    g = _gdm()
    op = g.GdmOperator(3, 5, 511, 0.0, 1.0, "advection", params=A3)
    m = O.Mesh(3, 5, 511, 0.0, 1.0)
    r = np.random.default_rng(9).uniform(-1, 1, m.n_dofs)
    x = op.new_vector(local=False)
    op.mass_solve(torch.from_numpy(r).cuda(), x)
    got = x.cpu().numpy()
    del x
    assert _rel(got, m.kron_mass_inverse(r)) < 1e-12
