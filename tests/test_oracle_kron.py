"""Oracle self-consistency: reference-faithful cell loops == Kronecker form.

The cell loops in oracle/gdm_oracle.c follow the reference's FEValues loops;
the Kronecker form in oracle/gdm_oracle_kron.c is the structure the GPU
kernels exploit.  Agreement to ~1e-13 here is what licenses using the
Kronecker form as the checker at sizes the cell loop cannot reach.  CPU only.
"""
import numpy as np
import pytest

import oracle as O


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("dim,p,n", [(1, 3, 17), (2, 3, 9), (2, 5, 12), (3, 3, 7), (3, 5, 8)])
def test_mass_cell_loop_equals_kron(dim, p, n):
    m = O.Mesh(dim, p, n, 0.0, 1.3)
    rng = np.random.default_rng(20251010)
    u = rng.uniform(-1, 1, m.n_dofs)
    rp, cols, vals = m.matrix_csr(kind=0)
    y_csr = O.csr_vmult(rp, cols, vals, u)
    Ms = [m.matrices_1d(d)[0] for d in range(dim)]
    y_k = m.kron_apply([tuple(Ms + [None] * (3 - dim))], u)
    assert _rel(y_k, y_csr) < 1e-13


@pytest.mark.parametrize("dim,p,n", [(1, 5, 20), (2, 3, 9), (2, 5, 12), (3, 5, 7)])
@pytest.mark.parametrize("a", [(1.0, 0.15, -0.05), (-0.7, 0.4, 0.3)])
def test_advection_cell_loop_equals_kron(dim, p, n, a):
    """stiffness.h:345-532 (alpha=0, uncut, u+ = 0) == sum_d B_d (x) M (x) M."""
    m = O.Mesh(dim, p, n, -0.5, 0.5)
    rng = np.random.default_rng(7)
    u = rng.uniform(-1, 1, m.n_dofs)
    nb = m.n_boundary_points()
    ref = m.advection_rhs(a[:dim], u, np.zeros(nb))
    M = [m.matrices_1d(d)[0] for d in range(dim)]
    B = [m.advection_outflow_B(d, a[d]) for d in range(dim)]
    terms = []
    for d in range(dim):
        ops = [B[e] if e == d else M[e] for e in range(dim)] + [None] * (3 - dim)
        terms.append(tuple(ops))
    y = m.kron_apply(terms, u)
    assert _rel(y, ref) < 1e-12


@pytest.mark.parametrize("dim,p,n", [(1, 7, 20), (2, 5, 10), (3, 3, 7), (3, 7, 8)])
def test_wave_cell_loop_equals_kron(dim, p, n):
    """wave/stiffness.h:171-181 (impl part, uncut, no Nitsche) == -sum_d L_d (x) M (x) M."""
    m = O.Mesh(dim, p, n, -1.21, 1.21)
    rng = np.random.default_rng(3)
    u = rng.uniform(-1, 1, m.n_dofs)
    ref = m.wave_rhs(u, impl=True)
    M = [m.matrices_1d(d)[0] for d in range(dim)]
    L = [-m.matrices_1d(d)[2] for d in range(dim)]
    terms = [tuple([L[e] if e == d else M[e] for e in range(dim)] + [None] * (3 - dim)) for d in range(dim)]
    y = m.kron_apply(terms, u)
    assert _rel(y, ref) < 1e-12


@pytest.mark.parametrize("dim,p,n", [(1, 5, 30), (2, 3, 12), (3, 5, 9)])
def test_mass_inverse_kron_equals_cg(dim, p, n):
    """Exact Kronecker mass inverse == CG (rel 1e-14) on the assembled matrix
    (the reference's solve, advection/problem.h:236-267)."""
    m = O.Mesh(dim, p, n)
    rng = np.random.default_rng(11)
    r = rng.uniform(-1, 1, m.n_dofs)
    rp, cols, vals = m.matrix_csr(kind=0)
    x_cg, its = O.cg(rp, cols, vals, r, precond=1, max_it=5000, abs_tol=1e-20, rel_tol=1e-14)
    assert its > 0
    x_k = m.kron_mass_inverse(r)
    assert _rel(x_k, x_cg) < 1e-12
