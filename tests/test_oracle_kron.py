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


def _numpy_cg_history(A, b, max_it, abs_tol, rel_tol):
    """deal.II SolverCG + ReductionControl (identity preconditioner) in numpy."""
    x = np.zeros_like(b)
    r = b.copy()
    res = [np.linalg.norm(r)]
    tol = max(abs_tol, rel_tol * res[0])
    p = r.copy()
    gh = r @ r
    for it in range(1, max_it + 1):
        if it > 1:
            gh_new = r @ r
            p = r + gh_new / gh * p
            gh = gh_new
        v = A @ p
        alpha = gh / (p @ v)
        x += alpha * p
        r -= alpha * v
        res.append(np.linalg.norm(r))
        if res[-1] <= tol:
            return it, np.array(res), tol
    return -1, np.array(res), tol


def test_cg_history_reference_order():
    """The CSR assembly follows the reference's summation order (q outer,
    mass.h:160-170 / matrix_creator.h:45-50): identity CG on Laplace + mass,
    2D p=5 n=12, rel 1e-6 -- the case whose residual sits at 0.90 x tol one
    iteration early -- stops where an independent numpy CG on the same matrix
    stops (89; the sum-factorised assembly of round 3 gave 91), and the
    history returned by cg_history is the one cg() stops on."""
    m = O.Mesh(2, 5, 12, 0.0, 1.0)
    b = np.random.default_rng(3).uniform(-1, 1, m.n_dofs)
    rp, cols, vals = m.matrix_csr(kind=1)
    vals = vals + m.matrix_csr(kind=0)[2]
    _, its = O.cg(rp, cols, vals, b, precond=0, max_it=5000, abs_tol=1e-10, rel_tol=1e-6)
    _, its_h, hist, tol = O.cg_history(rp, cols, vals, b, precond=0, max_it=5000, abs_tol=1e-10, rel_tol=1e-6)
    assert its == its_h == len(hist) - 1 == 89
    assert hist[-1] <= tol and np.all(hist[:-1] > tol)
    import scipy.sparse as sps

    A = sps.csr_matrix((vals, cols, rp), shape=(m.n_dofs, m.n_dofs))
    its_np, hist_np, tol_np = _numpy_cg_history(A, b, 5000, 1e-10, 1e-6)
    assert its_np == its
    np.testing.assert_allclose(hist_np[:8], hist[:8], rtol=1e-6)


def test_csr_assembly_symmetric_and_tuple_cached():
    """The per-category-tuple element matrices give a symmetric assembled mass
    / Laplace matrix whose mass entries sum to the domain volume."""
    m = O.Mesh(3, 3, (5, 6, 4), (0.0, 0.0, 0.0), (1.0, 0.5, 2.0))
    for kind in (0, 1):
        rp, cols, vals = m.matrix_csr(kind=kind)
        import scipy.sparse as sps

        A = sps.csr_matrix((vals, cols, rp), shape=(m.n_dofs, m.n_dofs))
        assert abs(A - A.T).max() <= 1e-14 * abs(A).max()
        if kind == 0:
            assert abs(vals.sum() - 1.0) < 1e-12
        else:
            assert abs(A @ np.ones(m.n_dofs)).max() < 1e-9
