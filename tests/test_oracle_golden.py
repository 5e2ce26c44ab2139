"""Pin the CPU restatement (oracle/) against the reference's own golden data.

Every expected number here comes from tests/golden/*.json, which
tests/golden/make_golden.py parsed from the reference's golden output files
(or produced by running the reference's scripts/create_coefficients.py).
CPU only.
"""
import json
import os

import numpy as np
import pytest

import oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")
REF = json.load(open(os.path.join(G, "reference_outputs.json")))
COEF = json.load(open(os.path.join(G, "coefficients.json")))["p"]


@pytest.mark.parametrize("p", [1, 3, 5, 7, 9])
def test_basis_coefficients_match_create_coefficients_script(p):
    """fe.h:55-336 tables == scripts/create_coefficients.py output == oracle."""
    ncat = 1 if p == 1 else p
    table = COEF[str(p)]
    assert len(table) == ncat
    for cat in range(ncat):
        for i in range(p + 1):
            expect = np.array([a / b for a, b in table[cat][i]])[::-1]  # ascending
            got = O.basis_coefficients(p, cat, i)
            np.testing.assert_allclose(got, expect, rtol=1e-11, atol=1e-13)


@pytest.mark.parametrize("p", [1, 3, 5, 7, 9])
def test_poly_01_values(p):
    """tests/poly_01.output: every 1D GDM polynomial at x = j/20 (printed %7.3f)."""
    ref = REF["poly_01"]["values"][str(p)]
    xs = REF["poly_01"]["x"]
    for cat, tab in enumerate(ref):
        for j, x in enumerate(xs):
            got = [O.basis_value(p, cat, i, x) for i in range(p + 1)]
            np.testing.assert_allclose(got, tab[j], atol=5.1e-4)


@pytest.mark.parametrize("p", [3, 5, 7, 9])
def test_fe_02_derivatives_at_zero(p):
    """tests/fe_02_gdm.output: |d^k phi_i/dx^k (0)|, k = 0..4, interior category p/2."""
    ref = np.array(REF["fe_02"]["abs_values_d0_to_d4"][str(p)])
    got = np.array([[abs(O.basis_value(p, p // 2, i, 0.0, k)) for k in range(5)] for i in range(p + 1)])
    np.testing.assert_allclose(got, ref, atol=5.1e-4, rtol=5e-4)


def _zero_boundary(rowptr, cols, vals, bnd):
    """AffineConstraints zero constraints: decouple constrained rows/columns."""
    bset = set(int(b) for b in bnd)
    vals = vals.copy()
    n = len(rowptr) - 1
    for r in range(n):
        for k in range(rowptr[r], rowptr[r + 1]):
            c = cols[k]
            if r in bset or c in bset:
                vals[k] = 1.0 if (r == c) else 0.0
    return vals


@pytest.mark.parametrize("p", [1, 3, 5, 7, 9])
def test_poisson_01(p):
    """tests/poisson_01_gdm.cc: 1D -u''=1, n=10, zero Dirichlet, CG identity
    ReductionControl(100, 1e-10, 1e-4): iteration count, nodal values, L2 error."""
    ref = REF["poisson_01"]["cases"][str(p)]
    m = O.Mesh(1, p, 10)
    rp, cols, vals = m.matrix_csr(kind=1)
    vals = _zero_boundary(rp, cols, vals, [0, 10])
    fq = np.ones(m.n_cells * (p + 1))
    rhs = m.wave_rhs(np.zeros(m.n_dofs), impl=False, fq=fq)
    rhs[[0, 10]] = 0.0
    x, its = O.cg(rp, cols, vals, rhs, precond=0, max_it=100, abs_tol=1e-10, rel_tol=1e-4)
    assert its == ref["iterations"]
    np.testing.assert_allclose(x, ref["values"], atol=1e-6)
    xq = m.cell_qpoints()[:, 0]
    exact = 0.125 - 0.5 * (xq - 0.5) ** 2
    err = m.l2_error(x, exact)
    assert abs(err - ref["l2_error"]) < 1e-8


def _projection_error(n_comp):
    p, n = 3, 40
    m = O.Mesh(2, p, n)
    rp, cols, vals = m.matrix_csr(kind=0)
    nq = (p + 1) ** 2
    xq = m.cell_qpoints()
    # expand to n_comp interleaved components: dof*n_comp + c (system.h:238-244)
    N = m.n_dofs
    rows = np.repeat(np.arange(N), np.diff(rp))
    R, C, V = [], [], []
    for c in range(n_comp):
        R.append(rows * n_comp + c)
        C.append(cols * n_comp + c)
        V.append(vals)
    R, C, V = np.concatenate(R), np.concatenate(C), np.concatenate(V)
    order = np.lexsort((C, R))
    R, C, V = R[order], C[order], V[order]
    rp2 = np.zeros(N * n_comp + 1, dtype=np.int64)
    np.add.at(rp2, R + 1, 1)
    rp2 = np.cumsum(rp2)
    rhs = np.zeros(N * n_comp)
    for c in range(n_comp):
        rhs_c = m.wave_rhs(np.zeros(N), impl=False, fq=xq[:, 0] + c)
        rhs[c::n_comp] = rhs_c
    x, its = O.cg(rp2, C.astype(np.int64), V, rhs, precond=1, max_it=100, abs_tol=1e-10, rel_tol=1e-8)
    err2 = 0.0
    for c in range(n_comp):
        err2 += m.l2_error(x[c::n_comp], xq[:, 0] + c) ** 2
    return np.sqrt(err2), its


def test_mass_01_projection():
    """tests/mass_01_gdm.cc: 2D L2 projection of x, p=3, n=40, CG-Jacobi 1e-8."""
    err, its = _projection_error(1)
    assert its > 0
    np.testing.assert_allclose(err, REF["mass_01"]["error"], rtol=1e-4)  # printed to 5 digits


def test_mass_02_projection_two_components():
    """tests/mass_02_gdm.cc: same with 2 interleaved components (x, x+1)."""
    err, its = _projection_error(2)
    np.testing.assert_allclose(err, REF["mass_02"]["error"], rtol=1e-5)  # printed to 6 digits


def test_poisson_02_partition_invariance_and_values():
    """tests/poisson_02_gdm.mpirun={1,3}.output: identical for 1 and 3 ranks;
    1D values are the exact nodal solution of -u''=1 on [0,1], n=20, p=3."""
    runs = REF["poisson_02"]["runs"]
    assert runs["1"] == runs["3"]
    m = O.Mesh(1, 3, 20)
    rp, cols, vals = m.matrix_csr(kind=1)
    vals = _zero_boundary(rp, cols, vals, [0, 20])
    rhs = m.wave_rhs(np.zeros(m.n_dofs), impl=False, fq=np.ones(m.n_cells * 4))
    rhs[[0, 20]] = 0
    x, _ = O.cg(rp, cols, vals, rhs, max_it=1000, abs_tol=1e-14, rel_tol=1e-14)
    np.testing.assert_allclose(x, runs["1"]["dim1"]["values"], atol=2e-6)
    # 2D: AMG-preconditioned CG stopped at rel 1e-4 -> compare with a loose bound
    m2 = O.Mesh(2, 3, 20)
    rp, cols, vals = m2.matrix_csr(kind=1)
    X, Y = m2.vertex_coords()
    bnd = np.where((X == 0) | (Y == 0) | (np.isclose(X, 1)) | (np.isclose(Y, 1)))[0]
    vals = _zero_boundary(rp, cols, vals, bnd)
    rhs = m2.wave_rhs(np.zeros(m2.n_dofs), impl=False, fq=np.ones(m2.n_cells * 16))
    rhs[bnd] = 0
    x2, _ = O.cg(rp, cols, vals, rhs, max_it=1000, abs_tol=1e-14, rel_tol=1e-14)
    ref2 = np.array(runs["1"]["dim2"]["values"])
    assert np.max(np.abs(x2 - ref2)) < 2e-3 * np.max(np.abs(ref2))


@pytest.mark.parametrize("n_procs", [1, 2, 3, 4, 8])
def test_partition_formula(n_procs):
    """system.h:720-757: slab ownership covers every vertex plane exactly once
    and every cell plane exactly once."""
    m = O.Mesh(3, 5, [11, 7, 29])
    planes, cells = [], []
    for r in range(n_procs):
        b, e, cb, ce = m.partition(n_procs, r)
        planes += list(range(b, e))
        cells += list(range(cb, ce))
    assert planes == list(range(30))
    assert cells == list(range(29))


@pytest.mark.parametrize("p", [3, 5, 7])
def test_categories_and_boxes(p):
    """system.h:195-246/404-424: box offsets and categories; nodes of category
    k sit at j - k relative to the cell's left vertex (Appendix A of SURVEY)."""
    n = 17
    for c in range(n):
        cat = O.lib().gdmo_category(c, p, n)
        off = O.lib().gdmo_offset(c, p, n)
        assert 0 <= cat < p
        assert off + p <= n
        assert off == c - cat  # node j of the box is at vertex off + j = c + (j - cat)
