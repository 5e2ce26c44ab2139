"""Product-side cut-cell assembly (libgdm_hip.so, csrc/gdm_cut.cpp, ABI
"Cut-cell systems"; host code, no GPU) against the 2D cut-cell restatement
oracle/cut2d.py (pinned to prototypes/cut_poisson_01_gdm.output by
tests/test_cut2d_golden.py):

  * the assembled matrix equals the oracle's entry for entry (the oracle also
    stores the structural zeros of the flux / cell sparsity pattern) to 1e-13
    of the largest entry, the rhs to 1e-14; same cell classification counts;
  * the oracle's CG (deal.II SolverCG semantics) on the library's system and
    the library's L2 error reproduce the reference's printed error lines
    (ghost penalty: to 1.5e-4; without: to 1 %, the spread of the
    unconverged, unstabilised CG iterate under fp64 summation order);
  * the library's L2 error of the oracle's solution equals the oracle's;
  * argument checks (even p, bad radius) fail with GDM_ERR_ARG.
"""
import numpy as np
import pytest

import cut2d
import oracle as O


def _lib():
    import gdm_amd

    return gdm_amd


@pytest.mark.parametrize("ghost_penalty", [True, False])
def test_cut_assembly_matches_oracle(ghost_penalty):
    import scipy.sparse as sp

    g = _lib()
    S = g.CutPoisson(3, 64, ghost_penalty=ghost_penalty)
    P = cut2d.CutPoisson2D(3, 64, ghost_penalty=ghost_penalty)
    rp, cols, vals, rhs = P.assemble()
    n = len(rhs)
    assert S.n_rows == n
    assert S.n_intersected_cells == int(np.sum(P.loc == cut2d.INTERSECTED))
    assert S.n_inside_cells == int(np.sum(P.loc == cut2d.INSIDE))
    rp2, c2, v2 = S.csr()
    assert np.all(np.diff(rp2) >= 1)
    for r in range(0, n, 97):  # ascending columns per row
        assert np.all(np.diff(c2[rp2[r]:rp2[r + 1]].astype(np.int64)) > 0)
    A = sp.csr_matrix((vals, cols, rp), shape=(n, n))
    B = sp.csr_matrix((v2, c2.astype(np.int64), rp2), shape=(n, n))
    assert abs(A - B).max() <= 1e-13 * abs(A).max()
    assert np.max(np.abs(S.rhs() - rhs)) <= 1e-14 * np.max(np.abs(rhs))
    # the library's error functional on the oracle's solution
    u, _ = P.solve(rp, cols, vals, rhs)
    assert abs(S.l2_error(u) - P.l2_error(u)) <= 1e-15


@pytest.mark.parametrize("ghost_penalty,golden,tol", [(True, 4.3420e-04, 1.5e-4), (False, 4.2303e-04, 1e-2)])
def test_cut_assembly_golden(ghost_penalty, golden, tol):
    """without ghost penalty the printed error is that of one unconverged CG
    trajectory on an unstabilised system: this CSR (no structural zeros, other
    SpMV summation order) stops at an iterate with 4.2594e-04 (oracle CSR:
    4.2301e-04, golden 4.2303e-04, converged 4.2918e-04), hence 1 %"""
    g = _lib()
    S = g.CutPoisson(3, 64, ghost_penalty=ghost_penalty)
    rp, c, v = S.csr()
    u, its = O.cg(rp, c.astype(np.int64), v, S.rhs(), precond=0, max_it=S.n_rows, abs_tol=1e-10, rel_tol=1e-6)
    assert its > 0
    e = S.l2_error(u)
    assert abs(e - golden) / golden < tol, e
    assert "%.4f" % S.h == "0.0378"


def test_cut_assembly_converges():
    """O(h^2) L2 convergence of the converged discrete solutions (p = 3,
    ghost penalty) on refinement -- second order because the FE_Q(1) level
    set approximates the circle to O(h^2) (measured 1.77e-3 -> 4.33e-4): the
    assembly is a consistent discretisation, not just a fit to one golden."""
    g = _lib()
    errs = []
    for n in (32, 64):
        S = g.CutPoisson(3, n, ghost_penalty=True)
        rp, c, v = S.csr()
        u, its = O.cg(rp, c.astype(np.int64), v, S.rhs(), precond=0, max_it=50 * S.n_rows, abs_tol=1e-30,
                      rel_tol=1e-13)
        errs.append(S.l2_error(u))
    assert errs[1] < errs[0] / 3.5, errs


def test_cut_assembly_arguments():
    g = _lib()
    with pytest.raises(g.GdmError):
        g.CutPoisson(4, 64)
    with pytest.raises(g.GdmError):
        g.CutPoisson(3, 64, radius=-1.0)
