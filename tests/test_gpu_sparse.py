"""GPU parity of the assembled-sparse-matrix path (include/gdm_hip.h,
"Assembled sparse matrices"; SURVEY §8 a14 + f2) against the oracle.

  * vmult: relative L2 error <= 1e-14 against oracle/gdm_oracle.c:gdmo_csr_vmult
    on the oracle-assembled GDM mass / Laplace matrices (cell-loop assembly,
    pinned to mass_0x / poisson_01 goldens) and on ragged random matrices
    (empty rows, long rows, rectangular, nnz = 0).  fp64 summation order is the
    only difference, hence the tolerance.
  * CG: deal.II SolverCG + ReductionControl semantics (oracle gdmo_cg): the
    device's stopping iteration is where the oracle's residual history
    crosses the threshold (within 1 % of it at rel 1e-6, a factor 2 at rel
    1e-14 where rounding of the residual recurrence is of the order of tol;
    _cg_stop_ok), and the solutions
    agree to the solver tolerance when the counts are equal.
  * triplet files (wave-ev.cc:93-127): bit-exact round trip, deal.II entry order.
  * config 5 size (2D p=3, 4096^2 vertices, full structural stencil): the
    device SpMV equals the same Kronecker operator applied as a 7x7 fp64
    stencil (49 shifted fp64 adds in torch) to <= 1e-13, and is linear.
"""
import os

import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RTOL_SPMV = 1e-14


def _sp():
    from gdm_amd import sparse

    return sparse


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _vmult(A, x, m):
    y = torch.zeros(m, dtype=torch.float64, device="cuda")
    A.vmult(y, dev(x))
    return host(y)


@pytest.mark.parametrize("dim,p,n", [(1, 3, 40), (2, 3, 12), (2, 5, 11), (3, 3, 6), (3, 5, 6)])
@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("lanes", ["", "4", "16", "64"])
def test_vmult_gdm_matrices_vs_oracle(dim, p, n, kind, lanes, monkeypatch):
    if lanes:
        monkeypatch.setenv("GDM_CSR_LANES", lanes)
    sp = _sp()
    m = O.Mesh(dim, p, n, 0.0, 1.0)
    rp, cols, vals = m.matrix_csr(kind=kind)
    A = sp.SparseMatrix(rp, cols.astype(np.uint32), vals)
    assert (A.m(), A.n(), A.n_nonzero_elements()) == (m.n_dofs, m.n_dofs, len(vals))
    x = np.random.default_rng(1).uniform(-1, 1, m.n_dofs)
    assert rel(_vmult(A, x, m.n_dofs), O.csr_vmult(rp, cols, vals, x)) < RTOL_SPMV


def _random_csr(rng, n_rows, n_cols, max_len, empty_frac=0.2):
    lens = rng.integers(0, max_len + 1, n_rows)
    lens[rng.random(n_rows) < empty_frac] = 0
    lens = np.minimum(lens, n_cols)
    rp = np.zeros(n_rows + 1, dtype=np.int64)
    rp[1:] = np.cumsum(lens)
    cols = np.concatenate([np.sort(rng.choice(n_cols, l, replace=False)) for l in lens] or [np.zeros(0)])
    return rp, cols.astype(np.int64), rng.uniform(-1, 1, int(rp[-1]))


@pytest.mark.parametrize("n_rows,n_cols,max_len", [(1, 1, 1), (257, 257, 3), (1000, 700, 40), (300, 5000, 300),
                                                   (5000, 5000, 80), (64, 64, 0)])
@pytest.mark.parametrize("lanes", ["", "2", "8", "32"])
def test_vmult_ragged_vs_oracle(n_rows, n_cols, max_len, lanes, monkeypatch):
    if lanes:
        monkeypatch.setenv("GDM_CSR_LANES", lanes)
    sp = _sp()
    rng = np.random.default_rng(n_rows + max_len)
    rp, cols, vals = _random_csr(rng, n_rows, n_cols, max_len)
    A = sp.SparseMatrix(rp, cols, vals, n_cols=n_cols)
    x = rng.uniform(-1, 1, n_cols)
    y = _vmult(A, x, n_rows)
    ref = np.array([vals[rp[i]:rp[i + 1]] @ x[cols[rp[i]:rp[i + 1]]] for i in range(n_rows)])
    if np.linalg.norm(ref) == 0:
        assert np.all(y == 0)
    else:
        assert rel(y, ref) < RTOL_SPMV


def test_device_arrays_equal_host_arrays():
    sp = _sp()
    m = O.Mesh(2, 5, 20, 0.0, 1.0)
    rp, cols, vals = m.matrix_csr(kind=1)
    A = sp.SparseMatrix(rp, cols.astype(np.uint32), vals)
    B = sp.SparseMatrix(torch.from_numpy(rp).cuda(), torch.from_numpy(cols.astype(np.int32)).cuda(), dev(vals))
    x = np.random.default_rng(2).uniform(-1, 1, m.n_dofs)
    assert np.array_equal(_vmult(A, x, m.n_dofs), _vmult(B, x, m.n_dofs))
    for a, b in zip(A.to_host(), (rp, cols, vals)):
        assert np.array_equal(a, b.astype(a.dtype))


def test_invalid_structure_is_rejected():
    sp = _sp()
    from gdm_amd import GdmError

    rp = np.array([0, 2, 3], dtype=np.int64)
    with pytest.raises(GdmError):
        sp.SparseMatrix(rp, np.array([0, 5, 1], dtype=np.uint32), np.ones(3), n_cols=3)
    with pytest.raises(GdmError):
        sp.SparseMatrix(torch.tensor([0, 2, 3], device="cuda"), torch.tensor([0, 5, 1], dtype=torch.int32,
                                                                              device="cuda"),
                        torch.ones(3, dtype=torch.float64, device="cuda"), n_cols=3)
    with pytest.raises(GdmError):
        sp.SparseMatrix(torch.tensor([0, 3, 2], device="cuda"), torch.tensor([0, 1, 1], dtype=torch.int32,
                                                                              device="cuda"),
                        torch.ones(3, dtype=torch.float64, device="cuda"), n_cols=3)


def _sum_csr(a, b):
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    return a[0], a[1], a[2] + b[2]


def _cg_stop_ok(k, hist, tol, slack):
    """The device's stopping iteration k is consistent with the oracle's
    residual history when the oracle's residual at k is below the threshold
    (within the factor 1 + slack) and every earlier residual is above it
    (within the same factor): identity-CG residuals are not monotone, so an
    exact +-1 window flips on ulp-level changes of the matrix."""
    if k >= len(hist):
        return False
    return hist[k] <= tol * (1 + slack) and bool(np.all(hist[:k] > tol / (1 + slack)))


@pytest.mark.parametrize("dim,p,n", [(1, 3, 64), (2, 3, 16), (2, 5, 12), (3, 3, 7)])
@pytest.mark.parametrize("precond", ["identity", "jacobi"])
def test_cg_vs_oracle(dim, p, n, precond):
    """SPD systems: mass (advection/problem.h:236-267 tolerances) and
    Laplace + mass (cut_poisson_01_gdm.cc:330-335 tolerances)."""
    sp = _sp()
    m = O.Mesh(dim, p, n, 0.0, 1.0)
    b = np.random.default_rng(3).uniform(-1, 1, m.n_dofs)
    mass = m.matrix_csr(kind=0)
    lap_mass = _sum_csr(m.matrix_csr(kind=1), mass)
    pc = 1 if precond == "jacobi" else 0
    for (rp, cols, vals), abs_tol, rel_tol in ((mass, 1e-20, 1e-14), (lap_mass, 1e-10, 1e-6)):
        x_ref, its_ref, _, tol = O.cg_history(rp, cols, vals, b, precond=pc, max_it=5000, abs_tol=abs_tol,
                                              rel_tol=rel_tol)
        assert its_ref > 0
        # Band around tol inside which rounding decides the crossing.  At rel
        # 1e-6 the recurrence residuals of two summation orders agree to far
        # better than 1 %.  At rel 1e-14 the recurrence's rounding (about
        # eps kappa |b|) is itself of the order of tol: device and oracle
        # residuals there differ by up to ~2x (3D p=3 Jacobi mass: the
        # device stops at 64, where the oracle's residual is 1.42 tol), so
        # the band is a factor 2, about one iteration of the decay.
        slack = 1e-2 if rel_tol >= 1e-10 else 1.0
        # the same iterates run past the threshold (a lower one) for the
        # residuals after its_ref
        _, _, hist, _ = O.cg_history(rp, cols, vals, b, precond=pc, max_it=5000, abs_tol=abs_tol / (1 + slack),
                                     rel_tol=rel_tol / (1 + slack))
        A = sp.SparseMatrix(rp, cols.astype(np.uint32), vals)
        # repeated solves: the round-1 defect (a scalar slot read and written
        # in one kernel) showed up in some runs only
        for _ in range(3):
            x = torch.zeros(m.n_dofs, dtype=torch.float64, device="cuda")
            its, res = sp.solve_cg(A, x, dev(b), preconditioner=precond, max_it=5000, abs_tol=abs_tol,
                                   rel_tol=rel_tol)
            assert _cg_stop_ok(its, hist, tol, slack), (its, its_ref, hist[max(its - 2, 0):its + 2] / tol)
            if its == its_ref:
                assert rel(host(x), x_ref) < (1e-10 if rel_tol < 1e-12 else 1e-7)
            r = b - O.csr_vmult(rp, cols, vals, host(x))
            assert abs(np.linalg.norm(r) - res) <= 1e-6 * np.linalg.norm(b)


def test_cg_zero_rhs_and_no_convergence():
    sp = _sp()
    from gdm_amd import GdmError

    m = O.Mesh(2, 3, 16, 0.0, 1.0)
    rp, cols, vals = _sum_csr(m.matrix_csr(kind=1), m.matrix_csr(kind=0))
    A = sp.SparseMatrix(rp, cols.astype(np.uint32), vals)
    x = torch.zeros(m.n_dofs, dtype=torch.float64, device="cuda")
    its, res = sp.solve_cg(A, x, torch.zeros_like(x))
    assert its == 0 and res == 0.0
    b = dev(np.random.default_rng(4).uniform(-1, 1, m.n_dofs))
    with pytest.raises(GdmError):
        sp.solve_cg(A, x, b, max_it=2)


@pytest.mark.parametrize("binary", [True, False])
def test_triplet_round_trip(tmp_path, binary):
    sp = _sp()
    m = O.Mesh(2, 3, 9, 0.0, 1.0)
    rp, cols, vals = m.matrix_csr(kind=1)
    A = sp.SparseMatrix(rp, cols.astype(np.uint32), vals)
    f = tmp_path / ("m.bin" if binary else "m.txt")
    A.write_triplets(f, binary=binary)
    B = sp.SparseMatrix.from_triplets(f, binary=binary)
    for a, b in zip(A.to_host(), B.to_host()):
        assert np.array_equal(a, b)
    if binary:  # deal.II SparsityPattern order: rows ascending, diagonal first
        t = np.fromfile(f, dtype=np.dtype([("r", "<u4"), ("c", "<u4"), ("v", "<f8")]))
        assert len(t) == len(vals)
        starts = np.r_[0, np.flatnonzero(np.diff(t["r"].astype(np.int64))) + 1]
        assert np.all(np.diff(t["r"].astype(np.int64)) >= 0)
        assert np.array_equal(t["c"][starts], t["r"][starts])


def test_triplets_unsorted_with_duplicates(tmp_path):
    sp = _sp()
    f = tmp_path / "d.txt"
    f.write_text("2 1 1.5\n0 0 1\n2 1 0.25\n1 2 -3\n0 2 4\n")
    A = sp.SparseMatrix.from_triplets(f, binary=False)
    rp, ci, v = A.to_host()
    assert rp.tolist() == [0, 2, 3, 4]
    assert ci.tolist() == [0, 2, 2, 1]
    assert v.tolist() == [1.0, 4.0, -3.0, 1.75]


def _bands(p):
    # synthetic SPD Toeplitz bands (config 5 is quoted on structure; values synthetic)
    m = np.array([1.0, 4.0, 9.0, 16.0, 9.0, 4.0, 1.0]) if p == 3 else np.exp(-np.abs(np.arange(-p, p + 1)))
    l = -np.ones(2 * p + 1)
    l[p] = 2 * p + 1.0
    return m, l


def test_config5_full_size_vs_convolution():
    """2D p=3, 4096^2 vertices (16.8 M rows, 823 M stored entries)."""
    sp = _sp()
    n, p = 4096, 3
    mb, lb = _bands(p)
    rp, ci, v = sp.stencil_csr_2d(n, p, [(lb, mb), (mb, lb)])
    assert int(rp[-1]) == int(((np.minimum(np.arange(n) + p, n - 1) - np.maximum(np.arange(n) - p, 0) + 1).sum()) ** 2)
    A = sp.SparseMatrix(rp, ci, v)
    del rp, ci, v
    gen = torch.Generator(device="cuda").manual_seed(20251010)
    x = torch.rand(n * n, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    y = torch.rand(n * n, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    Ax = torch.empty_like(x)
    A.vmult(Ax, x)
    w = np.outer(lb, mb) + np.outer(mb, lb)
    xp = torch.nn.functional.pad(x.view(n, n), (p, p, p, p))
    ref = torch.zeros(n, n, dtype=torch.float64, device="cuda")
    for a in range(2 * p + 1):
        for b in range(2 * p + 1):
            ref += float(w[a, b]) * xp[a:a + n, b:b + n]
    ref = ref.view(-1)
    assert float(torch.linalg.norm(Ax - ref) / torch.linalg.norm(ref)) < 1e-13
    Ay, Axy = torch.empty_like(x), torch.empty_like(x)
    A.vmult(Ay, y)
    A.vmult(Axy, x + 2 * y)
    assert float(torch.linalg.norm(Axy - Ax - 2 * Ay) / torch.linalg.norm(Axy)) < 1e-13


@pytest.mark.parametrize("ghost_penalty", [True, False])
def test_cut_poisson_01_device_cg_golden(ghost_penalty):
    """Config-5 path on the reference's own cut-cell system: the cut-Poisson
    matrix and rhs of prototypes/cut_poisson_01_gdm.cc (2D p=3, 64 cells,
    unit-circle level set, Nitsche, ghost penalty; assembled by the 2D cut-cell
    restatement oracle/cut2d.py, pinned to the same golden on the CPU) solved
    by the device SpMV + SolverCG (identity, ReductionControl(n, 1e-10,
    1e-6), :326-335): the L2 error of the device solution reproduces
    prototypes/cut_poisson_01_gdm.output to the spread of the (unconverged,
    rel 1e-6) CG iterate's error under fp64 summation order: 1.5e-4 with
    ghost penalty, 1 % without (see tests/test_cut_assembly.py)."""
    import cut2d

    sp = _sp()
    P = cut2d.CutPoisson2D(3, 64, ghost_penalty=ghost_penalty)
    rp, cols, vals, rhs = P.assemble()
    _, its_ref = P.solve(rp, cols, vals, rhs)
    n = len(rhs)
    A = sp.SparseMatrix(rp, cols.astype(np.uint32), vals)
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    its, res = sp.solve_cg(A, x, dev(rhs), preconditioner="identity", max_it=n, abs_tol=1e-10, rel_tol=1e-6)
    e = P.l2_error(host(x))
    golden = 4.3420e-04 if ghost_penalty else 4.2303e-04
    # the device sums in another order than deal.II / the oracle: with ghost
    # penalty the printed last digit of the CG iterate's error moves by one
    # (4.34198e-04 oracle, 4.34205e-04 device); without, the unstabilised
    # system's unconverged iterate moves by up to 1 % (4.2301 / 4.2303 / 4.2594 /
    # 4.2631e-04 for four summation orders, converged 4.2918e-04)
    assert abs(e - golden) / golden < (1.5e-4 if ghost_penalty else 1e-2), e
    # (without ghost penalty the iteration count moves with the order as well: 595 oracle, 663 row-block SpMV)
    assert abs(its - its_ref) <= (5 if ghost_penalty else its_ref // 5), (its, its_ref)
    assert res <= 1e-6 * np.linalg.norm(rhs)


def test_cut_poisson_library_device_cg_golden():
    """The product path end to end: the library's own cut-cell assembly
    (gdm_amd.CutPoisson = csrc/gdm_cut.cpp, ghost penalty) -> device CSR ->
    device SolverCG(identity, ReductionControl(n, 1e-10, 1e-6)) -> the
    library's L2 error reproduces prototypes/cut_poisson_01_gdm.output
    (4.3420e-04, to the 1.5e-4 fp64-order spread of the unconverged iterate)."""
    import gdm_amd

    S = gdm_amd.CutPoisson(3, 64, ghost_penalty=True)
    A = S.matrix()
    assert A.m() == S.n_rows and A.n_nonzero_elements() == S.nnz
    x = torch.zeros(S.n_rows, dtype=torch.float64, device="cuda")
    b = dev(S.rhs())
    its, res = gdm_amd.solve_cg(A, x, b, "identity", S.n_rows, 1e-10, 1e-6)
    e = S.l2_error(x)
    assert abs(e - 4.3420e-04) / 4.3420e-04 < 1.5e-4, (e, its)
    # SpMV of the device CSR against the host CSR
    rp, c, v = S.csr()
    u = np.random.default_rng(5).uniform(-1, 1, S.n_rows)
    y = torch.zeros(S.n_rows, dtype=torch.float64, device="cuda")
    A.vmult(y, dev(u))
    assert rel(host(y), O.csr_vmult(rp, c.astype(np.int64), v, u)) < RTOL_SPMV
