"""Periodicity constraints and the matrix-free CG (config C1,
prototypes/advection_01_gdm.cc) on the device vs the oracle.

Oracle side: the reference-faithful convective cell loop (oracle/gdm_oracle.c
gdmo_convective_rhs, advection_01_gdm.cc:164-206) wrapped in the
AffineConstraints semantics of System::make_periodicity_constraints
(system.h:427-463): distribute the input (x_last = x_first per direction),
condense the assembled vector and matrix (P^T r, P^T M P; constrained rows
decoupled), SolverCG + PreconditionJacobi (oracle/gdm_oracle.c gdmo_cg,
deal.II ReductionControl semantics) from zero, RK4 + DiscreteTime from
oracle/cut1d.py (pinned by the wave_0 / heat_1 goldens).

Tolerances: per-solve CG iteration counts identical; solution after the RK
steps rel-L2 <= 1e-9 (CG to rel 1e-8 on both sides, same iterates up to
round-off).
"""
import numpy as np
import pytest
import scipy.sparse as sp

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


class PeriodicOracle:
    def __init__(self, m):
        self.m = m
        N = m.n_dofs
        Ns = m.N
        idx = np.arange(N)
        coords = [idx % Ns[0], (idx // Ns[0]) % Ns[1], idx // (Ns[0] * Ns[1])]
        master = idx.copy()
        self.constrained = np.zeros(N, dtype=bool)
        stride = [1, Ns[0], Ns[0] * Ns[1]]
        for d in range(m.dim):  # chains resolve to the first vertex of every periodic direction
            at_end = coords[d] == Ns[d] - 1
            master = np.where(at_end, master - (Ns[d] - 1) * stride[d], master)
            self.constrained |= at_end
        self.P = sp.csr_matrix((np.ones(N), (idx, master)), shape=(N, N))
        rp, cols, vals = m.matrix_csr(kind=0)
        M = sp.csr_matrix((vals, cols, rp), shape=(N, N))
        A = (self.P.T @ M @ self.P).tolil()
        for i in np.where(self.constrained)[0]:
            A[i, i] = 1.0
        A = A.tocsr()
        A.sort_indices()
        self.A = (A.indptr.astype(np.int64), A.indices.astype(np.int64), A.data)

    def distribute(self, u):
        return self.P @ u

    def condense(self, r):
        return self.P.T @ r

    def rhs(self, a, u, its):
        r = self.condense(self.m.convective_rhs(a, self.distribute(u)))
        x, it = O.cg(*self.A, r, precond=1, max_it=100, abs_tol=1e-10, rel_tol=1e-8)
        its.append(it)
        return x


def _exact(m, t, a):
    X = m.vertex_coords()
    v = np.sin(2.0 * np.pi * (X[0] - a[0] * t))
    for d in range(1, m.dim):
        v = v * np.cos(2.0 * np.pi * (X[d] - a[d] * t))
    return v


@pytest.mark.parametrize("dim,p,n,steps", [(1, 3, 1024, None), (1, 5, 40, None), (2, 3, 20, 4), (2, 5, 12, 3)])
def test_advection_01_periodic_vs_oracle(dim, p, n, steps):
    """C1 = advection_01_gdm with dim = 1, p = 3, 1024 cells, dt = 0.5 / n,
    t in [0, 0.1] (all 205 steps); smaller 1D / 2D cases for p = 5."""
    import gdm_amd

    a = (1.0, 0.15, -0.05)[:dim]
    m = O.Mesh(dim, p, n)
    orc = PeriodicOracle(m)
    u0 = _exact(m, 0.0, a)
    dt = 1.0 / n * 0.5
    its_ref = []
    u = u0.copy()
    time = cut1d.DiscreteTime(0.0, 0.1, dt)
    k = 0
    while not time.is_at_end() and (steps is None or k < steps):
        u = cut1d.rk4_step(lambda t, y: orc.rhs(a, y, its_ref), time.t, time.next_step_size(), u)
        u = orc.distribute(u)
        time.advance()
        k += 1
    op = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "convective", params=a, periodic=(1 << dim) - 1)
    prob = gdm_amd.Advection01(op)
    prob.u.copy_(dev(u0))
    assert prob.run(0.0, 0.1, dt, max_steps=steps) == k
    assert prob.cg_iterations == its_ref
    assert rel(host(prob.u), u) < 1e-9
    if dim == 1 and n == 1024:
        assert k == 205
        # the transported sine after t = 0.1: the scheme's error, not the parity bound
        assert rel(host(prob.u), _exact(m, 0.1, a)) < 1e-6


@pytest.mark.parametrize("dim,p,n", [(1, 3, 30), (2, 5, 11), (3, 3, 6)])
def test_periodic_mass_apply_and_cg_vs_condensed(dim, p, n):
    """gdm_mass_apply with periodic constraints = P^T M P u (constrained rows
    zero); gdm_mass_solve_cg (Jacobi, rel 1e-12) solves the condensed system;
    the exact Kronecker solve refuses periodic meshes."""
    import gdm_amd

    m = O.Mesh(dim, p, n)
    orc = PeriodicOracle(m)
    op = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass", periodic=(1 << dim) - 1)
    rng = np.random.default_rng(4)
    u = rng.uniform(-1, 1, m.n_dofs)
    y = op.new_vector(False)
    op.mass_apply(dev(u), y)
    rp, cols, vals = orc.A
    ref = O.csr_vmult(rp, cols, vals, orc.distribute(u) * 1.0)
    ref[orc.constrained] = 0.0
    assert rel(host(y), ref) < 1e-13
    b = orc.condense(rng.uniform(-1, 1, m.n_dofs))
    x_ref, it_ref = O.cg(rp, cols, vals, b, precond=1, max_it=1000, abs_tol=1e-20, rel_tol=1e-12)
    x = op.new_vector(False)
    its, res = op.mass_solve_cg(dev(b), x, rel_tol=1e-12, abs_tol=1e-20, max_it=1000, precond=1)
    assert its == it_ref
    assert rel(host(x), x_ref) < 1e-10
    with pytest.raises(gdm_amd.GdmError):
        op.mass_solve(dev(b), x)


def test_mass_solve_cg_nonperiodic_matches_exact():
    """gdm_mass_solve_cg (Jacobi) on a plain mesh converges to the exact
    Kronecker inverse and reports the oracle's CG iteration count."""
    import gdm_amd

    m = O.Mesh(2, 5, 17, 0.0, 2.0)
    op = gdm_amd.GdmOperator(2, 5, 17, 0.0, 2.0, "mass")
    r = np.random.default_rng(5).uniform(-1, 1, m.n_dofs)
    rp, cols, vals = m.matrix_csr(kind=0)
    x_ref, it_ref = O.cg(rp, cols, vals, r, precond=1, max_it=1000, abs_tol=1e-20, rel_tol=1e-14)
    x = op.new_vector(False)
    its, _ = op.mass_solve_cg(dev(r), x, rel_tol=1e-14, abs_tol=1e-20, max_it=1000, precond=1)
    assert abs(its - it_ref) <= 1
    assert rel(host(x), m.kron_mass_inverse(r)) < 1e-10
