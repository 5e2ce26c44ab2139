"""Device postprocess: gdm_error_norms vs the oracle.

Oracle: oracle/gdm_oracle.c gdmo_error_norms -- the cell loop of
integrate_difference (include/gdm/vector_tools.h:25-86) and of the volume part
of the advection postprocess (applications/advection/include/gdm/advection/
problem.h:330-425), whose L2 branch is pinned by the poisson_01 / mass_01
goldens (tests/test_oracle_golden.py).  The exact function is evaluated in
numpy at the oracle's cell quadrature points.

Tolerances: Linf, L1, L2 rel <= 1e-11 (summation order differs); per-cell L2
errors <= 1e-11 * max.  Multi-rank: the per-rank norms reduced as the
reference does (max, sum, sqrt of the sum of squares) equal the one-rank
norms to 1e-12.
"""
import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


SINE = [0.7, -0.3, 0.2, 1.0, 2.0, 1.5, 0.1, 0.4, -0.2]


def exact(kind, prm, X, t, dim):
    """X: (n, 3) coordinates.  Same definitions as include/gdm_hip.h gdm_fn_kind."""
    if kind == 0:
        return np.full(len(X), prm[0])
    if kind == 1:
        r = np.sqrt(sum((X[:, d] - prm[1 + d]) ** 2 for d in range(dim)))
        return np.maximum(0.0, prm[0] - r)
    v = np.ones(len(X))
    for d in range(dim):
        v = v * np.sin(2 * np.pi * prm[3 + d] * (X[:, d] - prm[d] * t) + prm[6 + d])
    return v


def field(m, kind, prm, t, seed):
    """vertex interpolant of the exact function plus noise (so errors are O(1e-2))"""
    V = m.vertex_coords()
    X = np.zeros((m.n_dofs, 3))
    for d in range(m.dim):
        X[:, d] = V[d]
    u = exact(kind, prm, X, t, m.dim)
    return u + 0.01 * np.random.default_rng(seed).standard_normal(m.n_dofs)


def reference(m, u, kind, prm, t):
    xq = m.cell_qpoints()
    return m.error_norms(u, exact(kind, prm, xq, t, m.dim), cells=True)


CASES = [
    (1, 3, 37, 2, SINE), (1, 9, 23, 1, [0.3, 0.4]), (2, 5, (19, 13), 2, SINE), (2, 1, 17, 0, [0.25]),
    (3, 3, (9, 7, 8), 2, SINE), (3, 5, (11, 9, 10), 1, [0.4, 0.1, 0.2, -0.3]), (3, 7, 9, 2, SINE),
    (3, 5, (70, 6, 6), 2, SINE),  # two x chunks of 64 cells
]


@pytest.mark.parametrize("dim,p,n,kind,prm", CASES)
def test_error_norms_vs_oracle(dim, p, n, kind, prm):
    import gdm_amd

    m = O.Mesh(dim, p, n, -0.5, 1.25)
    op = gdm_amd.GdmOperator(dim, p, n, -0.5, 1.25, "mass")
    t = 0.37
    u = field(m, kind, prm, t, seed=dim * 10 + p)
    (ref, ref_cells) = reference(m, u, kind, prm, t)
    cells = torch.zeros(op.n_owned_cells, dtype=torch.float64, device="cuda")
    got = op.error_norms(dev(u), kind, prm, t, cells)
    for g, r in zip(got, ref):
        assert abs(g - r) <= 1e-11 * abs(r), (got, ref)
    c = host(cells)
    assert np.max(np.abs(c - ref_cells)) <= 1e-11 * np.max(ref_cells)


@pytest.mark.parametrize("dim,p,n,n_ranks", [(3, 5, (12, 10, 23), 3), (2, 3, (20, 17), 2), (1, 5, 41, 2)])
def test_error_norms_multi_rank(dim, p, n, n_ranks):
    """owned-cell norms of each rank's slab, reduced max / sum / sqrt(sum sq)
    (problem.h:410-425), reproduce the one-rank norms; cell errors tile."""
    import gdm_amd

    m = O.Mesh(dim, p, n)
    u = field(m, 2, SINE, 0.1, seed=7)
    one = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass")
    ref = one.error_norms(dev(u), 2, SINE, 0.1)
    ref_cells = torch.zeros(one.n_owned_cells, dtype=torch.float64, device="cuda")
    one.error_norms(dev(u), 2, SINE, 0.1, ref_cells)
    linf, l1, l2sq, cells = 0.0, 0.0, 0.0, []
    for r in range(n_ranks):
        op = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass", n_ranks=n_ranks, rank=r)
        L = op.layout
        first = (L["owned_plane_begin"] - L["ghost_planes_below"]) * L["plane_size"]
        loc = dev(u[first:first + op.n_local])
        c = torch.zeros(max(op.n_owned_cells, 1), dtype=torch.float64, device="cuda")
        e = op.error_norms(loc, 2, SINE, 0.1, c if op.n_owned_cells else None)
        linf, l1, l2sq = max(linf, e[0]), l1 + e[1], l2sq + e[2] ** 2
        cells.append(host(c)[:op.n_owned_cells])
    assert abs(linf - ref[0]) <= 1e-14 * ref[0]
    assert abs(l1 - ref[1]) <= 1e-12 * ref[1]
    assert abs(np.sqrt(l2sq) - ref[2]) <= 1e-12 * ref[2]
    np.testing.assert_allclose(np.concatenate(cells), host(ref_cells), rtol=0, atol=1e-15 * float(ref[0]) + 1e-300)


def test_error_norms_convergence_full_size():
    """Size-independent property at a C3-class size: the GDM vertex interpolant
    of a smooth function converges at O(h^(p+1)) in L2 (p = 5: factor ~64 per
    halving); the device evaluation sees it on 64^3 -> 128^3 -> 256^3 cells."""
    import gdm_amd

    prm = [0.0, 0.0, 0.0, 1.0, 1.0, 1.0, 0.3, 0.1, 0.2]
    errs = []
    for n in (32, 64, 128):
        op = gdm_amd.GdmOperator(3, 5, n, 0.0, 1.0, "mass")
        x = torch.linspace(0.0, 1.0, n + 1, dtype=torch.float64, device="cuda")
        sx = torch.sin(2 * np.pi * x + 0.3)
        sy = torch.sin(2 * np.pi * x + 0.1)
        sz = torch.sin(2 * np.pi * x + 0.2)
        u = (sz[:, None, None] * sy[None, :, None] * sx[None, None, :]).reshape(-1).contiguous()
        errs.append(op.error_norms(u, 2, prm, 0.0))
    for a, b in zip(errs, errs[1:]):
        assert 40.0 < a[2] / b[2] < 90.0, errs
        assert 40.0 < a[1] / b[1] < 90.0, errs
