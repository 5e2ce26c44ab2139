"""GPU parity: HIP path (through the C ABI) vs the CPU restatement (oracle/).

Tolerances (fp64):
  * operator applications: relative L2 error <= 1e-12 against the
    reference-faithful cell loops (advection/stiffness.h:345-532,
    wave/stiffness.h:151-330, mass.h:144-156),
  * mass solve: <= 1e-10 against CG(rel 1e-14) on the assembled matrix
    (advection/problem.h:236-267),
  * DoF indexing / slab layout / boundary-point order: bit-exact.
"""
import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RTOL_APPLY = 1e-12
RTOL_SOLVE = 1e-10


def _gdm():
    import gdm_amd

    return gdm_amd


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


CASES_SMALL = [
    (1, 1, 9), (1, 3, 17), (1, 5, 23), (1, 7, 31), (1, 9, 20),
    (2, 1, 7), (2, 3, 9), (2, 5, 13), (2, 7, 15), (2, 9, 11),
    (3, 1, 5), (3, 3, 6), (3, 5, 7), (3, 7, 8),
]


@pytest.mark.parametrize("dim,p,n", CASES_SMALL)
def test_mass_apply_vs_cell_loop(dim, p, n):
    g = _gdm()
    op = g.GdmOperator(dim, p, n, -0.3, 1.1, "mass")
    m = O.Mesh(dim, p, n, -0.3, 1.1)
    u = np.random.default_rng(1).uniform(-1, 1, m.n_dofs)
    rp, cols, vals = m.matrix_csr(kind=0)
    ref = O.csr_vmult(rp, cols, vals, u)
    y = op.new_vector(local=False)
    op.apply(dev(u), y)
    assert rel(host(y), ref) < RTOL_APPLY


@pytest.mark.parametrize("dim,p,n", CASES_SMALL)
@pytest.mark.parametrize("a", [(1.0, 0.15, -0.05), (-0.6, 0.9, 0.35)])
def test_advection_apply_vs_cell_loop(dim, p, n, a):
    """compute_rhs block(1): cell term + box faces incl. inflow data u+."""
    g = _gdm()
    a = a[:dim]
    op = g.GdmOperator(dim, p, n, -0.5, 0.5, "advection", params=a)
    m = O.Mesh(dim, p, n, -0.5, 0.5)
    rng = np.random.default_rng(2)
    u = rng.uniform(-1, 1, m.n_dofs)
    nb = m.n_boundary_points()
    assert op.n_bc_points == nb
    bc_ref = rng.uniform(-1, 1, nb)
    perm = op.bc_reference_order()
    assert sorted(perm.tolist()) == list(range(nb))
    bc_dev = np.zeros(nb)
    bc_dev[perm] = bc_ref
    # the device point coordinates in reference order equal the oracle's
    np.testing.assert_allclose(op.bc_points()[perm], m.boundary_points(), atol=1e-13)
    ref = m.advection_rhs(a, u, bc_ref)
    y = op.new_vector(local=False)
    op.apply(dev(u), y, dev(bc_dev))
    assert rel(host(y), ref) < RTOL_APPLY


@pytest.mark.parametrize("dim,p,n", [(2, 5, (600, 9)), (2, 9, (9, 530)), (3, 5, (300, 7, 6)), (3, 3, (5, 270, 4))])
def test_advection_inflow_faces_multi_chunk(dim, p, n):
    """Faces whose tangential node range spans several face-kernel chunks
    (FACE_CHUNK = 256 nodes per workgroup)."""
    g = _gdm()
    a = (0.7, 0.4, -0.3)[:dim]
    op = g.GdmOperator(dim, p, n, 0.0, 1.0, "advection", params=a)
    m = O.Mesh(dim, p, list(n), 0.0, 1.0)
    rng = np.random.default_rng(12)
    u = rng.uniform(-1, 1, m.n_dofs)
    bc_ref = rng.uniform(-1, 1, m.n_boundary_points())
    bc_dev = np.zeros_like(bc_ref)
    bc_dev[op.bc_reference_order()] = bc_ref
    ref = m.advection_rhs(a, u, bc_ref)
    y = op.new_vector(local=False)
    op.apply(dev(u), y, dev(bc_dev))
    assert rel(host(y), ref) < RTOL_APPLY
    # the boundary-data part alone (linearity in u+)
    ref0 = m.advection_rhs(a, u, np.zeros_like(bc_ref))
    z = op.new_vector(local=False)
    op.add_boundary_data(dev(bc_dev), z)
    assert rel(host(z), ref - ref0) < 1e-11


@pytest.mark.parametrize("dim,p,n", CASES_SMALL)
@pytest.mark.parametrize("nitsche", [0.0, 15.0])
def test_wave_apply_vs_cell_loop(dim, p, n, nitsche):
    g = _gdm()
    params = (nitsche,) if nitsche > 0 else ()
    op = g.GdmOperator(dim, p, n, -1.21, 1.21, "wave", params=params)
    m = O.Mesh(dim, p, n, -1.21, 1.21)
    u = np.random.default_rng(3).uniform(-1, 1, m.n_dofs)
    ref = m.wave_rhs(u, impl=True, nitsche=nitsche)
    y = op.new_vector(local=False)
    op.apply(dev(u), y)
    assert rel(host(y), ref) < RTOL_APPLY


@pytest.mark.parametrize("dim,p,n", [(1, 3, 40), (2, 5, 12), (3, 3, 7)])
def test_convective_apply_vs_cell_loop(dim, p, n):
    g = _gdm()
    a = (1.0, 0.15, -0.05)[:dim]
    op = g.GdmOperator(dim, p, n, 0.0, 1.0, "convective", params=a)
    m = O.Mesh(dim, p, n)
    u = np.random.default_rng(4).uniform(-1, 1, m.n_dofs)
    ref = m.convective_rhs(a, u)
    y = op.new_vector(local=False)
    op.apply(dev(u), y)
    assert rel(host(y), ref) < RTOL_APPLY


@pytest.mark.parametrize("dim,p,n", [(1, 3, 40), (1, 9, 30), (2, 3, 12), (2, 5, 17), (3, 5, 9), (3, 7, 8)])
def test_mass_solve_vs_cg(dim, p, n):
    g = _gdm()
    op = g.GdmOperator(dim, p, n, 0.0, 2.0, "mass")
    m = O.Mesh(dim, p, n, 0.0, 2.0)
    r = np.random.default_rng(5).uniform(-1, 1, m.n_dofs)
    rp, cols, vals = m.matrix_csr(kind=0)
    x_ref, its = O.cg(rp, cols, vals, r, precond=1, max_it=5000, abs_tol=1e-20, rel_tol=1e-14)
    x = op.new_vector(local=False)
    op.mass_solve(dev(r), x)
    assert rel(host(x), x_ref) < RTOL_SOLVE


@pytest.mark.parametrize("shape", [(70, 33, 20), (64, 64, 64), (131, 5, 9), (8, 9, 100), (97, 61, 130), (300, 40)])
@pytest.mark.parametrize("p", [3, 5, 7])
@pytest.mark.parametrize("in_place", [False, True])
def test_mass_solve_ragged_vs_kron(shape, p, in_place):
    """Mass inverse v2 (gdm_mass.hip: strided z/y passes, LDS-staged x pass)
    on ragged sizes (odd row lengths: no 16-B vector rows), out of place and
    in place, against the Kronecker inverse of the oracle's 1D matrices."""
    g = _gdm()
    dim = len(shape)
    n = tuple(max(s, p) for s in shape)
    lo, hi = (0.0,) * dim, (1.0, 0.7, 1.3)[:dim]
    op = g.GdmOperator(dim, p, n, lo, hi, "mass")
    m = O.Mesh(dim, p, list(n), lo, hi)
    r = np.random.default_rng(21).uniform(-1, 1, m.n_dofs)
    ref = m.kron_mass_inverse(r)
    rd = dev(r)
    x = rd if in_place else op.new_vector(local=False)
    op.mass_solve(rd, x)
    assert rel(host(x), ref) < 1e-12


@pytest.mark.parametrize("shape", [(499, 7, 8), (7, 433, 8), (7, 8, 601), (239, 190), (1023, 7), (8, 7, 145)])
@pytest.mark.parametrize("p", [3, 5, 7])
def test_mass_solve_v3_long_lines(shape, p):
    """Mass inverse v3 (single-sweep line solves with the truncated backward
    warm-up, gdm_mass.hip) on lines of many chunks (C = 48 / 56 positions),
    lengths that are not chunk multiples, both the table and the interior
    fixed-point coefficient paths: against the exact Kronecker inverse (the
    oracle's two-sweep banded Cholesky, oracle/gdm_oracle_kron.c)."""
    g = _gdm()
    dim = len(shape)
    lo, hi = (0.0,) * dim, (1.0, 0.7, 1.3)[:dim]
    m = O.Mesh(dim, p, list(shape), lo, hi)
    r = np.random.default_rng(33).uniform(-1, 1, m.n_dofs)
    ref = m.kron_mass_inverse(r)
    op = g.GdmOperator(dim, p, shape, lo, hi, "mass")
    x = op.new_vector(local=False)
    op.mass_solve(dev(r), x)
    got = host(x)
    assert rel(got, ref) < 1e-12
    assert np.max(np.abs(got - ref)) < 1e-13 * np.max(np.abs(ref))


@pytest.mark.parametrize("shape", [(70, 33, 20), (64, 64, 64), (131, 5, 9), (5, 5, 100), (150, 90, 70), (97, 61, 130)])
@pytest.mark.parametrize("p", [5, 7])
def test_ragged_3d_vs_kron(shape, p):
    """Ragged / non-multiple-of-tile sizes against the Kronecker oracle."""
    g = _gdm()
    n = tuple(max(s, p) for s in shape)
    a = (0.8, -0.3, 0.45)
    op = g.GdmOperator(3, p, n, (0, 0, 0), (1.0, 0.7, 1.3), "advection", params=a)
    m = O.Mesh(3, p, n, (0, 0, 0), (1.0, 0.7, 1.3))
    u = np.random.default_rng(6).uniform(-1, 1, m.n_dofs)
    M = [m.matrices_1d(d)[0] for d in range(3)]
    B = [m.advection_outflow_B(d, a[d]) for d in range(3)]
    ref = m.kron_apply([(B[0], M[1], M[2]), (M[0], B[1], M[2]), (M[0], M[1], B[2])], u)
    y = op.new_vector(local=False)
    op.apply(dev(u), y)
    assert rel(host(y), ref) < RTOL_APPLY


@pytest.mark.parametrize("kind", ["mass", "wave"])
@pytest.mark.parametrize("p", [5, 7])
def test_stencil_walls_3d_vs_kron(kind, p):
    """Shapes large enough for the v8 stencil (wall rows handled by
    corrections, interior-z split): mass and wave (+ Nitsche) vs Kronecker."""
    g = _gdm()
    n = (130, 75, 66)
    op = g.GdmOperator(3, p, n, (-1.0, 0.0, 0.5), (1.2, 0.9, 1.4), kind)
    m = O.Mesh(3, p, n, (-1.0, 0.0, 0.5), (1.2, 0.9, 1.4))
    u = np.random.default_rng(9).uniform(-1, 1, m.n_dofs)
    M = [m.matrices_1d(d)[0] for d in range(3)]
    if kind == "mass":
        terms = [(M[0], M[1], M[2])]
    else:
        B = [-m.matrices_1d(d)[2] for d in range(3)]
        terms = [(B[0], M[1], M[2]), (M[0], B[1], M[2]), (M[0], M[1], B[2])]
    ref = m.kron_apply(terms, u)
    y = op.new_vector(local=False)
    op.apply(dev(u), y)
    assert rel(host(y), ref) < RTOL_APPLY


@pytest.mark.parametrize("p", [5, 7])
def test_stencil_walls_2d_vs_cell_loop(p):
    """2D meshes large enough for the v8 stencil: wave with box Nitsche
    (rank-2 wall-row terms) and advection with inflow data vs the cell loops."""
    g = _gdm()
    n = (80, 50)
    m = O.Mesh(2, p, list(n), -1.21, 1.21)
    rng = np.random.default_rng(10)
    u = rng.uniform(-1, 1, m.n_dofs)
    op = g.GdmOperator(2, p, n, -1.21, 1.21, "wave", params=(15.0,))
    y = op.new_vector(local=False)
    op.apply(dev(u), y)
    assert rel(host(y), m.wave_rhs(u, impl=True, nitsche=15.0)) < RTOL_APPLY
    a = (-0.6, 0.9)
    op = g.GdmOperator(2, p, n, -1.21, 1.21, "advection", params=a)
    bc_ref = rng.uniform(-1, 1, m.n_boundary_points())
    bc_dev = np.zeros_like(bc_ref)
    bc_dev[op.bc_reference_order()] = bc_ref
    y = op.new_vector(local=False)
    op.apply(dev(u), y, dev(bc_dev))
    assert rel(host(y), m.advection_rhs(a, u, bc_ref)) < RTOL_APPLY


def test_full_size_properties_3d_p5():
    """BASELINE config C3 (512^3 DoFs, p=5): size-independent properties.
    Linearity of the stiffness action and M^-1 (M u) == u."""
    g = _gdm()
    n = 511
    op = g.GdmOperator(3, 5, n, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05))
    N = op.n_owned
    assert N == 512 ** 3
    gen = torch.Generator(device="cuda").manual_seed(20251010)
    u = torch.rand(N, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    v = torch.rand(N, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    Ku, Kv, Kw = (op.new_vector(local=False) for _ in range(3))
    op.apply(u, Ku)
    op.apply(v, Kv)
    w = 0.3 * u - 1.7 * v
    op.apply(w, Kw)
    lin = torch.linalg.norm(Kw - (0.3 * Ku - 1.7 * Kv)) / torch.linalg.norm(Kw)
    assert float(lin) < 1e-13
    del Kv, Kw, v, w
    Mu = op.new_vector(local=False)
    op.mass_apply(u, Mu)
    x = op.new_vector(local=False)
    op.mass_solve(Mu, x)
    err = torch.linalg.norm(x - u) / torch.linalg.norm(u)
    assert float(err) < 1e-12


@pytest.mark.gpu
def test_mass_solve_line_span_above_2gb():
    """A z-line spanning more than 2^31 bytes ((Z-1) * X * Y * 8 = 2.29e9 at
    640 x 640 x 700 vertices, 2.3 GB per vector): the v3 strided kernel's
    32-bit buffer offsets cannot reach it, so the pass must take the 64-bit
    addressed v2 kernel.  M^-1 (M u) == u over the whole vector,
    and over the last z-planes (the part a 32-bit offset would drop)."""
    g = _gdm()
    n = (639, 639, 699)
    op = g.GdmOperator(3, 5, n, 0.0, 1.0, "mass")
    N = op.n_owned
    assert (n[2]) * 640 * 640 * 8 > 2 ** 31
    gen = torch.Generator(device="cuda").manual_seed(7)
    u = torch.rand(N, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    Mu = op.new_vector(local=False)
    op.mass_apply(u, Mu)
    x = op.new_vector(local=False)
    op.mass_solve(Mu, x)
    del Mu
    err = torch.linalg.norm(x - u) / torch.linalg.norm(u)
    tail = slice(N - 40 * 640 * 640, N)
    err_tail = torch.linalg.norm(x[tail] - u[tail]) / torch.linalg.norm(u[tail])
    assert float(err) < 1e-12 and float(err_tail) < 1e-12, (float(err), float(err_tail))


@pytest.mark.parametrize("n_ranks,shape,p,kind", [
    (2, (20, 18, 31), 5, "advection"),
    (3, (140, 70, 100), 5, "advection"),
    (4, (90, 60, 121), 7, "wave"),
    (2, (100, 50, 64), 5, "mass"),
])
def test_slab_ranks_match_single_rank(n_ranks, shape, p, kind):
    """The z-slab partition (system.h:720-757) evaluated rank by rank in one
    process: each rank's operator on its [ghost | owned | ghost] local vector,
    ghosts filled from the global vector exactly as HaloExchange does, must
    reproduce the single-rank result on the owned planes (bit-identical DoF
    numbering, fp64 tolerance for the values).  Advection includes the inflow
    data of the x/y faces, whose owned nodes near a slab edge also collect the
    neighbour cells' boundary points (owner-computes instead of compress(add))."""
    g = _gdm()
    from gdm_amd.distributed import layout as slab_layout

    a = (0.7, -0.4, 0.3)
    params = a if kind == "advection" else ((9.0,) if kind == "wave" else ())
    lo, hi = (0.0, -0.5, 0.2), (1.0, 0.5, 1.7)
    full = g.GdmOperator(3, p, shape, lo, hi, kind, params=params)
    u = torch.rand(full.n_owned, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(3))
    def bc_for(op):  # smooth inflow data at the operator's device boundary points (ghost-cell points included)
        if kind != "advection":
            return None
        x = op.bc_points()
        return dev(np.sin(3 * x[:, 0] + 1) * np.cos(2 * x[:, 1] - 0.5) + x[:, 2])

    ref = full.new_vector(local=False)
    full.apply(u, ref, bc_for(full))
    ps = full.layout["plane_size"]
    out = torch.zeros_like(ref)
    for r in range(n_ranks):
        op = g.GdmOperator(3, p, shape, lo, hi, kind, params=params, rank=r, n_ranks=n_ranks)
        L = op.layout
        assert L == {**L, **{k: v for k, v in slab_layout(shape[2], n_ranks, r, ps, p).items() if k in L}}
        first = L["owned_plane_begin"] - L["ghost_planes_below"]
        local = u[first * ps:first * ps + L["n_local"]].clone()
        y = op.new_vector(local=False)
        op.apply(local, y, bc_for(op))
        assert op.n_bc_points_ref <= op.n_bc_points
        b = L["owned_plane_begin"] * ps
        out[b:b + L["n_owned"]] = y
    torch.cuda.synchronize()
    assert rel(host(out), host(ref)) < RTOL_APPLY


@pytest.mark.parametrize("dim,p,n", [(1, 5, 40), (2, 3, 30), (3, 5, 24), (3, 7, 17)])
def test_mass_solve_lines_compose_to_mass_solve(dim, p, n):
    """gdm_mass_solve_lines along every direction (the building block of the
    slab-distributed inverse, gdm_amd.distributed.DistributedMassSolve) ==
    gdm_mass_solve; the distributed driver on one rank uses exactly that path."""
    g = _gdm()
    from gdm_amd.distributed import DistributedMassSolve

    op = g.GdmOperator(dim, p, n, 0.0, 1.5, "mass")
    m = O.Mesh(dim, p, n, 0.0, 1.5)
    r = dev(np.random.default_rng(13).uniform(-1, 1, m.n_dofs))
    x1 = op.new_vector(local=False)
    op.mass_solve(r, x1)
    x2 = op.new_vector(local=False)
    DistributedMassSolve(dim, [n + 1] * dim, 1, 0, op=op).solve(r, x2)
    assert rel(host(x2), host(x1)) < 1e-14
    ref = m.kron_mass_inverse(host(r))
    assert rel(host(x2), ref) < 1e-12


@pytest.mark.parametrize("n_ranks,rank", [(3, 1), (3, 0), (4, 3)])
def test_apply_planes_overlap_split(n_ranks, rank):
    """apply_overlapped's plane split (interior planes during the exchange,
    the p planes at each slab edge after it) == one gdm_apply on that rank."""
    g = _gdm()
    from gdm_amd.distributed import apply_overlapped

    shape, p = (100, 70, 120), 5
    a = (0.7, -0.4, 0.3)
    op = g.GdmOperator(3, p, shape, 0.0, 1.0, "advection", params=a, rank=rank, n_ranks=n_ranks)
    gen = torch.Generator(device="cuda").manual_seed(5)
    src = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen)
    bc = torch.rand(op.n_bc_points, dtype=torch.float64, device="cuda", generator=gen)
    y1, y2 = op.new_vector(local=False), op.new_vector(local=False)
    op.apply(src, y1, bc)
    y2.fill_(7.0)
    apply_overlapped(op, None, src, y2, bc)
    assert rel(host(y2), host(y1)) < 1e-14


@pytest.mark.parametrize("p,kind", [(5, "advection"), (7, "wave")])
def test_apply_planes2_equals_two_range_launches(p, kind):
    """gdm_apply_planes2 (both slab-edge ranges in one launch, ABI 13) gives
    the bits of two gdm_apply_planes calls; overlapping ranges are refused."""
    g = _gdm()
    shape = (100, 70, 64)
    params = (0.7, -0.4, 0.3) if kind == "advection" else ()
    op = g.GdmOperator(3, p, shape, 0.0, 1.0, kind, params=params, rank=1, n_ranks=3)
    L = op.layout
    pb, pe = L["owned_plane_begin"], L["owned_plane_end"]
    gen = torch.Generator(device="cuda").manual_seed(9)
    src = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen)
    y1, y2 = op.new_vector(local=False), op.new_vector(local=False)
    y1.fill_(3.0)
    y2.fill_(3.0)
    op.apply_planes(src, y1, pb, pb + p)
    op.apply_planes(src, y1, pe - p, pe)
    op.apply_planes2(src, y2, pb, pb + p, pe - p, pe)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    with pytest.raises(g.GdmError, match="overlapping"):
        op.apply_planes2(src, y2, pb, pb + 2 * p, pb + p, pe)
    # a first range wholly in the ghost planes is clipped away; the second
    # still runs
    y3, y4 = op.new_vector(local=False), op.new_vector(local=False)
    y3.fill_(3.0)
    y4.fill_(3.0)
    op.apply_planes2(src, y3, pb - p, pb, pe - p, pe)
    op.apply_planes(src, y4, pe - p, pe)
    op.apply_planes2(src, y3, pb, pb + p, pe, pe + p)
    op.apply_planes(src, y4, pb, pb + p)
    torch.cuda.synchronize()
    assert torch.equal(y3, y4) and torch.equal(y3, y1)
