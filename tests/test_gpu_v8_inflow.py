"""The timed path of the bench metric against the oracle in 3D (VERDICT r5
item 1): compute_rhs with inflow data on meshes large enough for the v8
stencil (y extent >= TY + 2p + 2, x extent >= 64 + 2p + 2 vertices,
gdm_capi.cpp launch_stencil), where the inflow faces' step 1 runs as the
stencil launch's tail work (row blocks claimed from a device counter) and
step 2 + the ordered adds follow in one launch.

Reference: advection/stiffness.h:345-532 -- the volume and outflow terms
through the oracle's Kronecker form (oracle/gdm_oracle_kron.c, pinned to the
cell loop in tests/test_oracle_kron.py), the inflow term (III, a.n < 0)
through the oracle's boundary-cell loop gdmo_advection_inflow, which equals
the cell loop gdmo_advection_rhs(u = 0) bit for bit (tests/test_oracle_golden.py).
All 8 sign patterns of the advection field, so every box face is an inflow
face in some case.  Tolerance rel-L2 1e-12 (fp64 summation order)."""
import itertools

import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SIGNS = list(itertools.product((1.0, -1.0), repeat=3))
A_MAG = (0.8, 0.45, 0.3)


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def _host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def _volume_ref(m, a, u):
    M = [m.matrices_1d(d)[0] for d in range(3)]
    B = [m.advection_outflow_B(d, a[d]) for d in range(3)]
    return m.kron_apply([(B[0], M[1], M[2]), (M[0], B[1], M[2]), (M[0], M[1], B[2])], u)


@pytest.mark.parametrize("shape,p", [((100, 70, 64), 5), ((130, 75, 66), 3), ((130, 75, 66), 5), ((90, 40, 50), 7)])
@pytest.mark.parametrize("signs", SIGNS, ids=lambda s: "".join("+" if v > 0 else "-" for v in s))
def test_v8_compute_rhs_with_inflow_vs_oracle(shape, p, signs):
    import gdm_amd

    a = tuple(s * v for s, v in zip(signs, A_MAG))
    lo, hi = (-0.5, 0.0, 0.2), (0.7, 0.9, 1.5)
    op = gdm_amd.GdmOperator(3, p, shape, lo, hi, "advection", params=a)
    m = O.Mesh(3, p, list(shape), lo, hi)
    rng = np.random.default_rng(hash((shape, p, signs)) & 0xFFFF)
    u = rng.uniform(-1, 1, m.n_dofs)
    nb = m.n_boundary_points()
    assert op.n_bc_points == nb
    bc_ref = rng.uniform(-1, 1, nb)
    bc_dev = np.zeros(nb)
    bc_dev[op.bc_reference_order()] = bc_ref
    inflow = m.advection_inflow(a, bc_ref)
    ref = _volume_ref(m, a, u) + inflow
    ud, bd = _dev(u), _dev(bc_dev)
    # compute_rhs as the bench times it: volume + inflow tail + step 2 / adds
    y = op.new_vector(local=False)
    op.apply(ud, y, bd)
    got = _host(y)
    assert _rel(got, ref) < 1e-12
    # the inflow part alone: y(u, bc) - y(u) against the boundary-cell oracle
    y0 = op.new_vector(local=False)
    op.apply(ud, y0)
    assert _rel(got - _host(y0), inflow) < 1e-11
    # the separate face launches (gdm_add_boundary_data) agree with the tail form
    z = op.new_vector(local=False)
    op.add_boundary_data(bd, z)
    assert _rel(_host(z), inflow) < 1e-11


@pytest.mark.parametrize("shape,p", [((100, 70, 64), 5), ((130, 75, 66), 3)])
@pytest.mark.parametrize("signs", [(1.0, 1.0, 1.0), (-1.0, 1.0, -1.0), (-1.0, -1.0, -1.0)])
def test_v8_apply_bc_fn_bitwise_and_vs_oracle(shape, p, signs):
    """gdm_apply_bc_fn on a v8 mesh (stage boundary values computed by the
    engine, step 1 as tail work) == eval_boundary + apply, bitwise; and the
    explicit path against the oracle with the same boundary values in
    reference order."""
    import gdm_amd

    a = tuple(s * v for s, v in zip(signs, A_MAG))
    op = gdm_amd.GdmOperator(3, p, shape, 0.0, 1.0, "advection", params=a)
    m = O.Mesh(3, p, list(shape), 0.0, 1.0)
    sine = [1.0, 0.15, -0.05, 1.0, 1.0, 1.0, 0.3, 0.0, 0.7]
    u = _dev(np.random.default_rng(4).uniform(-1, 1, m.n_dofs))
    nb = op.n_bc_points
    t_g, alpha, t_k = 0.0125, 0.015, 0.0375
    g = torch.zeros(nb, dtype=torch.float64, device="cuda")
    k = torch.zeros_like(g)
    Y = torch.zeros_like(g)
    scratch = torch.zeros_like(g)
    op.eval_boundary(2, sine, t_g, 0, g)
    op.eval_boundary(2, sine, t_k, 1, k)
    op.rk_update(0.0, k, g, scratch, alpha, g, Y)
    ref = op.new_vector(local=False)
    op.apply(u, ref, Y)
    out = op.new_vector(local=False)
    op.apply_bc_fn(u, out, 2, sine, t_g, alpha, t_k)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), float((out - ref).abs().max())
    bc_ref = _host(Y)[op.bc_reference_order()]
    want = _volume_ref(m, a, _host(u)) + m.advection_inflow(a, bc_ref)
    assert _rel(_host(out), want) < 1e-12


def test_v8_tail_repeated_streams_and_graph_replay():
    """The tail's claim counter is per launch (no host-side claim
    base): many launches in a row, launches on alternating (ordered) streams,
    and a captured hipGraph replayed several times each give the bits of the
    first call."""
    import gdm_amd

    shape, p, a = (100, 70, 64), 5, (-0.8, 0.45, -0.3)
    op = gdm_amd.GdmOperator(3, p, shape, 0.0, 1.0, "advection", params=a)
    gen = torch.Generator(device="cuda").manual_seed(2)
    u = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen)
    bc = torch.rand(op.n_bc_points, dtype=torch.float64, device="cuda", generator=gen)
    ref = op.new_vector(local=False)
    op.apply(u, ref, bc)
    torch.cuda.synchronize()
    outs = [op.new_vector(local=False) for _ in range(6)]
    for y in outs:
        op.apply(u, y, bc)
    torch.cuda.synchronize()
    for y in outs:
        assert torch.equal(y, ref)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for i, y in enumerate(outs):
        y.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(streams[i % 2]):
            op.use_torch_stream()
            op.apply(u, y, bc)
        torch.cuda.synchronize()
    op.use_torch_stream()
    for y in outs:
        assert torch.equal(y, ref)
    # graph capture of the whole compute_rhs, replayed
    y = op.new_vector(local=False)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        op.use_torch_stream()
        op.apply(u, y, bc)  # warm-up on the capture stream
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            op.apply(u, y, bc)
    torch.cuda.synchronize()
    for _ in range(3):
        y.zero_()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, ref)
    op.use_torch_stream()


def test_c3_inflow_part_full_size():
    """BASELINE C3 (512^3 DoFs, p = 5) with the metric's inflow data: the
    inflow part y(u, bc) - y(u, 0) of the device's compute_rhs against the
    oracle's boundary-cell loop (1.6 M boundary cells, ~7 s of CPU)."""
    import gdm_amd

    a = (1.0, 0.15, -0.05)
    op = gdm_amd.GdmOperator(3, 5, 511, 0.0, 1.0, "advection", params=a)
    m = O.Mesh(3, 5, 511, 0.0, 1.0)
    nb = m.n_boundary_points()
    assert op.n_bc_points == nb
    rng = np.random.default_rng(11)
    bc_ref = rng.uniform(-1, 1, nb)
    bc_dev = np.empty(nb)
    bc_dev[op.bc_reference_order()] = bc_ref
    del bc_ref
    gen = torch.Generator(device="cuda").manual_seed(12)
    u = torch.rand(op.n_owned, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    y1, y0 = op.new_vector(local=False), op.new_vector(local=False)
    op.apply(u, y1, _dev(bc_dev))
    op.apply(u, y0)
    y1 -= y0
    del y0, u
    got = _host(y1)
    del y1
    bc_ref = np.empty(nb)
    bc_ref[:] = bc_dev[op.bc_reference_order()]
    want = m.advection_inflow(a, bc_ref)
    assert _rel(got, want) < 1e-11
