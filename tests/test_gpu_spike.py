"""Distributed exact mass inverse on the device (gdm_mass_solve_slab +
ghost exchange + gdm_mass_solve_interface, include/gdm_hip.h), all ranks of
the partition as operators in one process, the exchange done by copying the
neighbours' edge planes (what HaloExchange / MPI do between processes).

Reference: the one-rank exact Kronecker inverse gdm_mass_solve, itself pinned
to CG(1e-14) on the oracle's assembled mass matrix (test_gpu_parity.py) --
the reference's *Problem::solve (advection/problem.h:236-267).
Thin slabs (C4 at 8 ranks: 32 planes at p = 7, far-spike coupling 2e-8) run
the refinement rounds of gdm_mass_spike_rounds (gdm_mass_solve_interface_round
+ one more exchange each).
Tolerance: rel-L2 <= 1e-13 (the remaining interface coupling is < 1e-15)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _ranks(gdm_amd, dim, p, n, R):
    ops = [gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass", n_ranks=R, rank=r) for r in range(R)]
    return ops


def _exchange(ops, xs):
    """fill ghost planes of every local vector from the neighbours' owned planes"""
    for r, op in enumerate(ops):
        L, ps = op.layout, op.layout["plane_size"]
        gb, ga = L["ghost_planes_below"], L["ghost_planes_above"]
        own = L["n_owned"] // ps
        if r > 0 and gb:
            Ln = ops[r - 1].layout
            e = (Ln["ghost_planes_below"] + Ln["n_owned"] // ps) * ps
            xs[r][:gb * ps] = xs[r - 1][e - gb * ps:e]
        if r + 1 < len(ops) and ga:
            Ln = ops[r + 1].layout
            b = Ln["ghost_planes_below"] * ps
            xs[r][(gb + own) * ps:(gb + own + ga) * ps] = xs[r + 1][b:b + ga * ps]


@pytest.mark.parametrize("dim,p,n,R", [(3, 5, (12, 10, 130), 2), (3, 5, (9, 8, 200), 3), (2, 3, (20, 150), 3),
                                       (1, 5, 400, 4), (3, 7, (8, 9, 240), 2), (2, 9, (12, 260), 2),
                                       (3, 1, (6, 5, 120), 4), (3, 7, (8, 9, 255), 8), (2, 5, (30, 150), 6),
                                       (3, 7, (255, 255, 255), 8)])
def test_slab_mass_solve_matches_single_rank(dim, p, n, R):
    import gdm_amd

    rounds = gdm_amd._capi.mass_spike_rounds(dim, p, n, R)
    assert rounds >= 0
    if (p, R) == (7, 8):  # the C4 partition: one refinement round
        assert rounds == 1
    one = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass")
    N = one.n_owned
    r = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, N)).cuda()
    ref = one.new_vector(False)
    one.mass_solve(r, ref)
    ops = _ranks(gdm_amd, dim, p, n, R)
    xs = []
    for op in ops:
        L = op.layout
        a = L["owned_plane_begin"] * L["plane_size"]
        x = op.new_vector(True)
        op.mass_solve_slab(r[a:a + op.n_owned].contiguous(), op.owned_view(x))
        xs.append(x)
    torch.cuda.synchronize()
    _exchange(ops, xs)
    for k in range(rounds):
        for op, x in zip(ops, xs):
            op.mass_solve_interface_round(x, k)
        torch.cuda.synchronize()
        _exchange(ops, xs)
    for op, x in zip(ops, xs):
        op.mass_solve_interface(x)
    got = torch.cat([op.owned_view(x) for op, x in zip(ops, xs)])
    assert float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref)) < 1e-13


def test_slab_mass_solve_refuses_slabs_thinner_than_2p():
    """8 ranks of p = 7 on 100 cells (12-13 planes < 2p): refused instead of
    an approximate inverse."""
    import gdm_amd

    assert gdm_amd._capi.mass_spike_rounds(3, 7, (8, 8, 100), 8) == -1
    op = gdm_amd.GdmOperator(3, 7, (8, 8, 100), 0.0, 1.0, "mass", n_ranks=8, rank=3)
    x = op.new_vector(False)
    with pytest.raises(gdm_amd.GdmError, match="too thin"):
        op.mass_solve_slab(x, x)


def test_interface_refuses_skipped_or_out_of_order_rounds():
    """The C4 partition needs one refinement round: an interface call without
    it, a round before the slab solve, a round out of order and a second
    interface call after one solve are refused (GDM_ERR_STATE) instead of a
    silently wrong inverse from stale saved edge planes."""
    import gdm_amd

    n, R = (8, 9, 255), 8
    assert gdm_amd._capi.mass_spike_rounds(3, 7, n, R) == 1
    op = gdm_amd.GdmOperator(3, 7, n, 0.0, 1.0, "mass", n_ranks=R, rank=3)
    x = op.new_vector(True)
    r = torch.ones(op.n_owned, dtype=torch.float64, device="cuda")
    with pytest.raises(gdm_amd.GdmError, match="gdm_mass_solve_slab first"):
        op.mass_solve_interface_round(x, 0)
    op.mass_solve_slab(r, op.owned_view(x))
    with pytest.raises(gdm_amd.GdmError, match="0 of 1 refinement rounds"):
        op.mass_solve_interface(x)
    op.mass_solve_interface_round(x, 0)
    with pytest.raises(gdm_amd.GdmError, match="in order"):
        op.mass_solve_interface_round(x, 0)
    op.mass_solve_interface(x)
    with pytest.raises(gdm_amd.GdmError, match="gdm_mass_solve_slab first"):
        op.mass_solve_interface(x)
    # SlabMassSolve without an explicit count asks the C ABI for it
    from gdm_amd.distributed import SlabMassSolve

    assert SlabMassSolve(op, None).rounds == 1


@pytest.mark.parametrize("dim,p,n,R", [(3, 5, (12, 10, 130), 2), (2, 3, (20, 150), 3), (1, 5, 400, 4),
                                       (3, 7, (8, 9, 255), 8)])
def test_interface_ghosts_give_the_neighbours_planes(dim, p, n, R):
    """gdm_mass_solve_interface_ghosts (ABI 14): the owned part is bitwise
    gdm_mass_solve_interface's, and the ghost planes hold the neighbours'
    owned edge planes of M^-1 rhs (the interface solution both ranks of a
    pair compute) to 1e-13 of the vector's max -- what the one-exchange RK
    stage relies on (C4 at 8 ranks: after its refinement round)."""
    import gdm_amd

    rounds = gdm_amd._capi.mass_spike_rounds(dim, p, n, R)
    one = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass")
    r = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, one.n_owned)).cuda()
    del one
    ops = _ranks(gdm_amd, dim, p, n, R)
    out = {}
    for ghosts in (False, True):
        xs = []
        for op in ops:
            a = op.layout["owned_plane_begin"] * op.layout["plane_size"]
            x = op.new_vector(True)
            op.mass_solve_slab(r[a:a + op.n_owned].contiguous(), op.owned_view(x))
            xs.append(x)
        torch.cuda.synchronize()
        _exchange(ops, xs)
        for k in range(rounds):
            for op, x in zip(ops, xs):
                op.mass_solve_interface_round(x, k)
            torch.cuda.synchronize()
            _exchange(ops, xs)
        for op, x in zip(ops, xs):
            (op.mass_solve_interface_ghosts if ghosts else op.mass_solve_interface)(x)
        torch.cuda.synchronize()
        out[ghosts] = xs
    scale = max(float(x.abs().max()) for x in out[False])
    for r_, op in enumerate(ops):
        assert torch.equal(op.owned_view(out[True][r_]), op.owned_view(out[False][r_]))
    # ghost planes == the neighbours' owned values
    ref = [x.clone() for x in out[True]]
    _exchange(ops, ref)
    for x, y in zip(out[True], ref):
        assert float((x - y).abs().max()) <= 1e-13 * scale


@pytest.mark.parametrize("dim,p,n,R", [(3, 5, (12, 10, 130), 2), (2, 3, (20, 150), 3), (1, 5, 400, 4),
                                       (3, 7, (8, 9, 255), 8), (3, 5, (33, 17, 200), 5)])
def test_interface_rk_is_interface_ghosts_plus_update_bitwise(dim, p, n, R):
    """gdm_mass_solve_interface_rk (ABI 15): the interface correction fused
    with the stage update -- every local plane of acc_out / Y, ghost planes
    included, has the bits of mass_solve_interface_ghosts + rk_update over
    n_local, for the three argument patterns of the low-storage RK4 stages
    (acc_in == y at stage 0, acc_in == acc_out in between, no Y at the last),
    with and without refinement rounds (C4 at 8 ranks: one round)."""
    import gdm_amd

    rounds = gdm_amd._capi.mass_spike_rounds(dim, p, n, R)
    assert rounds >= 0
    one = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "mass")
    r = torch.from_numpy(np.random.default_rng(9).uniform(-1, 1, one.n_owned)).cuda()
    del one
    ops = _ranks(gdm_amd, dim, p, n, R)
    gen = torch.Generator(device="cuda").manual_seed(4)

    def solved():
        xs = []
        for op in ops:
            a = op.layout["owned_plane_begin"] * op.layout["plane_size"]
            x = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen)  # ghosts: stale data
            op.mass_solve_slab(r[a:a + op.n_owned].contiguous(), op.owned_view(x))
            xs.append(x)
        torch.cuda.synchronize()
        _exchange(ops, xs)
        for k in range(rounds):
            for op, x in zip(ops, xs):
                op.mass_solve_interface_round(x, k)
            torch.cuda.synchronize()
            _exchange(ops, xs)
        return xs

    beta, alpha = 0.37, -1.25
    for pattern in ("stage0", "middle", "last"):
        ks = [op.mass_solve_interface_ghosts(x) for op, x in zip(ops, solved())]
        xs_copy = solved()  # a second solve for the fused call (same bits)
        for op, k, xc in zip(ops, ks, xs_copy):
            y = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen)
            acc = torch.rand_like(y)
            want_acc, want_Y = torch.empty_like(y), torch.empty_like(y)
            got_acc, got_Y = torch.empty_like(y), torch.empty_like(y)
            if pattern == "stage0":
                op.rk_update(beta, k, y, want_acc, alpha, y, want_Y)
                op.mass_solve_interface_rk(xc, beta, y, got_acc, alpha, y, got_Y)
            elif pattern == "middle":
                want_acc.copy_(acc)
                got_acc.copy_(acc)
                op.rk_update(beta, k, want_acc, want_acc, alpha, y, want_Y)
                op.mass_solve_interface_rk(xc, beta, got_acc, got_acc, alpha, y, got_Y)
            else:
                op.rk_update(beta, k, acc, want_acc)
                op.mass_solve_interface_rk(xc, beta, acc, got_acc)
            torch.cuda.synchronize()
            assert torch.equal(got_acc, want_acc), (pattern, float((got_acc - want_acc).abs().max()))
            if pattern != "last":
                assert torch.equal(got_Y, want_Y), pattern
        # the fused call consumes the solve like the interface call
        v0 = ops[0].new_vector(True)
        with pytest.raises(gdm_amd.GdmError, match="gdm_mass_solve_slab first"):
            ops[0].mass_solve_interface_rk(xs_copy[0], beta, v0, v0.clone())


def test_interface_rk_refusals():
    """x_local overlapping an output, a partial overlap of acc_out and
    acc_in, and a single-rank operator are refused."""
    import gdm_amd

    n, R = (12, 10, 130), 2
    op = gdm_amd.GdmOperator(3, 5, n, 0.0, 1.0, "mass", n_ranks=R, rank=1)
    x = op.new_vector(True)
    op.mass_solve_slab(torch.ones(op.n_owned, dtype=torch.float64, device="cuda"), op.owned_view(x))
    acc = op.new_vector(True)
    with pytest.raises(gdm_amd.GdmError, match="must not overlap"):
        op.mass_solve_interface_rk(x, 1.0, acc, x)
    big = torch.zeros(op.n_local + 8, dtype=torch.float64, device="cuda")
    with pytest.raises(gdm_amd.GdmError, match="must not overlap"):
        op.mass_solve_interface_rk(x, 1.0, big[:op.n_local], big[8:])
    single = gdm_amd.GdmOperator(3, 5, n, 0.0, 1.0, "mass")
    v = single.new_vector(True)
    with pytest.raises(gdm_amd.GdmError, match="multi-rank only"):
        single.mass_solve_interface_rk(v, 1.0, v.clone(), v.clone())


@pytest.mark.parametrize("dim,p,n,R,kind", [(3, 5, (70, 40, 130), 3, "advection"), (2, 5, (90, 150), 4, "advection"),
                                            (3, 7, (40, 33, 255), 8, "advection")])
def test_one_exchange_rk_step_matches_two_exchange(dim, p, n, R, kind):
    """SlabRK4 (gdm_amd.distributed): RK4 steps with one exchange per stage
    (the stage's ghost planes from the SPIKE interface solution) == the
    reference's two exchanges per stage (stiffness.h:343 + the solve's) to
    1e-13, with the engine's inflow data (gdm_apply_bc_fn) -- and the
    two-exchange path == the single-rank AdvectionProblem step to 1e-12."""
    import gdm_amd
    from gdm_amd.distributed import SlabRK4

    a = (1.0, 0.15, -0.05)[:dim]
    sine = [1.0, 0.15, -0.05, 1.0, 1.0, 1.0, 0.3, 0.0, 0.7]
    one = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, kind, params=a)
    gen = torch.Generator(device="cuda").manual_seed(17)
    u0 = torch.rand(one.n_owned, dtype=torch.float64, device="cuda", generator=gen) - 0.5
    h, steps = 2e-3, 3
    pr = gdm_amd.AdvectionProblem(one, 2, sine)
    pr.u.copy_(u0)
    for s in range(steps):
        pr.step(s * h, h)
    torch.cuda.synchronize()
    single = pr.u.clone()
    del pr, one
    ops = [gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, kind, params=a, rank=r, n_ranks=R) for r in range(R)]
    ps = ops[0].layout["plane_size"]
    res, local = {}, {}
    for one_ex, fused in ((False, False), (True, False), (True, True)):
        rk = SlabRK4(ops, lambda vs: (torch.cuda.synchronize(), _exchange(ops, vs)), 2, sine, one_exchange=one_ex,
                     fused=fused)
        rk.set_solution([u0[op.layout["owned_plane_begin"] * ps:op.layout["owned_plane_end"] * ps] for op in ops])
        for s in range(steps):
            rk.step(s * h, h)
        torch.cuda.synchronize()
        res[one_ex, fused] = torch.cat([op.owned_view(y) for op, y in zip(ops, rk.y)])
        local[one_ex, fused] = [y.clone() for y in rk.y]
    # the fused interface + update launch (gdm_mass_solve_interface_rk) gives
    # the bits of interface_ghosts + rk_update, ghost planes included
    for a_, b_ in zip(local[True, True], local[True, False]):
        assert torch.equal(a_, b_)
    res[True] = res[True, True]
    res[False] = res[False, False]
    assert float(torch.linalg.norm(res[True] - res[False]) / torch.linalg.norm(res[False])) < 1e-13
    assert float(torch.linalg.norm(res[False] - single) / torch.linalg.norm(single)) < 1e-12
