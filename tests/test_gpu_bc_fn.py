"""gdm_apply_bc_fn (include/gdm_hip.h): the RK stage boundary values
g(t_g) + alpha dg/dt(t_k) computed by the engine (gdm_apply_bc_fn) give the same
bits as the explicit block(0) path of the reference's RK stages
(advection/problem.h:62-94; gdm_eval_boundary + gdm_vec_rk_update +
gdm_apply with the stage vector), and AdvectionProblem's default step (no
block(0) vectors) the same state as carry_bc=True.  Bitwise: both paths run
the same device expressions in the same order.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SINE = [1.0, 0.15, -0.05, 1.0, 1.0, 1.0, 0.3, 0.0, 0.7]


def _explicit(op, u, fn, prm, t_g, alpha, t_k):
    nb = op.n_bc_points
    z = lambda: torch.zeros(max(nb, 1), dtype=torch.float64, device="cuda")  # noqa: E731
    g, k, Y, scratch = z(), z(), z(), z()
    op.eval_boundary(fn, prm, t_g, 0, g[:nb])
    if alpha != 0.0:
        op.eval_boundary(fn, prm, t_k, 1, k[:nb])
        op.rk_update(0.0, k[:nb], g[:nb], scratch[:nb], alpha, g[:nb], Y[:nb])
    else:
        Y = g
    out = op.new_vector(local=False)
    op.apply(u, out, Y[:nb])
    return out


@pytest.mark.parametrize("dim,p,n", [(2, 5, (13, 10)), (3, 5, 9), (3, 3, (7, 8, 6)), (3, 7, 17)])
@pytest.mark.parametrize("fn,prm", [(2, SINE), (1, [0.3, 0.2, 0.4, 0.5]), (0, [0.7])])
@pytest.mark.parametrize("alpha,t_k", [(0.0, 0.0), (0.015, 0.0375), (-0.02, 0.11)])
def test_apply_bc_fn_bitwise_equals_explicit(dim, p, n, fn, prm, alpha, t_k):
    import gdm_amd

    a = (1.0, 0.15, -0.05)[:dim]
    op = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "advection", params=a)
    assert op.n_bc_points > 0
    g = torch.Generator(device="cuda").manual_seed(7)
    u = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=g)
    t_g = 0.0125
    ref = _explicit(op, u, fn, prm, t_g, alpha, t_k)
    out = op.new_vector(local=False)
    op.apply_bc_fn(u, out, fn, prm, t_g, alpha, t_k)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), float((out - ref).abs().max())


@pytest.mark.parametrize("dim,p,n", [(2, 5, (13, 10)), (3, 5, 9)])
def test_advection_problem_fast_step_bitwise(dim, p, n):
    import gdm_amd

    a = (1.0, 0.15, -0.05)[:dim]
    ops = [gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "advection", params=a) for _ in range(2)]
    probs = [gdm_amd.AdvectionProblem(ops[0], 2, SINE, carry_bc=True), gdm_amd.AdvectionProblem(ops[1], 2, SINE)]
    g = torch.Generator(device="cuda").manual_seed(3)
    u0 = torch.rand(ops[0].n_owned, dtype=torch.float64, device="cuda", generator=g)
    h = 0.01
    for pr in probs:
        pr.u.copy_(u0)
        assert pr.run(0.0, 3 * h, h) == 3
    torch.cuda.synchronize()
    assert torch.equal(probs[0].u, probs[1].u), float((probs[0].u - probs[1].u).abs().max())


def test_apply_bc_fn_argument_errors():
    import gdm_amd

    op = gdm_amd.GdmOperator(2, 3, 6, 0.0, 1.0, "advection", params=(1.0, 0.5))
    u = op.new_vector(local=True)
    out = op.new_vector(local=False)
    with pytest.raises(gdm_amd.GdmError):
        op.apply_bc_fn(u, out, 5, [0.0], 0.0)
    with pytest.raises(gdm_amd.GdmError):
        op.apply_bc_fn(u, out, 2, [1.0, 2.0], 0.0)
    wave = gdm_amd.GdmOperator(2, 3, 6, -1.0, 1.0, "wave")
    with pytest.raises(gdm_amd.GdmError):
        wave.apply_bc_fn(wave.new_vector(local=True), wave.new_vector(local=False), 0, [1.0], 0.0)


@pytest.mark.parametrize("dim,p,n", [(3, 5, 181), (3, 7, 183), (3, 3, 200), (2, 5, (300, 200)), (3, 5, 9)])
@pytest.mark.parametrize("mode", ["Y", "noY", "alias"])
def test_mass_solve_rk_bitwise_equals_separate(dim, p, n, mode):
    """gdm_mass_solve_rk (the RK update fused into the x line-solve pass when
    that pass runs unsegmented, 3D meshes with >= 32768 lines per pass; the
    separate kernels otherwise) == gdm_mass_solve + gdm_vec_rk_update, bitwise"""
    import gdm_amd

    op = gdm_amd.GdmOperator(dim, p, n, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05)[:dim])
    m = op.n_owned
    g = torch.Generator(device="cuda").manual_seed(11)
    r = lambda: torch.rand(m, dtype=torch.float64, device="cuda", generator=g) - 0.5  # noqa: E731
    rhs, acc, y = r(), r(), r()
    beta, alpha = 0.0123456789, -0.0234567891
    # reference: separate solve + update
    k = rhs.clone()
    op.mass_solve(k, k)
    acc_ref, Y_ref = acc.clone(), torch.empty_like(y)
    if mode == "Y":
        op.rk_update(beta, k, acc, acc_ref, alpha, y, Y_ref)
    elif mode == "noY":
        op.rk_update(beta, k, acc, acc_ref)
    else:
        op.rk_update(beta, k, acc_ref, acc_ref, alpha, y, Y_ref)
    acc_out, Y = acc.clone(), torch.empty_like(y)
    rhs2 = rhs.clone()
    if mode == "Y":
        op.mass_solve_rk(rhs2, beta, acc, acc_out, alpha, y, Y)
    elif mode == "noY":
        op.mass_solve_rk(rhs2, beta, acc, acc_out)
    else:
        op.mass_solve_rk(rhs2, beta, acc_out, acc_out, alpha, y, Y)
    torch.cuda.synchronize()
    assert torch.equal(acc_out, acc_ref), float((acc_out - acc_ref).abs().max())
    if mode != "noY":
        assert torch.equal(Y, Y_ref), float((Y - Y_ref).abs().max())


@pytest.mark.parametrize("dim,p,n", [(3, 5, 181), (2, 5, (13, 10))])
def test_wave_problem_fused_step_vs_oracle_form(dim, p, n):
    """WaveProblem (v block through gdm_mass_solve_rk) == the same stages with
    mass_solve + rk_update, bitwise"""
    import gdm_amd
    from gdm_amd.problem import RK4_A, RK4_B

    op = gdm_amd.GdmOperator(dim, p, n, -1.21, 1.21, "wave")
    g = torch.Generator(device="cuda").manual_seed(5)
    u0 = torch.rand(op.n_owned, dtype=torch.float64, device="cuda", generator=g)
    pr = gdm_amd.WaveProblem(op)
    pr.u.copy_(u0)
    h = 1e-3
    pr.step(0.0, h)
    # unfused restatement of one step
    y = (u0.clone(), torch.zeros_like(u0))
    acc = [torch.empty_like(u0) for _ in range(2)]
    Y = [torch.empty_like(u0) for _ in range(2)]
    kv = torch.empty_like(u0)
    stage = y
    for s in range(4):
        op.apply(stage[0], kv)
        op.mass_solve(kv, kv)
        last = s == 3
        ai, ao = (y if s == 0 else acc), (y if last else acc)
        a_next = 0.0 if last else h * RK4_A[s]
        op.rk_update(h * RK4_B[s], stage[1], ai[0], ao[0], a_next, None if last else y[0], None if last else Y[0])
        op.rk_update(h * RK4_B[s], kv, ai[1], ao[1], a_next, None if last else y[1], None if last else Y[1])
        stage = Y
    torch.cuda.synchronize()
    assert torch.equal(pr.u, y[0]) and torch.equal(pr.v, y[1])
