"""gdm_apply_bc_fn (include/gdm_hip.h): the RK stage boundary values
g(t_g) + alpha dg/dt(t_k) evaluated inside the face kernels give the same
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
