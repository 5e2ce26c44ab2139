"""Host logic of the device RK drivers (gdm_amd/problem.py), no GPU: a
recording stand-in for GdmOperator checks the stage sequence that
AdvectionProblem / WaveProblem issue against classic RK4 (deal.II
RK_CLASSIC_FOURTH_ORDER, advection/problem.h:62-94): the stage boundary values
g(t_n) + h a_{s,s-1} dg/dt(t_n + c_{s-1} h), the fused solve + update
arguments, and that the explicit block(0) path (carry_bc=True) is still
selectable.  The numerics of these calls are covered on the GPU
(tests/test_gpu_bc_fn.py, tests/test_gpu_rk.py)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

from gdm_amd.problem import RK4_A, RK4_B, RK4_C, AdvectionProblem, WaveProblem  # noqa: E402


class _Vec:
    def __init__(self, name):
        self.name = name

    def copy_(self, other):
        return self

    def __repr__(self):
        return self.name


class _Mesh:
    n_ranks = 1


class _Op:
    """records the engine calls"""

    FN_SINE_PRODUCT = 2

    def __init__(self, n_bc=5):
        self.mesh = _Mesh()
        self.n_bc_points = n_bc
        self.n_owned = 7
        self.device = 0
        self.calls = []
        self._n = 0

    def new_vector(self, local=False):
        self._n += 1
        return _Vec("v%d" % self._n)

    def __getattr__(self, name):
        if name.startswith("_") or name in ("calls",):
            raise AttributeError(name)

        def rec(*args, **kw):
            self.calls.append((name, args, kw))
            return args[1] if len(args) > 1 else None

        return rec


@pytest.fixture()
def no_torch(monkeypatch):
    import types

    fake = types.SimpleNamespace(zeros=lambda m, dtype=None, device=None: _Vec("z%d" % m), float64=None)
    monkeypatch.setitem(sys.modules, "torch", fake)


def test_advection_stage_boundary_arguments(no_torch):
    op = _Op()
    prm = [1.0, 0.15, -0.05, 1, 1, 1, 0.3, 0, 0.7]
    pr = AdvectionProblem(op, 2, prm)
    t, h = 0.25, 0.01
    pr.step(t, h)
    applies = [c for c in op.calls if c[0] == "apply_bc_fn"]
    solves = [c for c in op.calls if c[0] == "mass_solve_rk"]
    assert [c[0] for c in op.calls] == ["apply_bc_fn", "mass_solve_rk"] * 4
    for s, (_, args, _) in enumerate(applies):
        _, _, fn, params, t_g, alpha, t_k = args
        assert fn == 2 and params == prm and t_g == t
        if s == 0:
            assert alpha == 0.0
        else:
            assert alpha == h * RK4_A[s - 1] and t_k == t + RK4_C[s - 1] * h
    y = pr.u
    acc = pr._acc[1]
    for s, (_, args, _) in enumerate(solves):
        k, beta, acc_in, acc_out, alpha, yv, Y = args
        last = s == 3
        assert beta == h * RK4_B[s]
        assert acc_in is (y if s == 0 else acc) and acc_out is (y if last else acc)
        assert alpha == (0.0 if last else h * RK4_A[s])
        assert (yv is None and Y is None) if last else (yv is y and Y is pr._Y[1])
    # each stage's input is the previous stage's Y
    assert applies[0][1][0] is y and all(a[1][0] is pr._Y[1] for a in applies[1:])


def test_advection_carry_bc_path_kept(no_torch):
    op = _Op()
    pr = AdvectionProblem(op, 2, [0.0] * 9, carry_bc=True)
    pr.step(0.0, 0.1)
    names = [c[0] for c in op.calls]
    assert names.count("eval_boundary") == 1 + 4 and "apply_bc_fn" not in names
    assert names.count("rk_update") == 8 and names.count("mass_solve") == 4


def test_wave_stage_order(no_torch):
    op = _Op(n_bc=0)
    pr = WaveProblem(op)
    pr.step(0.0, 0.1)
    names = [c[0] for c in op.calls]
    # apply (reads stage u), u-block update (reads stage v), fused v-block solve + update
    assert names == ["apply", "rk_update", "mass_solve_rk"] * 4
    for s in range(4):
        _, (src, kv), _ = op.calls[3 * s]
        assert src is (pr.u if s == 0 else pr._Y[0])
        _, args, _ = op.calls[3 * s + 1]
        assert args[1] is (pr.v if s == 0 else pr._Y[1])  # ku = stage v, before it is overwritten


def test_advection_no_block0_vectors_without_carry_bc(no_torch):
    """with the engine computing the stage boundary values, no
    block(0) vector is allocated (28 M points at C3) and .bc refuses"""
    from gdm_amd._capi import GdmError

    pr = AdvectionProblem(_Op(), 2, [0.0] * 9)
    assert pr._acc[0] is None and pr._Y[0] is None and pr._k[0] is None
    with pytest.raises(GdmError):
        pr.bc
    pr2 = AdvectionProblem(_Op(), 2, [0.0] * 9, carry_bc=True)
    assert pr2.bc is not None and pr2._acc[0] is not None


def test_advection_initialize_time_step_without_carry_bc(no_torch):
    """the public initialize_time_step() stays callable on the
    default (engine-computed boundary values) path -- a no-op there -- and
    fills block(0) on the explicit path"""
    op = _Op()
    pr = AdvectionProblem(op, 2, [0.0] * 9)
    assert pr.initialize_time_step(0.5) is False
    assert op.calls == []
    op2 = _Op()
    pr2 = AdvectionProblem(op2, 2, [0.0] * 9, carry_bc=True)
    assert pr2.initialize_time_step(0.5) is True
    assert [c[0] for c in op2.calls] == ["eval_boundary"] and op2.calls[0][1][2] == 0.5
