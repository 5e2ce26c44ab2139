"""The cut-cell wave / heat application on the device (gdm_amd.CutWave,
CutWaveProblem: include/gdm_hip.h "Cut-cell wave") against the reference's
own application goldens applications/wave/tests/{wave_0,heat_1,heat_0,
wave_composite_0,heat_composite_0}.output (wave-rk 111 steps, heat-rk 820
steps, heat-impl 6 steps, and the composite inside / outside pairs on the 1D
mesh cut by the FE_Q(3) sphere level set): every (L2, L1, Linf) of every step to the
2e-8 of tests/test_cut1d_golden.py, every time to the printed 5 decimals.
The host assembly is checked piece by piece in tests/test_cut_wave_host.py."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_outputs.json")))["wave_app"]["cases"]


@pytest.mark.parametrize("case,simulation", [("wave_0", "wave"), ("heat_1", "heat-rk"), ("heat_0", "heat-impl")])
def test_device_run_reproduces_golden(case, simulation):
    from gdm_amd.cut_wave import CutWaveProblem, preset

    prob = CutWaveProblem(preset(simulation))
    assert prob.cw.cells == dict(inside=32, intersected=2, outside=6)
    rows = prob.run()
    ref = REF[case]["steps"]
    assert len(rows) == len(ref)
    for got, exp in zip(rows, ref):
        assert got[0] == exp[0]
        assert abs(got[1] - exp[1]) <= 5.000001e-6
        np.testing.assert_allclose(got[2:], exp[2:], rtol=2e-8, atol=0)


def test_operators_are_consistent():
    """M^-1 (M u) == u through the device product and the banded solve;
    compute_rhs = its operator part + its data part"""
    from gdm_amd.cut_wave import CutWave, preset

    P = preset("heat-rk")
    cw = CutWave(P["p"], P["n"], P["left"], P["right"], P["level_set"], ghost_parameter_M=P["gamma_M"],
                 ghost_parameter_A=P["gamma_A"], nitsche=P["nitsche"])
    g = torch.Generator(device="cuda").manual_seed(3)
    u = torch.rand(cw.n_dofs, dtype=torch.float64, device="cuda", generator=g)
    Mu, x = cw.new_vector(), cw.new_vector()
    cw.mass_apply(u, Mu)
    cw.mass_solve(Mu, x)
    assert float(torch.linalg.norm(x - u) / torch.linalg.norm(u)) < 1e-12
    fq = torch.rand(max(cw.n_quad, 1), dtype=torch.float64, device="cuda", generator=g)
    gs = torch.rand(max(cw.n_surface, 1), dtype=torch.float64, device="cuda", generator=g)
    r_full, r_op, r_data = cw.new_vector(), cw.new_vector(), cw.new_vector()
    cw.compute_rhs(u, fq, gs, r_full)
    cw.compute_rhs(u, None, None, r_op)
    cw.compute_rhs(None, fq, gs, r_data)
    assert float(torch.linalg.norm(r_full - r_op - r_data) / torch.linalg.norm(r_full)) < 1e-14


@pytest.mark.parametrize("case,simulation", [("wave_composite_0", "wave-composite"),
                                             ("heat_composite_0", "heat-composite")])
def test_composite_run_reproduces_golden(case, simulation):
    """two device handles (inside / outside, domain Dirichlet data, interface
    coupling through gdm_cut_wave_couple) against the composite goldens"""
    from gdm_amd.cut_wave import CutWaveCompositeProblem, preset

    rows = CutWaveCompositeProblem(preset(simulation)).run()
    ref = REF[case]["steps"]
    assert len(rows) == len(ref)
    for got, exp in zip(rows, ref):
        assert got[0] == exp[0]
        assert abs(got[1] - exp[1]) <= 5.000001e-6
        np.testing.assert_allclose(got[2:], exp[2:], rtol=2e-8, atol=0)
