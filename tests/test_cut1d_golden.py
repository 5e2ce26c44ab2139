"""The 1D cut-cell restatement of the reference's wave application
(oracle/cut1d.py) against the reference's own application goldens
applications/wave/tests/{wave_0,heat_0,heat_1,wave_composite_0,heat_composite_0}.output (parsed into
tests/golden/reference_outputs.json by tests/golden/make_golden.py).

These pin, for dim = 1 with the trivial 1D cut, the wave-rk loop
(problem.h:280-346: RK_CLASSIC_FOURTH_ORDER on (u, v), DiscreteTime, mass
solve per stage), heat-rk (:70-127) and heat-impl (:218-268), the mass matrix
with ghost penalty (wave/mass.h:47-249), compute_rhs with surface Nitsche and
ghost penalty (wave/stiffness.h:42-407), the assembled stiffness matrix
(:602-800), vertex interpolation and the error postprocess (:504-590).

Tolerance: the goldens print 9 significant digits; every (L2, L1, Linf) of
every step must agree to a relative 2e-8 and every time to the printed 5 decimals.
"""
import json
import os

import numpy as np
import pytest

import cut1d

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "reference_outputs.json")))["wave_app"]["cases"]


@pytest.mark.parametrize("case,simulation", [("wave_0", "wave"), ("heat_0", "heat-impl"), ("heat_1", "heat-rk")])
def test_wave_app_golden(case, simulation):
    ref = REF[case]
    assert ref["config"]["dim"] == 1
    rows = cut1d.run(simulation)
    assert len(rows) == len(ref["steps"])
    for got, exp in zip(rows, ref["steps"]):
        assert got[0] == exp[0]
        assert abs(got[1] - exp[1]) <= 5.000001e-6  # printed %8.5f
        np.testing.assert_allclose(got[2:], exp[2:], rtol=2e-8, atol=0)


@pytest.mark.parametrize("case,simulation", [("wave_composite_0", "wave-composite"),
                                             ("heat_composite_0", "heat-composite")])
def test_wave_app_composite_golden(case, simulation):
    """the composite presets: inside and outside fields with their own masses
    and ghost penalties, domain Dirichlet data on the boundary faces, the
    interface coupling of compute_rhs(BlockVector) (wave/stiffness.h:420-575);
    rows alternate inside / outside"""
    ref = REF[case]
    assert ref["config"]["dim"] == 1
    rows = cut1d.run_composite(simulation)
    assert len(rows) == len(ref["steps"])
    for got, exp in zip(rows, ref["steps"]):
        assert got[0] == exp[0]
        assert abs(got[1] - exp[1]) <= 5.000001e-6
        np.testing.assert_allclose(got[2:], exp[2:], rtol=2e-8, atol=0)


def test_discrete_time_last_step():
    """DiscreteTime: wave_0 takes 110 steps of 0.3 h and a shrunk 111th to
    t = 2; heat_0 5 steps and a shrunk 6th to t = 0.1 (the goldens' times)."""
    h = 2.42 / 40
    for end, n in ((2.0, 111), (0.1, 6)):
        t = cut1d.DiscreteTime(0.0, end, 0.3 * h)
        steps = 0
        while not t.is_at_end():
            t.advance()
            steps += 1
        assert steps == n and t.t == end


def test_cut_classification():
    """wave-app geometry: 40 cells on [-1.21, 1.21], sphere r = 1: cells 0-2
    and 37-39 outside, 3 and 36 cut at x = -1 / +1, the rest inside; one
    ghost-penalty face per cut, visited from both sides."""
    m = cut1d.Cut1D(3, 40, -1.21, 1.21, lambda x: abs(x) - 1.0)
    locs = [c["loc"] for c in m.cells]
    assert [i for i, l in enumerate(locs) if l == m.INTERSECTED] == [3, 36]
    assert all(locs[i] == m.OUTSIDE for i in (0, 1, 2, 37, 38, 39))
    assert all(locs[i] == m.INSIDE for i in range(4, 36))
    surf = [s for c in m.cells for s in c["surface"]]
    assert len(surf) == 2
    np.testing.assert_allclose([s[0] for s in surf], [-1.0, 1.0], atol=1e-14)
    assert [s[1] for s in surf] == [-1.0, 1.0]
    faces = sorted((min(c, nb), max(c, nb)) for c, nb, _ in m.gp_faces())
    assert faces == [(3, 4), (3, 4), (35, 36), (35, 36)]
