"""The 2D cut-cell advection restatement (oracle/cut_advection2d.py: the
reference's advection application -- compute_rhs terms (I) cell, (II) cut
surface, (III) box faces with upwind inflow data, (IV) ghost penalty; mass
with ghost penalty; RK4 + DiscreteTime; the six-norm postprocess) against
applications/advection/tests/test_01.output, the ConvergenceTable of
advection-convergence.cc's "parallel-ramp-degree" case (p = 3, 5; n = 40;
rotations 5..45 degrees; end_t 0.1): all 18 rows x 6 columns.

Tolerance: the printed digits (half a unit of the 5th significant digit)
plus 5e-13 absolute -- the reference's mass solves stop at a relative
residual of 1e-14 (SolverCG + ILU, problem.h:236-267), which leaves ~1e-13
in u; the oracle solves exactly, and a Jacobi-CG to the same tolerance moves
the p = 5 surface norms (~5e-8) by up to 4e-13.  103 of the 108 numbers
match with the printed-digit rule alone."""
import json
import os

import numpy as np
import pytest

import cut_advection2d as CA

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_outputs.json")))["advection_test_01"]


def _printed_ok(got, want, extra=5e-13):
    e = np.floor(np.log10(abs(want)))
    half_unit = 0.5 * 10.0 ** (e - 4)
    return abs(got - want) <= half_unit * (1 + 1e-9) + extra


@pytest.mark.parametrize("row", range(18))
def test_parallel_ramp_degree_row(row):
    ref = GOLD["rows"][row]
    p, cfl, n, rot0, rot1 = ref[:5]
    factor = int(round(rot0 / 5.0))
    got = CA.table_row(p, factor, n)
    assert got[:5] == (p, cfl, n, rot0, rot1)
    for c, (g, w) in enumerate(zip(got[5:], ref[5:])):
        assert _printed_ok(g, w), (GOLD["columns"][5 + c], g, w)


def test_boundary_points_and_operator_structure():
    """The stage boundary-value block has one entry per surface / inside box
    face point (stiffness.h:40-160); the cut surface is parallel to the
    transport direction (a . n = 0 up to round-off there), so only the box
    faces carry inflow data; outside DoFs have identity mass rows."""
    P = CA.CutAdvection2D(3, 40, 3)
    x, y = P.points[:, 0], P.points[:, 1]
    on_box = (np.abs(x) < 1e-14) | (np.abs(x - 1) < 1e-14) | (np.abs(y) < 1e-14) | (np.abs(y - 1) < 1e-14)
    Fa = abs(P.F).tocsc()
    colmax = np.array([Fa[:, c].max() if Fa[:, c].nnz else 0.0 for c in range(Fa.shape[1])])
    cols = np.flatnonzero(colmax > 1e-12)
    assert np.all(on_box[cols])
    # on the cut surface a.n is zero up to round-off (either sign: the upwind switch of (II) may pick u+ there)
    assert np.all(colmax[~on_box] < 1e-14)
    assert len(P.points) > len(cols)  # surface + outflow points carry no inflow data
    g = P.geo
    out = [i for i in range(P.N * P.N) if P.M[i, i] == 1.0 and P.K.getrow(i).nnz == 0]
    assert len(out) > 0
