"""Host assembly of the device cut-cell wave operators at dim = 2
(csrc/gdm_cut_wave.cpp assemble2d + gdm_cut.cpp saye_poly: the matrices
gdm_cut_wave_create uploads) against the 2D restatement
oracle/cut_wave2d.py, on the CPU.

The device evaluates compute_rhs = [impl] (Z S u + C u) + Ff f(x_q) + Fg g(x_s)
with S = -(grad v, grad u) of the uncut box (the 2D wave stencil; here the
oracle's Kronecker form -(L x M + M x L)), Z zeroing the rows of DoFs in the
boxes of cut / outside cells.  Checked: classification, the quadrature (points,
weights, normals), M, K, the compute_rhs operator and data parts against the
oracle to 1e-12 relative (the two bisect the roots to within a few ulps of
each other; the Nitsche terms carry gamma_D / h = 248), and the device formulation of the wave-rk and
poisson runs against applications/wave/tests/{wave_1,step85_0}.output with the
tolerances of tests/test_cut_wave2d_golden.py."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import cut1d  # noqa: E402
import cut_wave2d as W  # noqa: E402
import oracle as O  # noqa: E402
from test_cut_wave2d_golden import WAVE_1_RTOL, _check_wave_1  # noqa: E402
from test_cut_wave_host import _arr, _lib  # noqa: E402

REF = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_outputs.json")))["wave_app"]["cases"]


def host_system2d(prm, location=-1, flags=1, n=None):
    """the device operator's host arrays (scipy CSR) for a 2D preset (the
    field of `location`, Nitsche data / coupling `flags`, n cells per
    direction if given)"""
    import gdm_amd.cut_wave as CW

    L = _lib()
    L.gdmh_cut_wave_splits.argtypes = [ctypes.c_void_p]
    p, left, right = prm["p"], prm["left"], prm["right"]
    n = prm["n"] if n is None else n
    h = (right - left) / n
    gl = CW.gauss_lobatto(p + 1)
    x = (left + np.arange(n) * h)[:, None] + gl[None, :] * h
    X = np.broadcast_to(x[None, :, None, :], (n, n, p + 1, p + 1))
    Y = np.broadcast_to(x[:, None, :, None], X.shape)
    ls = np.ascontiguousarray(np.hypot(X, Y).reshape(-1) - 1.0)
    S = ctypes.c_void_p()
    err = ctypes.create_string_buffer(256)
    assert L.gdmh_cut_wave_create(2, p, n, left, right, p, ls.ctypes.data, location, flags, prm["gamma_M"], prm["gamma_A"],
                                  prm["nitsche"], ctypes.byref(S), err, 256) == 0, err.value
    try:
        nd, nq, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        cells = (ctypes.c_int64 * 3)()
        L.gdmh_cut_wave_info(S, ctypes.byref(nd), ctypes.byref(nq), ctypes.byref(ns), cells)
        N, NQ, NS = nd.value, nq.value, ns.value
        shape = {0: (N, N), 1: (N, NQ), 2: (N, NS), 3: (NQ, N), 4: (N, N), 5: (N, N), 6: (N, N)}
        out = dict(splits=L.gdmh_cut_wave_splits(S), cells=tuple(cells))
        for w, name in enumerate(("C", "Ff", "Fg", "E", "M", "K", "X")):
            q = [ctypes.c_void_p() for _ in range(3)]
            L.gdmh_cut_wave_csr(S, w, *[ctypes.byref(v) for v in q])
            rows, cols = shape[w]
            rp = _arr(q[0], rows + 1, ctypes.c_int64)
            ci = _arr(q[1], rp[-1], ctypes.c_uint32).astype(np.int64)
            v = _arr(q[2], rp[-1], ctypes.c_double)
            out[name] = sp.csr_matrix((v, ci, rp), shape=(rows, cols))
        q = [ctypes.c_void_p() for _ in range(5)]
        nz = ctypes.c_int64()
        L.gdmh_cut_wave_points(S, *[ctypes.byref(v) for v in q], ctypes.byref(nz))
        out["qx"] = _arr(q[0], 2 * NQ, ctypes.c_double).reshape(-1, 2)
        out["qw"] = _arr(q[1], NQ, ctypes.c_double)
        out["sx"] = _arr(q[2], 2 * NS, ctypes.c_double).reshape(-1, 2)
        out["sn"] = _arr(q[3], 2 * NS, ctypes.c_double).reshape(-1, 2)
        out["zero"] = _arr(q[4], nz.value, ctypes.c_int64)
    finally:
        L.gdmh_cut_wave_destroy(S)
    m = O.Mesh(2, p, n, left, right)
    terms = [(-m.matrices_1d(0)[2], m.matrices_1d(1)[0]), (m.matrices_1d(0)[0], -m.matrices_1d(1)[2])]
    Z = np.ones(N)
    Z[out["zero"]] = 0.0
    out["apply"] = lambda u: Z * m.kron_apply(terms, u) + out["C"] @ u  # the device compute_rhs operator
    return out


@pytest.fixture(scope="module")
def wave_case():
    prm = W.wave_params()
    model = W.CutWave2D(prm["p"], prm["n"], prm["left"], prm["right"])
    return prm, model, model.matrices(prm["gamma_M"], prm["gamma_A"], prm["nitsche"]), host_system2d(prm)


def test_classification_and_quadrature(wave_case):
    _, m, ops, H = wave_case
    assert H["splits"] == 0
    assert H["cells"] == tuple(int((m.loc == c).sum()) for c in (W.INSIDE, W.INTERSECTED, W.OUTSIDE))
    # same points in the same order (cells lexicographic, generator order)
    np.testing.assert_allclose(H["qx"], ops["q"][:, :2], rtol=0, atol=1e-13)
    np.testing.assert_allclose(H["qw"], ops["q"][:, 2], rtol=1e-12, atol=1e-12 * ops["q"][:, 2].max())
    np.testing.assert_allclose(H["sx"], ops["s"][:, :2], rtol=0, atol=1e-13)
    np.testing.assert_allclose(H["sn"], ops["s"][:, 2:], rtol=0, atol=1e-12)


def test_matrices_and_rhs_match_oracle(wave_case):
    prm, m, ops, H = wave_case
    for name in ("M", "K", "Ff", "Fg", "E"):
        D = (H[name] - ops[name]).toarray()
        assert abs(D).max() <= 1e-12 * abs(ops[name]).max(), name
    rng = np.random.default_rng(3)
    for _ in range(3):
        u = rng.uniform(-1, 1, m.N * m.N)
        ref = -(ops["A"] @ u)
        assert np.abs(H["apply"](u) - ref).max() <= 1e-12 * np.abs(ref).max()


def test_device_formulation_wave_1(wave_case):
    """wave-rk with the device operators (compute_rhs = Z S u + C u + Fg g,
    exact mass solve, E postprocess) against wave_1.output"""
    prm, m, ops, H = wave_case
    lu = spla.splu(H["M"].tocsc())
    N = m.N * m.N
    g = prm["g"]
    q, s = H["qx"], H["sx"]

    def post(u, t):
        e = H["E"] @ u - prm["exact"](q[:, 0], q[:, 1], t)
        return np.sqrt(np.sum(e * e * H["qw"])), np.sum(np.abs(e) * H["qw"]), np.max(np.abs(e))

    def f(t, y):
        return np.concatenate([y[N:], lu.solve(H["apply"](y[:N]) + H["Fg"] @ g(s[:, 0], s[:, 1], t))])

    u = m.interpolate(prm["exact"], 0.0)
    y = np.concatenate([u, np.zeros(N)])
    time = cut1d.DiscreteTime(0.0, prm["end_t"], prm["cfl"] * m.h)
    rows, n = [(0, 0.0) + post(u, 0.0)], 0
    while not time.is_at_end():
        t0, dt = time.t, time.next_step_size()
        y = cut1d.rk4_step(f, t0, dt, y)
        n += 1
        rows.append((n, t0 + dt) + post(y[:N], t0 + dt))
        time.advance()
    _check_wave_1(rows, WAVE_1_RTOL)


def test_device_formulation_step85():
    prm = W.step85_params()
    H = host_system2d(prm)
    q, s = H["qx"], H["sx"]
    rhs = H["Ff"] @ prm["f"](q[:, 0], q[:, 1], 0.0) + H["Fg"] @ prm["g"](s[:, 0], s[:, 1], 0.0)
    u = spla.spsolve(H["K"].tocsc(), rhs)
    e = H["E"] @ u - prm["exact"](q[:, 0], q[:, 1], 0.0)
    got = (np.sqrt(np.sum(e * e * H["qw"])), np.sum(np.abs(e) * H["qw"]), np.max(np.abs(e)))
    np.testing.assert_allclose(got, REF["step85_0"]["steps"][0][2:], rtol=0, atol=2e-12)


@pytest.fixture(scope="module")
def composite_case():
    """the two fields of the 2D composite presets at n = 20 (the oracle's
    cell loops in seconds): inside and outside, domain data + coupling"""
    prm = W.composite_params("wave-composite")
    m = W.CutWave2D(prm["p"], 20, prm["left"], prm["right"])
    ops = [m.matrices(prm["gamma_M"], prm["gamma_A"], prm["nitsche"], location=loc, interface_data=False,
                      domain_data=True, coupled=True) for loc in (W.INSIDE, W.OUTSIDE)]
    return prm, m, ops, [host_system2d(prm, loc, 2 | 4, n=20) for loc in (-1, 1)]


def test_composite_fields_match_oracle(composite_case):
    """both fields of heat-composite / wave-composite at dim 2 (parity
    unpinned: the reference holds no 2D composite output): the region
    quadrature, the domain-face data points, M, Ff, Fg, E, the own operator
    (Z S + C) and the partner coupling X against oracle/cut_wave2d.py"""
    prm, m, ops, H = composite_case
    rng = np.random.default_rng(7)
    for o, h in zip(ops, H):
        np.testing.assert_allclose(h["qx"], o["q"][:, :2], rtol=0, atol=1e-13)
        np.testing.assert_allclose(h["qw"], o["q"][:, 2], rtol=1e-12, atol=1e-12 * o["q"][:, 2].max())
        np.testing.assert_allclose(h["sx"], o["s"][:, :2], rtol=0, atol=1e-13)
        np.testing.assert_allclose(h["sn"], o["s"][:, 2:], rtol=0, atol=1e-13)
        for name in ("M", "Ff", "Fg", "E", "X"):
            assert h[name].shape == o[name].shape, name
            if 0 in o[name].shape:
                continue
            D = (h[name] - o[name]).toarray()
            assert abs(D).max() <= 1e-12 * max(abs(o[name]).max(), 1.0), name
        for _ in range(2):
            u = rng.uniform(-1, 1, m.N * m.N)
            ref = -(o["A"] @ u)
            assert np.abs(h["apply"](u) - ref).max() <= 1e-12 * np.abs(ref).max()
    # the inside field has no data points (the box faces lie outside the circle), the outside field all of them
    assert len(H[0]["sx"]) == 0 and len(H[1]["sx"]) == 4 * 20 * (prm["p"] + 1)
    # the coupling is the transpose pair of one symmetric interface form
    assert abs(H[0]["X"] - H[1]["X"].T).max() <= 1e-13 * abs(H[0]["X"]).max()


def test_composite_restatement_stability():
    """the 2D composite presets at their own CFL (wave-app.cc:152-221,
    :286-347) are outside RK4's stability region in this restatement: the
    outside field's corner DoFs carry the box faces' Nitsche penalty, dt
    sqrt(lambda_max(M^-1 A)) = 3.45 > 2 sqrt(2) for wave-composite; the inside
    field (2.14) and the inside-only wave preset (2.70) are inside it.  The
    device runs are compared with the oracle over the first steps at the
    presets' CFL and over whole runs at a reduced one
    (tests/test_gpu_cut_wave2d.py)."""
    prm = W.composite_params("wave-composite")
    m = W.CutWave2D(prm["p"], 20, prm["left"], prm["right"])
    dt = prm["cfl"] * m.h
    lam = []
    for loc in (W.INSIDE, W.OUTSIDE):
        o = m.matrices(prm["gamma_M"], prm["gamma_A"], prm["nitsche"], location=loc, interface_data=False,
                       domain_data=True, coupled=True)
        lu = spla.splu(o["M"].tocsc())
        op = spla.LinearOperator(o["A"].shape, matvec=lambda v, lu=lu, A=o["A"]: lu.solve(A @ v))
        lam.append(abs(spla.eigs(op, k=1, which="LM", return_eigenvectors=False, maxiter=5000)[0]))
    assert dt * np.sqrt(lam[0]) < 2 * np.sqrt(2) < dt * np.sqrt(lam[1])


@pytest.mark.parametrize("name", ["wave-composite", "heat-composite"])
def test_composite_preset_2d_warns_about_its_cfl(name):
    """the 2D composite presets carry the reference's CFL, at which
    the outside field is unstable in this restatement; preset() says so (1D
    composite presets, pinned by the reference's goldens, do not warn)"""
    import warnings

    import gdm_amd.cut_wave as CW

    with pytest.warns(RuntimeWarning, match="unstable"):
        P = CW.preset(name, 2)
    assert P["simulation"] == name and P["dim"] == 2
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        CW.preset(name, 1)
