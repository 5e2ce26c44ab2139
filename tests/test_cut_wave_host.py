"""Host assembly of the device cut-cell wave / heat operators
(csrc/gdm_cut_wave.cpp, the matrices gdm_cut_wave_create uploads) against
the 1D restatement oracle/cut1d.py, on the CPU.

The device evaluates compute_rhs = [impl] (Z S u + C u) + Ff f(x_q) + Fg g(x_s)
with S = -(v', u') of the uncut box (the 1D wave stencil, here the oracle's
band matrix -L), Z zeroing the rows of DoFs in the boxes of cut / outside
cells; M and the heat-impl stiffness K are assembled; E evaluates u_h at the
inside quadrature points.  Checked here: every piece against the oracle's
cell loops to 1e-13, and the device formulation of the wave-rk, heat-rk and
heat-impl loops (these matrices, exact solves) against the reference goldens
applications/wave/tests/{wave_0,heat_1,heat_0}.output to the 2e-8 of
tests/test_cut1d_golden.py."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import cut1d  # noqa: E402
import oracle as O  # noqa: E402

REF = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_outputs.json")))["wave_app"]["cases"]


def _lib():
    import gdm_amd

    L = gdm_amd.load()
    P, I64, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
    L.gdmh_cut_wave_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, D, D, ctypes.c_int, P,
                                       ctypes.c_int, ctypes.c_int, D, D, D,
                                       ctypes.POINTER(P), ctypes.c_char_p, ctypes.c_size_t]
    L.gdmh_cut_wave_info.argtypes = [P] + [ctypes.POINTER(I64)] * 3 + [P]
    L.gdmh_cut_wave_csr.argtypes = [P, ctypes.c_int] + [ctypes.POINTER(ctypes.c_void_p)] * 3
    L.gdmh_cut_wave_points.argtypes = [P] + [ctypes.POINTER(ctypes.c_void_p)] * 5 + [ctypes.POINTER(I64)]
    L.gdmh_cut_wave_destroy.argtypes = [P]
    return L


def _arr(ptr, n, dt):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(dt)), shape=(n,)).copy() if n else np.zeros(0)


def host_system(prm, location=-1, flags=1):
    """dict of the device operator's host arrays (dense matrices) for a preset
    (the field of `location`, Nitsche data / coupling `flags`)"""
    import gdm_amd.cut_wave as CW

    L = _lib()
    p, n, left, right = prm["p"], prm["n"], prm["left"], prm["right"]
    h = (right - left) / n
    gl = CW.gauss_lobatto(p + 1)
    x = (left + np.arange(n) * h)[:, None] + gl[None, :] * h
    ls = np.ascontiguousarray((np.abs(x) - 1.0).reshape(-1))
    S = ctypes.c_void_p()
    err = ctypes.create_string_buffer(256)
    assert L.gdmh_cut_wave_create(1, p, n, left, right, p, ls.ctypes.data, location, flags, prm["gamma_M"], prm["gamma_A"],
                                  prm["nitsche"], ctypes.byref(S), err, 256) == 0, err.value
    try:
        nd, nq, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        cells = (ctypes.c_int64 * 3)()
        L.gdmh_cut_wave_info(S, ctypes.byref(nd), ctypes.byref(nq), ctypes.byref(ns), cells)
        N, NQ, NS = nd.value, nq.value, ns.value
        shape = {0: (N, N), 1: (N, NQ), 2: (N, NS), 3: (NQ, N), 4: (N, N), 5: (N, N), 6: (N, N)}
        out = {}
        for w, name in enumerate(("C", "Ff", "Fg", "E", "M", "K", "X")):
            q = [ctypes.c_void_p() for _ in range(3)]
            L.gdmh_cut_wave_csr(S, w, *[ctypes.byref(x) for x in q])
            rows, cols = shape[w]
            rp = _arr(q[0], rows + 1, ctypes.c_int64)
            ci = _arr(q[1], rp[-1], ctypes.c_uint32).astype(np.int64)
            v = _arr(q[2], rp[-1], ctypes.c_double)
            A = np.zeros((rows, cols))
            for r in range(rows):
                for k in range(rp[r], rp[r + 1]):
                    A[r, ci[k]] += v[k]
            out[name] = A
        q = [ctypes.c_void_p() for _ in range(5)]
        nz = ctypes.c_int64()
        L.gdmh_cut_wave_points(S, *[ctypes.byref(x) for x in q], ctypes.byref(nz))
        out["qx"], out["qw"] = _arr(q[0], NQ, ctypes.c_double), _arr(q[1], NQ, ctypes.c_double)
        out["sx"], out["sn"] = _arr(q[2], NS, ctypes.c_double), _arr(q[3], NS, ctypes.c_double)
        out["zero"] = _arr(q[4], nz.value, ctypes.c_int64)
        out["cells"] = tuple(cells)
    finally:
        L.gdmh_cut_wave_destroy(S)
    m = O.Mesh(1, p, n, left, right)
    Lb = m.matrices_1d(0)[2]  # band form of L = (v', u') of the uncut box
    Lf = np.zeros((N, N))
    for i in range(N):
        for k in range(2 * p + 1):
            j = i - p + k
            if 0 <= j < N:
                Lf[i, j] = Lb[i, k]
    Z = np.ones(N)
    Z[out["zero"]] = 0.0
    out["A"] = np.diag(Z) @ (-Lf) + out["C"]  # the device compute_rhs operator (impl part)
    return out


def _params(simulation):
    return cut1d.wave_params() if simulation == "wave" else cut1d.heat_params(simulation)


@pytest.mark.parametrize("simulation", ["wave", "heat-rk"])
def test_host_matrices_match_oracle(simulation):
    prm = _params(simulation)
    H = host_system(prm)
    m = cut1d.Cut1D(prm["p"], prm["n"], prm["left"], prm["right"], cut1d._sphere)
    N = m.N
    assert H["cells"] == (sum(c["loc"] == m.INSIDE for c in m.cells), sum(c["loc"] == m.INTERSECTED for c in m.cells),
                          sum(c["loc"] == m.OUTSIDE for c in m.cells))
    M = m.mass_matrix(prm["gamma_M"])
    K = m.stiffness_matrix(prm["gamma_A"], prm["nitsche"])
    np.testing.assert_allclose(H["M"], M, rtol=0, atol=1e-13 * abs(M).max())
    np.testing.assert_allclose(H["K"], K, rtol=0, atol=1e-13 * abs(K).max())
    # the operator part of compute_rhs, column by column (linear in u; zero
    # interface data: the oracle applies the surface Nitsche terms with g only)
    zero = lambda x, t: 0.0  # noqa: E731
    A = np.stack([m.rhs(e, 0.0, True, prm["gamma_A"], prm["nitsche"], g=zero) for e in np.eye(N)], axis=1)
    np.testing.assert_allclose(H["A"], A, rtol=0, atol=1e-13 * abs(A).max())
    # data parts at t = 0.3: (v, f) and the Nitsche data g
    t = 0.3
    f = prm["f"] or (lambda x, t: np.cos(3 * x) + t)
    r = m.rhs(np.zeros(N), t, False, prm["gamma_A"], prm["nitsche"], f=f, g=prm["g"])
    got = H["Ff"] @ np.array([f(x, t) for x in H["qx"]]) + H["Fg"] @ np.array([prm["g"](x, t) for x in H["sx"]])
    np.testing.assert_allclose(got, r, rtol=0, atol=1e-13 * abs(r).max())
    # postprocess pieces: E u at the quadrature points with their weights
    u = np.random.default_rng(1).uniform(-1, 1, N)
    vals = H["E"] @ u
    e = vals - np.array([prm["exact"](x, t) for x in H["qx"]])
    l2, l1, linf = np.sqrt(np.sum(e * e * H["qw"])), np.sum(np.abs(e) * H["qw"]), np.max(np.abs(e))
    np.testing.assert_allclose((l2, l1, linf), m.errors(u, prm["exact"], t), rtol=1e-13)


@pytest.mark.parametrize("case,simulation", [("wave_0", "wave"), ("heat_1", "heat-rk"), ("heat_0", "heat-impl")])
def test_device_formulation_reproduces_golden(case, simulation):
    """the wave application's time loop (cut1d.run's, which is pinned to the
    goldens) with the device operators: compute_rhs = A u + Ff f + Fg g, the
    assembled M, K and the quadrature postprocess"""
    prm = _params(simulation)
    H = host_system(prm)
    Minv = np.linalg.inv(H["M"])
    h = (prm["right"] - prm["left"]) / prm["n"]
    N = H["M"].shape[0]

    def rhs(u, t, impl):
        r = H["Ff"] @ np.array([prm["f"](x, t) for x in H["qx"]]) if prm["f"] else np.zeros(N)
        r = r + H["Fg"] @ np.array([prm["g"](x, t) for x in H["sx"]])
        return (H["A"] @ u + r) if impl else r

    def post(u, t):
        e = H["E"] @ u - np.array([prm["exact"](x, t) for x in H["qx"]])
        return np.sqrt(np.sum(e * e * H["qw"])), np.sum(np.abs(e) * H["qw"]), np.max(np.abs(e))

    xv = prm["left"] + np.arange(N) * h
    u = np.array([prm["exact"](x, prm["start_t"]) for x in xv])
    time = cut1d.DiscreteTime(prm["start_t"], prm["end_t"], prm["cfl"] * h ** prm["cfl_pow"])
    rows = [(0, 0.0) + post(u, 0.0)]
    y = np.concatenate([u, np.zeros(N)]) if simulation == "wave" else u
    n = 0
    while not time.is_at_end():
        t0, dt = time.t, time.next_step_size()
        if simulation == "wave":
            y = cut1d.rk4_step(lambda t, y: np.concatenate([y[N:], Minv @ rhs(y[:N], t, True)]), t0, dt, y)
            u = y[:N]
        elif simulation == "heat-rk":
            y = cut1d.rk4_step(lambda t, y: Minv @ rhs(y, t, True), t0, dt, y)
            u = y
        else:
            u = np.linalg.solve(H["M"] + dt * H["K"], H["M"] @ u + dt * rhs(u, t0 + dt, False))
        n += 1
        rows.append((n, t0 + dt) + post(u, t0 + dt))
        time.advance()
    ref = REF[case]["steps"]
    assert len(rows) == len(ref)
    for got, exp in zip(rows, ref):
        assert got[0] == exp[0] and abs(got[1] - exp[1]) <= 5.000001e-6
        np.testing.assert_allclose(got[2:], exp[2:], rtol=2e-8, atol=0)


@pytest.mark.parametrize("case,simulation", [("wave_composite_0", "wave-composite"),
                                             ("heat_composite_0", "heat-composite")])
def test_composite_device_formulation(case, simulation):
    """the composite presets with the device operators of two handles
    (inside: domain data + coupling, outside: domain data + coupling):
    r_own = (Z S + C) u_own + X u_other + Ff f + Fg g_D; the matrices against
    the oracle's, the time loop against the goldens"""
    P = cut1d.composite_params(simulation)
    flags = 2 | 4
    H = [host_system(P, loc, flags) for loc in (-1, 1)]
    m = cut1d.Cut1D(P["p"], P["n"], P["left"], P["right"], cut1d._sphere)
    N = m.N
    for h, loc in zip(H, (-1, 1)):
        M = m.mass_matrix(P["gamma_M"], loc)
        np.testing.assert_allclose(h["M"], M, rtol=0, atol=1e-13 * abs(M).max())
    # the operator parts, column by column: own field and partner
    for e in np.eye(N)[:: 3]:
        c0, c1 = m.coupling(e, np.zeros(N), P["nitsche"])
        d0, d1 = m.coupling(np.zeros(N), e, P["nitsche"])
        zero = lambda x, t: 0.0  # noqa: E731
        own0 = m.rhs(e, 0.0, True, P["gamma_A"], P["nitsche"], location=-1, g_domain=zero) + c0
        own1 = m.rhs(e, 0.0, True, P["gamma_A"], P["nitsche"], location=1, g_domain=zero) + d1
        for got, ref in ((H[0]["A"] @ e, own0), (H[1]["A"] @ e, own1), (H[0]["X"] @ e, d0), (H[1]["X"] @ e, c1)):
            np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * max(abs(ref).max(), 1.0))
    Minv = [np.linalg.inv(h["M"]) for h in H]
    h_ = (P["right"] - P["left"]) / P["n"]

    def data(h, t):
        r = h["Ff"] @ np.array([P["f"](x, t) for x in h["qx"]]) if P["f"] else np.zeros(N)
        return r + h["Fg"] @ np.array([P["g_domain"](x, t) for x in h["sx"]])

    def fields(t, u0, u1):
        r0 = H[0]["A"] @ u0 + H[0]["X"] @ u1 + data(H[0], t)
        r1 = H[1]["A"] @ u1 + H[1]["X"] @ u0 + data(H[1], t)
        return Minv[0] @ r0, Minv[1] @ r1

    def post(h, u, t):
        e = h["E"] @ u - np.array([P["exact"](x, t) for x in h["qx"]])
        return np.sqrt(np.sum(e * e * h["qw"])), np.sum(np.abs(e) * h["qw"]), np.max(np.abs(e))

    xv = P["left"] + np.arange(N) * h_
    u = np.array([P["exact"](x, P["start_t"]) for x in xv])
    if simulation == "wave-composite":
        y = np.concatenate([u, u, np.zeros(2 * N)])
        f = lambda t, y: np.concatenate([y[2 * N:], *fields(t, y[:N], y[N:2 * N])])  # noqa: E731
    else:
        y = np.concatenate([u, u])
        f = lambda t, y: np.concatenate(fields(t, y[:N], y[N:]))  # noqa: E731
    time = cut1d.DiscreteTime(P["start_t"], P["end_t"], P["cfl"] * h_ ** P["cfl_pow"])
    rows = [(0, 0.0) + post(H[0], u, 0.0), (0, 0.0) + post(H[1], u, 0.0)]
    n = 0
    while not time.is_at_end():
        t0, dt = time.t, time.next_step_size()
        y = cut1d.rk4_step(f, t0, dt, y)
        n += 1
        rows += [(n, t0 + dt) + post(H[0], y[:N], t0 + dt), (n, t0 + dt) + post(H[1], y[N:2 * N], t0 + dt)]
        time.advance()
    ref = REF[case]["steps"]
    assert len(rows) == len(ref)
    for got, exp in zip(rows, ref):
        assert got[0] == exp[0] and abs(got[1] - exp[1]) <= 5.000001e-6
        np.testing.assert_allclose(got[2:], exp[2:], rtol=2e-8, atol=0)
