"""CPU tests of the host side: the C-ABI library loads and exports every
entry point include/gdm_hip.h declares, fails loudly without a GPU, the slab
partition / local layout match the reference formula (oracle, system.h:
720-757), and the ghost-plane exchange of the multi-rank path is correct over
gloo with world_size 2 and 3 (the same code runs over RCCL on the GPU box).
"""
import ctypes
import os
import socket

import numpy as np
import pytest

import gdm_amd
from gdm_amd import _capi
from gdm_amd.distributed import HaloExchange, layout, slab
import oracle as O


def test_library_exports_every_declared_symbol():
    lib = _capi.load()
    declared = _capi.declared_symbols()
    assert len(declared) >= 20
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing


def test_abi_version_matches_header():
    txt = open(_capi.HEADER).read()
    import re

    v = int(re.search(r"#define\s+GDM_HIP_ABI_VERSION\s+(\d+)", txt).group(1))
    assert _capi.load().gdm_abi_version() == v


def test_null_arguments_are_rejected():
    lib = _capi.load()
    assert lib.gdm_op_create(None, 1, None, 0, 0, None) != _capi.GDM_OK
    assert "NULL" in _capi.last_error()
    assert lib.gdm_get_device_count(None) != _capi.GDM_OK


def test_bad_mesh_is_rejected_before_any_device_call():
    lib = _capi.load()
    m = _capi.MeshDesc()
    m.dim, m.fe_degree = 3, 4  # even degree: the reference tabulates odd p only (fe.h:321-323)
    m.n_subdivisions[:] = [8, 8, 8]
    m.hi[:] = [1.0, 1.0, 1.0]
    m.n_ranks, m.rank = 1, 0
    out = ctypes.c_void_p()
    rc = lib.gdm_op_create(ctypes.byref(m), 1, None, 0, 0, ctypes.byref(out))
    assert rc != _capi.GDM_OK and not out.value
    assert "odd" in _capi.last_error()
    m.fe_degree = 5
    m.n_subdivisions[:] = [4, 8, 8]  # fewer cells than p
    rc = lib.gdm_op_create(ctypes.byref(m), 1, None, 0, 0, ctypes.byref(out))
    assert rc != _capi.GDM_OK and ">= fe_degree" in _capi.last_error()
    m.n_subdivisions[:] = [8, 8, 8]
    a = (ctypes.c_double * 1)(1.0)
    rc = lib.gdm_op_create(ctypes.byref(m), 1, a, 1, 0, ctypes.byref(out))  # advection needs dim values
    assert rc != _capi.GDM_OK


@pytest.mark.skipif(_capi.device_count() > 0, reason="checks the no-GPU failure path")
def test_operator_fails_loudly_without_gpu():
    with pytest.raises(gdm_amd.GdmError):
        gdm_amd.GdmOperator(3, 3, 6, 0.0, 1.0, "advection", params=(1.0, 0.0, 0.0), device=0)


@pytest.mark.parametrize("n_last", [3, 7, 10, 31, 64, 511, 1023])
@pytest.mark.parametrize("n_ranks", [1, 2, 3, 4, 7, 8])
def test_slab_matches_reference_formula(n_last, n_ranks):
    m = O.Mesh(1, 1, n_last)
    owned = []
    for r in range(n_ranks):
        assert slab(n_last, n_ranks, r) == m.partition(n_ranks, r) or (
            # empty trailing ranks: the oracle keeps the raw (clamped) range
            slab(n_last, n_ranks, r)[1] == slab(n_last, n_ranks, r)[0]
        )
        pb, pe, cb, ce = slab(n_last, n_ranks, r)
        owned.extend(range(pb, pe))
    # every vertex plane is owned exactly once
    assert owned == list(range(n_last + 1))


@pytest.mark.parametrize("n_ranks", [2, 3, 4])
def test_layout_ghosts_cover_halo(n_ranks):
    n_last, ps, p = 40, 6, 5
    for r in range(n_ranks):
        L = layout(n_last, n_ranks, r, ps, p)
        assert L["ghost_planes_below"] == min(p, L["owned_plane_begin"])
        assert L["ghost_planes_above"] == min(p, n_last + 1 - L["owned_plane_end"])
        assert L["n_local"] == L["n_owned"] + (L["ghost_planes_below"] + L["ghost_planes_above"]) * ps


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _halo_worker(rank, world, port, n_last, ps, halo, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = layout(n_last, world, rank, ps, halo)
        gb = L["ghost_planes_below"]
        first = L["owned_plane_begin"] - gb
        n_planes = L["n_local"] // ps
        # owned planes hold their global plane index, ghosts -1
        v = torch.full((n_planes, ps), -1.0, dtype=torch.float64)
        own = L["owned_plane_end"] - L["owned_plane_begin"]
        for i in range(own):
            v[gb + i] = float(L["owned_plane_begin"] + i) + torch.arange(ps, dtype=torch.float64) / ps
        HaloExchange(n_last, world, rank, ps, halo).exchange(v.view(-1))
        expect = torch.stack([float(first + i) + torch.arange(ps, dtype=torch.float64) / ps for i in range(n_planes)])
        q.put((rank, bool(torch.equal(v, expect))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_last", [(2, 20), (3, 29)])
def test_halo_exchange_gloo(world, n_last):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, n_last, 7, 5, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    for p_ in procs:
        p_.join(120)
    assert all(p_.exitcode == 0 for p_ in procs), [p_.exitcode for p_ in procs]
    res = dict(q.get() for _ in range(world))
    assert all(res.values()), res


def test_local_layout_matches_oracle_partition_3d():
    """Global DoF numbering is lexicographic (x fastest, system.h:404-424), so
    an owned slab of vertex planes is one contiguous index range."""
    p, n = 3, (6, 5, 9)
    m = O.Mesh(3, p, list(n))
    for R in (2, 3):
        for r in range(R):
            pb, pe, cb, ce = m.partition(R, r)
            L = layout(n[2], R, r, (n[0] + 1) * (n[1] + 1), p)
            assert (L["owned_plane_begin"], L["owned_plane_end"]) == (pb, min(pe, n[2] + 1))
            # cells of the slab touch only owned + ghost planes
            for c in range(cb * n[0] * n[1], ce * n[0] * n[1], 7):
                dofs = m.cell_dofs(c).astype(np.int64)
                planes = dofs // ((n[0] + 1) * (n[1] + 1))
                lo = L["owned_plane_begin"] - L["ghost_planes_below"]
                hi = L["owned_plane_end"] + L["ghost_planes_above"]
                assert planes.min() >= lo and planes.max() < hi


def _np_line_solver(Ms):
    """line_solve(axis, v, n_lines, stride, A, B, C) over dense 1D mass matrices."""
    import torch

    def solve(axis, v, n_lines, stride, A, B, C):
        M = Ms[axis]
        n = M.shape[0]
        a = v.numpy()
        for l in range(n_lines):
            base = (l // A) * B + (l % A) * C
            idx = base + stride * np.arange(n)
            a[idx] = np.linalg.solve(M, a[idx])
        return v

    return solve


def _dense_1d(m, d):
    band = m.matrices_1d(d)[0]
    n, W = band.shape
    p = (W - 1) // 2
    M = np.zeros((n, n))
    for i in range(n):
        for k in range(W):
            j = i - p + k
            if 0 <= j < n:
                M[i, j] = band[i, k]
    return M


def _mass_worker(rank, world, port, dim, p, n, q):
    import torch
    import torch.distributed as dist
    from gdm_amd.distributed import DistributedMassSolve

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = O.Mesh(dim, p, n)
        Ms = [_dense_1d(m, d) for d in range(dim)]
        N = [n + 1] * dim
        ds = DistributedMassSolve(dim, N, world, rank, line_solve=_np_line_solver(Ms))
        r = np.random.default_rng(7).uniform(-1, 1, m.n_dofs)
        L = ds.lays[rank]
        P = ds.plane
        mine = torch.from_numpy(r[L["owned_plane_begin"] * P:L["owned_plane_end"] * P].copy())
        x = torch.empty_like(mine)
        ds.solve(mine, x)
        q.put((rank, L["owned_plane_begin"] * P, x.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dim,p,n", [(2, 3, 3, 7), (3, 3, 5, 11), (3, 2, 5, 13), (2, 1, 3, 20)])
def test_distributed_mass_solve_gloo(world, dim, p, n):
    """Slab-distributed exact mass inverse (local directions in place, the
    partitioned direction after a point-to-point transpose) == the global
    Kronecker inverse == CG(1e-14) on the assembled matrix (test_oracle_kron)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mass_worker, args=(r, world, port, dim, p, n, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p_ in procs:
        p_.join(120)
    assert all(p_.exitcode == 0 for p_ in procs), [p_.exitcode for p_ in procs]
    m = O.Mesh(dim, p, n)
    r = np.random.default_rng(7).uniform(-1, 1, m.n_dofs)
    ref = m.kron_mass_inverse(r)
    x = np.zeros_like(ref)
    for _, off, v in res:
        x[off:off + len(v)] = v
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) < 1e-12


def _plan(dim, p, n_sub, n_ranks, rank):
    m = _capi.MeshDesc()
    m.dim, m.fe_degree = dim, p
    for d in range(3):
        m.n_subdivisions[d] = n_sub[d] if d < dim else 1
        m.lo[d], m.hi[d] = 0.0, 1.0
    m.n_ranks, m.rank, m.periodic = n_ranks, rank, 0
    h = _capi.Halo()
    _capi.check(_capi.load().gdm_halo_plan(ctypes.byref(m), ctypes.byref(h)), "gdm_halo_plan")
    return h.as_dict()


@pytest.mark.parametrize("dim,p,n_sub", [(3, 5, (20, 9, 511)), (3, 7, (8, 8, 255)), (2, 5, (30, 100)),
                                         (3, 3, (6, 6, 40))])
@pytest.mark.parametrize("n_ranks", [2, 3, 4, 8])
def test_halo_plan_matches_exchange(dim, p, n_sub, n_ranks):
    """gdm_halo_plan (pure host ABI) describes exactly the ranges the
    torch.distributed exchange moves (gdm_amd.distributed.HaloExchange), the
    sends of one rank land in the receives of its neighbour, and the
    reference's deal.II ghost layer (system.h:657-688, 767-771: the DoF boxes
    of one ghost cell layer) is reported for the adapter."""
    nl = n_sub[dim - 1]
    plane = int(np.prod([n_sub[d] + 1 for d in range(dim - 1)]))
    plans = [_plan(dim, p, n_sub, n_ranks, r) for r in range(n_ranks)]
    m = O.Mesh(dim, p, list(n_sub))
    for r, h in enumerate(plans):
        me = layout(nl, n_ranks, r, plane, p)
        assert h["owned_offset"] == me["ghost_planes_below"] * plane
        if r > 0:
            lo = plans[r - 1]
            assert h["rank_below"] == r - 1 and lo["rank_above"] == r
            assert h["send_below_count"] == lo["recv_above_count"]
            assert h["recv_below_count"] == lo["send_above_count"]
            assert h["recv_below_offset"] == 0
            assert h["send_below_offset"] == h["owned_offset"]
        else:
            assert h["rank_below"] == -1
        if r + 1 < n_ranks:
            assert h["rank_above"] == r + 1
            assert h["recv_above_offset"] == me["n_local"] - h["recv_above_count"]
            assert h["send_above_offset"] + h["send_above_count"] == h["owned_offset"] + me["n_owned"]
        # deal.II ghost planes = locally active planes (DoF boxes of owned + one ghost cell layer) - owned
        pb, pe, cb, ce = slab(nl, n_ranks, r)
        lo_c, hi_c = max(cb - 1, 0), min(ce + 1, nl)
        planes = set()
        for c in range(lo_c, hi_c):
            cell = [0] * (dim - 1) + [c]
            idx = sum(ci * int(np.prod([n_sub[e] for e in range(d)])) for d, ci in enumerate(cell))
            planes |= {int(g) // plane for g in m.cell_dofs(idx)}
        assert h["dealii_ghost_planes_below"] == len([q for q in planes if q < pb])
        assert h["dealii_ghost_planes_above"] == len([q for q in planes if q >= pe])


class _NpSpikeOp:
    """numpy restatement of the distributed mass inverse's two steps (the
    truncated SPIKE scheme of gdm_mass_solve_slab / gdm_mass_solve_interface,
    include/gdm_hip.h) on dense 1D mass matrices -- a test double for the
    device operator, so the exchange orchestration of
    gdm_amd.distributed.SlabMassSolve runs on gloo without a GPU."""

    def __init__(self, dim, p, n, world, rank):
        from gdm_amd.distributed import layout, slab

        m = O.Mesh(dim, p, list(n))
        self.Ms = [_dense_1d(m, d) for d in range(dim)]
        self.dim, self.p = dim, p
        self.plane = int(np.prod([n[d] + 1 for d in range(dim - 1)])) if dim > 1 else 1
        self.L = layout(n[dim - 1], world, rank, self.plane, p)
        self.slabs = [slab(n[dim - 1], world, s)[:2] for s in range(world)]
        self.rank, self.world = rank, world

    def owned_view(self, local):
        b = self.L["ghost_planes_below"] * self.plane
        return local[b:b + self.L["n_owned"]]

    def _spikes(self, s):
        Mq, p = self.Ms[self.dim - 1], self.p
        pb, pe = self.slabs[s]
        A = Mq[pb:pe, pb:pe]
        V = np.linalg.solve(A, Mq[pb:pe, pe:pe + p]) if pe < Mq.shape[0] else np.zeros((pe - pb, p))
        W = np.linalg.solve(A, Mq[pb:pe, pb - p:pb]) if pb > 0 else np.zeros((pe - pb, p))
        return A, V, W

    def mass_solve_slab(self, rhs, x):
        A, _, _ = self._spikes(self.rank)
        v = rhs.numpy().reshape(A.shape[0], self.plane)
        v = np.linalg.solve(A, v)
        if self.dim >= 2:
            inner = self.Ms[0] if self.dim == 2 else np.kron(self.Ms[1], self.Ms[0])
            v = np.linalg.solve(inner, v.T).T
        x.numpy()[:] = v.reshape(-1)
        return x

    def _interface(self, x_local):
        p, P, r = self.p, self.plane, self.rank
        gb = self.L["ghost_planes_below"]
        a = x_local.numpy().reshape(-1, P)
        n = self.slabs[r][1] - self.slabs[r][0]
        own = a[gb:gb + n]
        _, V, W = self._spikes(r)
        b = np.zeros((p, P))
        t = np.zeros((p, P))
        if r > 0:
            _, Vl, _ = self._spikes(r - 1)
            S = np.block([[np.eye(p), Vl[-p:]], [W[:p], np.eye(p)]])
            b = np.linalg.solve(S, np.concatenate([a[gb - p:gb], own[:p]]))[:p]
        if r + 1 < self.world:
            _, _, Wh = self._spikes(r + 1)
            S = np.block([[np.eye(p), V[-p:]], [Wh[:p], np.eye(p)]])
            t = np.linalg.solve(S, np.concatenate([own[-p:], a[gb + n:gb + n + p]]))[p:]
        return own, V, W, b, t

    def mass_solve_interface_round(self, x_local, k):
        """refinement round: the edge planes become g - (dropped far-spike
        couplings at the current interface values)"""
        p = self.p
        own, V, W, b, t = self._interface(x_local)
        if k == 0:
            self.G0 = (own[:p].copy(), own[-p:].copy())
        own[:p] = self.G0[0] - V[:p] @ t
        own[-p:] = self.G0[1] - W[-p:] @ b
        return x_local

    def mass_solve_interface(self, x_local):
        p = self.p
        own, V, W, b, t = self._interface(x_local)
        if getattr(self, "G0", None) is not None:
            own[:p], own[-p:] = self.G0
            self.G0 = None
        own -= V @ t + W @ b
        return x_local


class _NpSlabRkOp(_NpSpikeOp):
    """_NpSpikeOp plus what SlabRK4 calls on a rank operator: the slab's
    compute_rhs (no inflow data) K = B_x (x) M_q + M_x (x) B_q (2D, outflow
    traces folded into B, advection/stiffness.h:411-417, :520-529) from the
    local vector's planes to the owned ones, the RK update, the interface with
    ghost planes (gdm_mass_solve_interface_ghosts: b / t into the ghosts)."""

    def __init__(self, p, n, world, rank, a):
        super().__init__(2, p, n, world, rank)
        m = O.Mesh(2, p, list(n))
        B = [m.advection_outflow_B(d, a[d]) for d in range(2)]
        self.Bs = [self._dense(band) for band in B]
        L = self.L
        self.lb = L["owned_plane_begin"] - L["ghost_planes_below"]
        self.le = L["owned_plane_end"] + L["ghost_planes_above"]
        self.n_local = L["n_local"]

    @staticmethod
    def _dense(band):
        n, W = band.shape
        p = (W - 1) // 2
        A = np.zeros((n, n))
        for i in range(n):
            for k in range(W):
                if 0 <= i - p + k < n:
                    A[i, i - p + k] = band[i, k]
        return A

    def new_vector(self, local=True):
        import torch

        return torch.zeros(self.n_local if local else self.L["n_owned"], dtype=torch.float64)

    def apply(self, src_local, dst_owned):
        L, P = self.L, self.plane
        pb, pe = L["owned_plane_begin"], L["owned_plane_end"]
        U = src_local.numpy().reshape(-1, P)
        Mq, Bq = self.Ms[1][pb:pe, self.lb:self.le], self.Bs[1][pb:pe, self.lb:self.le]
        out = Mq @ U @ self.Bs[0].T + Bq @ U @ self.Ms[0].T
        dst_owned.numpy()[:] = out.reshape(-1)
        return dst_owned

    def rk_update(self, beta, k, acc_in, acc_out, alpha=0.0, y=None, Y=None):
        kv, ai = k.numpy(), acc_in.numpy().copy()
        if Y is not None:
            Y.numpy()[:] = y.numpy() + alpha * kv
        acc_out.numpy()[:] = ai + beta * kv
        return acc_out

    def mass_solve_interface_ghosts(self, x_local):
        p, P, r = self.p, self.plane, self.rank
        gb = self.L["ghost_planes_below"]
        own, V, W, b, t = self._interface(x_local)
        if getattr(self, "G0", None) is not None:
            own[:p], own[-p:] = self.G0
            self.G0 = None
        own -= V @ t + W @ b
        a = x_local.numpy().reshape(-1, P)
        n = own.shape[0]
        if r > 0:
            a[gb - p:gb] = b
        if r + 1 < self.world:
            a[gb + n:gb + n + p] = t
        return x_local

    def mass_solve_interface_rk(self, x_local, beta, acc_in, acc_out, alpha=0.0, y=None, Y=None):
        k = self.mass_solve_interface_ghosts(x_local.clone())
        return self.rk_update(beta, k, acc_in, acc_out, alpha, y, Y)


def _rk_worker(rank, world, port, p, n, a, steps, q):
    import torch
    import torch.distributed as dist
    from gdm_amd.distributed import HaloExchange, SlabRK4

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        op = _NpSlabRkOp(p, n, world, rank, a)
        halo = HaloExchange(n[1], world, rank, op.plane, p)
        rounds = _capi.mass_spike_rounds(2, p, list(n), world)
        m = O.Mesh(2, p, list(n))
        u0 = np.sin(np.linspace(0.0, 7.0, m.n_dofs)) + 0.3 * np.cos(np.linspace(0.0, 23.0, m.n_dofs))
        L = op.L
        mine = torch.from_numpy(u0[L["owned_plane_begin"] * op.plane:L["owned_plane_end"] * op.plane].copy())
        out = {}
        for one in (False, True):
            rk = SlabRK4([op], lambda vs: [halo.exchange(v) for v in vs], one_exchange=one, rounds=rounds)
            rk.set_solution([mine])
            for s in range(steps):
                rk.step(0.01 * s, 0.01)
            out[one] = op.owned_view(rk.y[0]).numpy().copy()
        q.put((rank, L["owned_plane_begin"] * op.plane, out[False], out[True]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,p,n", [(2, 3, (6, 60)), (3, 5, (5, 90)), (4, 3, (4, 48))])
def test_one_exchange_rk_matches_two_exchange_gloo(world, p, n):
    """the RK4 step with ONE exchange per stage (the
    stage vector's ghost planes maintained from the SPIKE interface solution,
    updates over the local vectors) == the reference's two exchanges per stage
    (update_ghost_values before compute_rhs, stiffness.h:343, + the solve's),
    to 1e-13 after 6 steps, and both == the single-rank RK4 of
    y' = M^-1 K y to 1e-12 -- SlabRK4 over gloo with a numpy test double of
    the rank operator (4 ranks of 12 planes at p = 3: one refinement round)."""
    import torch.multiprocessing as mp

    a, steps = (0.8, -0.6), 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rk_worker, args=(r, world, port, p, n, a, steps, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p_ in procs:
        p_.join(120)
    assert all(p_.exitcode == 0 for p_ in procs), [p_.exitcode for p_ in procs]
    m = O.Mesh(2, p, list(n))
    two, one = np.zeros(m.n_dofs), np.zeros(m.n_dofs)
    for _, off, v2, v1 in res:
        two[off:off + len(v2)] = v2
        one[off:off + len(v1)] = v1
    assert np.linalg.norm(one - two) / np.linalg.norm(two) < 1e-13
    # single-rank reference: classic RK4 of y' = M^-1 K y
    d = _NpSlabRkOp(p, n, 1, 0, a)
    Mi = np.kron(d.Ms[1], d.Ms[0])
    K = np.kron(d.Ms[1], d.Bs[0]) + np.kron(d.Bs[1], d.Ms[0])
    f = lambda y: np.linalg.solve(Mi, K @ y)  # noqa: E731
    y = np.sin(np.linspace(0.0, 7.0, m.n_dofs)) + 0.3 * np.cos(np.linspace(0.0, 23.0, m.n_dofs))
    h = 0.01
    for _ in range(steps):
        k1 = f(y)
        k2 = f(y + 0.5 * h * k1)
        k3 = f(y + 0.5 * h * k2)
        k4 = f(y + h * k3)
        y = y + h / 6 * k1 + h / 3 * k2 + h / 3 * k3 + h / 6 * k4
    assert np.linalg.norm(two - y) / np.linalg.norm(y) < 1e-12


def _spike_worker(rank, world, port, dim, p, n, q):
    import torch
    import torch.distributed as dist
    from gdm_amd.distributed import HaloExchange, SlabMassSolve

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        op = _NpSpikeOp(dim, p, n, world, rank)
        halo = HaloExchange(n[dim - 1], world, rank, op.plane, p)
        m = O.Mesh(dim, p, list(n))
        r = np.random.default_rng(11).uniform(-1, 1, m.n_dofs)
        L = op.L
        mine = torch.from_numpy(r[L["owned_plane_begin"] * op.plane:L["owned_plane_end"] * op.plane].copy())
        x_local = torch.zeros(L["n_local"], dtype=torch.float64)
        rounds = _capi.mass_spike_rounds(dim, p, list(n), world)
        x = SlabMassSolve(op, halo, rounds).solve(mine, x_local)
        q.put((rank, L["owned_plane_begin"] * op.plane, x.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dim,p,n", [(2, 2, 3, (5, 200)), (3, 2, 5, (5, 240)), (4, 1, 3, (400,)),
                                           (2, 3, 3, (3, 3, 150)), (8, 1, 7, (255,)), (8, 3, 7, (7, 8, 255)),
                                           (6, 2, 5, (5, 150))])
def test_slab_mass_solve_gloo(world, dim, p, n):
    """Distributed exact mass inverse by slab-local solves + one p-plane
    exchange (+ the refinement rounds of gdm_mass_spike_rounds for thin
    slabs: C4 at 8 ranks = 32 planes at p = 7, and 25 planes at p = 5) + the
    2p x 2p interface systems (SlabMassSolve over gloo, numpy test double of
    the device steps) == the global Kronecker inverse to 1e-13; the library's
    pure-host gdm_mass_spike_eps reports the dropped coupling the numpy
    spikes show."""
    import torch.multiprocessing as mp

    eps = _capi.mass_spike_eps(dim, p, list(n), world)
    rounds = _capi.mass_spike_rounds(dim, p, list(n), world)
    assert rounds == next(m for m in range(4) if eps ** (m + 1) <= 1e-15), (eps, rounds)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spike_worker, args=(r, world, port, dim, p, n, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p_ in procs:
        p_.join(120)
    assert all(p_.exitcode == 0 for p_ in procs), [p_.exitcode for p_ in procs]
    m = O.Mesh(dim, p, list(n))
    r = np.random.default_rng(11).uniform(-1, 1, m.n_dofs)
    ref = m.kron_mass_inverse(r)
    x = np.zeros_like(ref)
    for _, off, v in res:
        x[off:off + len(v)] = v
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) < 1e-13


@pytest.mark.parametrize("dim,p,n,world", [(2, 3, (5, 60), 2), (1, 5, (120,), 3), (3, 7, (7, 7, 255), 4),
                                           (3, 7, (7, 7, 255), 8)])
def test_mass_spike_eps_matches_numpy(dim, p, n, world):
    """gdm_mass_spike_eps (C++ host math) == the largest far-spike entry of
    the numpy restatement; thin slabs (C4, 8 ranks: 32 planes at p = 7) are
    reported above the 1e-15 the solve accepts."""
    ops = [_NpSpikeOp(dim, p, n, world, s) for s in range(world)]
    eps = 0.0
    for s, op in enumerate(ops):
        _, V, W = op._spikes(s)
        if s > 0:
            eps = max(eps, np.abs(W[-p:]).max())
        if s + 1 < world:
            eps = max(eps, np.abs(V[:p]).max())
    got = _capi.mass_spike_eps(dim, p, list(n), world)
    assert got == pytest.approx(eps, rel=1e-6, abs=1e-300)
    if (dim, p, world) == (3, 7, 8):
        # thin slabs: one refinement round (error ~ eps^2 = 4e-16)
        assert got > 1e-15 and got ** 2 < 1e-15
        assert _capi.mass_spike_rounds(dim, p, list(n), world) == 1


def test_mass_spike_rounds_refuses_slabs_thinner_than_2p():
    """8 ranks of p = 7 on 100 cells: 12-13 planes per slab < 2p, the edge
    planes of the refinement rounds would overlap -> refused (-1)."""
    assert _capi.mass_spike_rounds(1, 7, (100,), 8) == -1
    assert _capi.mass_spike_rounds(3, 5, (5, 5, 511), 8) == 0
