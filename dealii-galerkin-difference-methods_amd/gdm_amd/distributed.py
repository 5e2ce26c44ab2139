"""Slab partition and ghost-plane exchange (one process per GPU).

Mirrors the reference's MPI distribution: cells and vertex planes of the last
coordinate are dealt out in slabs (include/gdm/system.h:720-757), and the
ghost DoFs a rank reads (solution.update_ghost_values(),
applications/advection/include/gdm/advection/stiffness.h:343) are imported
from its two slab neighbours.  Owner-computes: each rank imports p planes from
each neighbour and writes only its owned rows, so no compress(add) export
step is needed (stiffness.h:605).

The exchange moves whole contiguous planes with torch.distributed
point-to-point calls: RCCL over xGMI for CUDA tensors (backend "nccl"), gloo
for the CPU tests of the same code path.
"""


def slab(n_cells_last, n_ranks, rank):
    """(plane_begin, plane_end, cell_begin, cell_end) -- system.h:723-757."""
    stride = (n_cells_last + n_ranks - 1) // n_ranks
    pb = min(0 if rank == 0 else stride * rank + 1, n_cells_last + 1)
    pe = min(stride * (rank + 1) + 1, n_cells_last + 1)
    cb = min(stride * rank, n_cells_last)
    ce = min(stride * (rank + 1), n_cells_last)
    return pb, max(pb, pe), cb, max(cb, ce)


def layout(n_cells_last, n_ranks, rank, plane_size, halo):
    """Local layout [ghost below | owned | ghost above] of one rank (the same
    numbers gdm_op_layout reports)."""
    pb, pe, cb, ce = slab(n_cells_last, n_ranks, rank)
    n_planes = n_cells_last + 1
    own = pe - pb
    gb = min(halo, pb) if own > 0 else 0
    ga = min(halo, n_planes - pe) if own > 0 else 0
    return {
        "owned_plane_begin": pb,
        "owned_plane_end": pe,
        "cell_plane_begin": cb,
        "cell_plane_end": ce,
        "ghost_planes_below": gb,
        "ghost_planes_above": ga,
        "plane_size": plane_size,
        "n_owned": own * plane_size,
        "n_local": (own + gb + ga) * plane_size,
    }


class HaloExchange:
    """Fill the ghost planes of a local vector from the slab neighbours."""

    def __init__(self, n_cells_last, n_ranks, rank, plane_size, halo, group=None):
        self.rank, self.n_ranks = rank, n_ranks
        self.me = layout(n_cells_last, n_ranks, rank, plane_size, halo)
        self.lo = layout(n_cells_last, n_ranks, rank - 1, plane_size, halo) if rank > 0 else None
        self.hi = layout(n_cells_last, n_ranks, rank + 1, plane_size, halo) if rank + 1 < n_ranks else None
        self.ps = plane_size
        self.group = group
        me = self.me
        own = me["owned_plane_end"] - me["owned_plane_begin"]
        for nb in (self.lo, self.hi):
            if nb is not None and own > 0:
                need = nb["ghost_planes_above"] if nb is self.lo else nb["ghost_planes_below"]
                if need > own:
                    raise ValueError("slab of rank %d (%d planes) thinner than the halo (%d)" % (rank, own, need))

    def _ops(self, local):
        import torch.distributed as dist

        me, ps = self.me, self.ps
        gb, ga = me["ghost_planes_below"], me["ghost_planes_above"]
        own = me["owned_plane_end"] - me["owned_plane_begin"]
        ops = []
        if self.lo is not None and own > 0:
            n_send = self.lo["ghost_planes_above"]  # my first planes -> their "above" ghosts
            ops.append(dist.P2POp(dist.isend, local[gb * ps:(gb + n_send) * ps], self.rank - 1, group=self.group))
            ops.append(dist.P2POp(dist.irecv, local[0:gb * ps], self.rank - 1, group=self.group))
        if self.hi is not None and own > 0:
            n_send = self.hi["ghost_planes_below"]  # my last planes -> their "below" ghosts
            e = (gb + own) * ps
            ops.append(dist.P2POp(dist.isend, local[e - n_send * ps:e], self.rank + 1, group=self.group))
            ops.append(dist.P2POp(dist.irecv, local[e:e + ga * ps], self.rank + 1, group=self.group))
        return ops

    def start(self, local):
        import torch.distributed as dist

        ops = self._ops(local)
        return dist.batch_isend_irecv(ops) if ops else []

    @staticmethod
    def finish(reqs):
        for r in reqs:
            r.wait()

    def exchange(self, local):
        self.finish(self.start(local))
        return local


def chunks(n, n_ranks):
    """Contiguous split of n items over n_ranks: [(begin, end)] per rank."""
    base, extra = divmod(n, n_ranks)
    out, b = [], 0
    for r in range(n_ranks):
        e = b + base + (1 if r < extra else 0)
        out.append((b, e))
        b = e
    return out


class DistributedMassSolve:
    """x = M^-1 r on a slab-partitioned mesh (replaces the CG + ILU/AMG solve of
    applications/advection/include/gdm/advection/problem.h:236-267 and
    applications/wave/include/gdm/wave/problem.h:457-502 across ranks).

    M^-1 = M_q^-1 (x) ... (x) M_0^-1 exactly (Kronecker form of the uncut mass
    matrix).  The directions inside a slab are solved in place; the
    partitioned direction q = dim - 1 is solved after a transpose: every rank
    sends the part of its owned planes that falls into each rank's chunk of
    the plane (contiguous entries of the lexicographic plane), so rank s ends
    up with all N_q planes of its chunk, solves those lines, and the inverse
    transpose restores the slab layout.  Point-to-point only (RCCL over xGMI
    for device tensors, gloo for the CPU tests).

    line_solve(axis, v, n_lines, stride, A, B, C) solves in place along
    `axis`; default: the operator's gdm_mass_solve_lines."""

    def __init__(self, dim, n_vertices, n_ranks, rank, op=None, line_solve=None, group=None):
        self.dim, self.N = dim, list(n_vertices) + [1] * (3 - dim)
        self.n_ranks, self.rank, self.group = n_ranks, rank, group
        q = dim - 1
        self.plane = 1
        for d in range(q):
            self.plane *= self.N[d]
        self.lays = [layout(self.N[q] - 1, n_ranks, r, self.plane, 0) for r in range(n_ranks)]
        self.chunk = chunks(self.plane, n_ranks)
        self.solve_lines = line_solve or (lambda *a: op.mass_solve_lines(*a))

    def _planes(self, r):
        L = self.lays[r]
        return L["owned_plane_end"] - L["owned_plane_begin"]

    def _local(self, x):
        """In-place solves along the directions inside the slab."""
        Nx, Ny = self.N[0], self.N[1]
        npl = self._planes(self.rank)
        if npl == 0:
            return
        if self.dim >= 2:  # x lines
            n = npl * (Ny if self.dim == 3 else 1)
            self.solve_lines(0, x, n, 1, n, 0, Nx)
        if self.dim == 3:  # y lines: (x, plane) -> base = plane * Nx * Ny + x
            self.solve_lines(1, x, Nx * npl, Nx, Nx, Nx * Ny, 1)

    def _exchange(self, send_of, recv_into):
        import torch.distributed as dist

        ops = []
        for s in range(self.n_ranks):
            if s == self.rank:
                continue
            b = send_of(s)
            if b is not None and b.numel():
                ops.append(dist.P2POp(dist.isend, b, s, group=self.group))
            c = recv_into(s)
            if c is not None and c.numel():
                ops.append(dist.P2POp(dist.irecv, c, s, group=self.group))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()

    def solve(self, rhs_owned, x_owned):
        import torch

        x = x_owned
        if x.data_ptr() != rhs_owned.data_ptr():
            x.copy_(rhs_owned)
        self._local(x)
        me, P = self.rank, self.plane
        c0, c1 = self.chunk[me]
        w = c1 - c0
        first = [L["owned_plane_begin"] for L in self.lays]
        npl = [self._planes(r) for r in range(self.n_ranks)]
        Nq = self.N[self.dim - 1]
        x2 = x.view(npl[me], P) if npl[me] else x.view(0, P)
        # forward transpose: Z[plane, chunk entry] for all planes of my chunk
        Z = torch.empty((Nq, w), dtype=x.dtype, device=x.device)
        sendbuf = {s: x2[:, self.chunk[s][0]:self.chunk[s][1]].contiguous() for s in range(self.n_ranks)}
        recvbuf = {s: torch.empty((npl[s], w), dtype=x.dtype, device=x.device) for s in range(self.n_ranks)}
        recvbuf[me] = sendbuf[me]
        self._exchange(lambda s: sendbuf[s], lambda s: recvbuf[s])
        for s in range(self.n_ranks):
            if npl[s]:
                Z[first[s]:first[s] + npl[s]] = recvbuf[s]
        if w:
            self.solve_lines(self.dim - 1, Z.view(-1), w, w, w, 0, 1)
        # inverse transpose
        back = {s: Z[first[s]:first[s] + npl[s]].contiguous() for s in range(self.n_ranks)}
        got = {s: torch.empty((npl[me], self.chunk[s][1] - self.chunk[s][0]), dtype=x.dtype, device=x.device)
               for s in range(self.n_ranks)}
        got[me] = back[me]
        self._exchange(lambda s: back[s], lambda s: got[s])
        for s in range(self.n_ranks):
            a, b = self.chunk[s]
            if npl[me] and b > a:
                x2[:, a:b] = got[s]
        return x


class SlabMassSolve:
    """x = M^-1 r across slab ranks by the SPIKE scheme of
    gdm_mass_solve_slab / gdm_mass_solve_interface (include/gdm_hip.h): the
    slab-local solve, one ghost-plane exchange (the same p planes as the
    stencil's update_ghost_values, advection/stiffness.h:343), `rounds`
    refinement rounds of one more exchange each for slabs too thin for the
    truncated interface systems (gdm_mass_spike_rounds; C4 at 8 ranks: one),
    and the interface correction.  Moves 2 p planes per rank and exchange,
    against the whole vector twice for DistributedMassSolve's transposes.

    `op` is the rank's GdmOperator (or any object with mass_solve_slab /
    mass_solve_interface[_round] / owned_view), `halo` its HaloExchange (None on
    one rank).  solve(rhs_owned, x_local) returns the owned view of x_local.
    `rounds` None asks gdm_mass_spike_rounds for the operator's mesh (the C
    ABI refuses an interface call whose rounds did not all run)."""

    def __init__(self, op, halo, rounds=None, ghosts=False):
        if rounds is None:
            from . import _capi

            rounds = _capi.mesh_spike_rounds(op.mesh)
        self.op, self.halo, self.rounds, self.ghosts = op, halo, int(rounds), bool(ghosts)

    def solve(self, rhs_owned, x_local):
        """ghosts=True: the ghost planes of x_local end up holding the
        neighbours' edge planes of the result (gdm_mass_solve_interface_ghosts).
        rhs_owned may be the owned view of x_local (in place)."""
        x_owned = self.op.owned_view(x_local)
        self.op.mass_solve_slab(rhs_owned, x_owned)
        if self.halo is not None:
            self.halo.exchange(x_local)
        for k in range(self.rounds):
            self.op.mass_solve_interface_round(x_local, k)
            if self.halo is not None:
                self.halo.exchange(x_local)
        if self.ghosts:
            self.op.mass_solve_interface_ghosts(x_local)
        else:
            self.op.mass_solve_interface(x_local)
        return x_owned


RK4_A = (0.5, 0.5, 1.0)  # a_{s+1,s}
RK4_B = (1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0)
RK4_C = (0.0, 0.5, 0.5, 1.0)


class SlabRK4:
    """The advection problem's RK4 step (advection/problem.h:62-94: per stage
    update_ghost_values + compute_rhs, stiffness.h:343-605, and the mass
    solve, problem.h:236-267) on z-slab ranks with the exact distributed mass
    inverse (SPIKE).  `ops` are rank operators evaluated in lockstep -- one per
    process over torch.distributed, or several in one process for the tests --
    and `exchange(vectors)` fills the ghost planes of each rank's local vector
    (HaloExchange.exchange for one rank per process).

    one_exchange=False: the reference's two exchanges per stage -- the stage
    vector's ghost planes before the stencil and the SPIKE planes of the solve.
    one_exchange=True: the SPIKE interface systems already give each rank the
    neighbours' edge planes of k (gdm_mass_solve_interface_ghosts), so k is a
    valid local vector; the low-storage updates acc = acc + h b_s k, Y = y +
    h a k and the last stage's y = acc + h b_3 k then run over the whole local
    vectors and keep the ghost planes of y, acc and Y current: the stage's
    stencil needs no exchange, one per stage remains (+ the refinement rounds
    of thin slabs).  The ghost planes then carry the neighbours' values as the
    interface solution gives them (<= 1e-15 relative apart from the owner's,
    the truncation of the interface systems); `resync` > 0 exchanges y's ghost
    planes every `resync` steps.  fused (one_exchange only): the interface
    correction and the stage update run as one launch
    (gdm_mass_solve_interface_rk), k is never stored -- the same bits.

    The inflow data of a built-in boundary function (fn_kind, fn_params) are
    computed by the engine per stage (gdm_apply_bc_fn); fn_kind None: no inflow
    data.  State: self.y[r] (local vectors); the owned values are
    ops[r].owned_view(self.y[r])."""

    def __init__(self, ops, exchange, fn_kind=None, fn_params=(), one_exchange=True, rounds=None, resync=0,
                 fused=True):
        from . import _capi

        self.ops, self.exchange = list(ops), exchange
        self.fn, self.prm = fn_kind, list(fn_params)
        self.one = bool(one_exchange)
        self.fused = self.one and bool(fused)
        self.rounds = _capi.mesh_spike_rounds(self.ops[0].mesh) if rounds is None else int(rounds)
        if self.rounds < 0:
            raise ValueError("SlabRK4: the partition is too thin for the SPIKE mass inverse")
        self.resync, self.steps = int(resync), 0
        self.y = [op.new_vector(True) for op in self.ops]
        self._acc = [op.new_vector(True) for op in self.ops]
        self._Y = [op.new_vector(True) for op in self.ops]
        self._k = [op.new_vector(True) for op in self.ops]

    def set_solution(self, owned_values):
        """owned_values[r]: rank r's owned DoF values; the ghost planes are
        exchanged once"""
        for op, y, v in zip(self.ops, self.y, owned_values):
            y.zero_()
            op.owned_view(y).copy_(v)
        self.exchange(self.y)

    def _rhs(self, t, h, s, stage):
        for op, src, k in zip(self.ops, stage, self._k):
            dst = op.owned_view(k)
            if self.fn is None:
                op.apply(src, dst)
            else:
                alpha, t_k = (0.0, t) if s == 0 else (h * RK4_A[s - 1], t + RK4_C[s - 1] * h)
                op.apply_bc_fn(src, dst, self.fn, self.prm, t, alpha, t_k)
        for op, k in zip(self.ops, self._k):
            own = op.owned_view(k)
            op.mass_solve_slab(own, own)
        self.exchange(self._k)
        for rnd in range(self.rounds):
            for op, k in zip(self.ops, self._k):
                op.mass_solve_interface_round(k, rnd)
            self.exchange(self._k)
        if self.fused:
            return
        for op, k in zip(self.ops, self._k):
            if self.one:
                op.mass_solve_interface_ghosts(k)
            else:
                op.mass_solve_interface(k)

    def step(self, t, h):
        stage = self.y
        for s in range(4):
            if not self.one:
                self.exchange(stage)  # update_ghost_values of the stage vector (stiffness.h:343)
            self._rhs(t, h, s, stage)
            last = s == 3
            for op, k, y, acc, Y in zip(self.ops, self._k, self.y, self._acc, self._Y):
                if self.fused and last:
                    op.mass_solve_interface_rk(k, h * RK4_B[s], acc, y)
                elif self.fused:
                    op.mass_solve_interface_rk(k, h * RK4_B[s], y if s == 0 else acc, acc, h * RK4_A[s], y, Y)
                elif last:
                    op.rk_update(h * RK4_B[s], k, acc, y)
                else:
                    op.rk_update(h * RK4_B[s], k, y if s == 0 else acc, acc, h * RK4_A[s], y, Y)
            stage = self._Y
        self.steps += 1
        if self.one and self.resync > 0 and self.steps % self.resync == 0:
            self.exchange(self.y)


SPIKE_TOL = 1e-15


def make_mass_solver(op, halo, dim, p, n_subdivisions, n_ranks, rank, lo=0.0, hi=1.0, group=None):
    """The distributed exact mass inverse for this partition: SlabMassSolve
    (with the refinement rounds gdm_mass_spike_rounds asks for), else -- a
    slab thinner than 2p planes -- the transposes of DistributedMassSolve.
    Both expose solve(rhs_owned, x_local) -> owned."""
    from . import _capi

    rounds = _capi.mass_spike_rounds(dim, p, n_subdivisions, n_ranks, lo, hi)
    if rounds >= 0:
        return SlabMassSolve(op, halo, rounds)
    ns = list(n_subdivisions) if hasattr(n_subdivisions, "__len__") else [n_subdivisions] * dim
    ds = DistributedMassSolve(dim, [n + 1 for n in ns[:dim]], n_ranks, rank, op=op, group=group)

    class _Transposed:
        def solve(self, rhs_owned, x_local):
            x_owned = op.owned_view(x_local)
            return ds.solve(rhs_owned, x_owned)

    return _Transposed()


def apply_overlapped(op, halo, src_local, dst_owned, bc_values=None):
    """compute_rhs of one slab with the ghost-plane exchange overlapped: the
    output planes whose 2p+1 input planes are all owned are computed while the
    exchange (update_ghost_values, advection/stiffness.h:343) is in flight, the
    p planes next to each slab edge after it (gdm_apply_planes), then the inflow
    boundary data.  `halo` may be None (single rank)."""
    L = op.layout
    p = L["halo_depth"]
    pb, pe = L["owned_plane_begin"], L["owned_plane_end"]
    lo = pb + (p if L["ghost_planes_below"] else 0)
    hi = pe - (p if L["ghost_planes_above"] else 0)
    reqs = halo.start(src_local) if halo is not None else []
    if hi > lo:
        op.apply_planes(src_local, dst_owned, lo, hi)
    if halo is not None:
        halo.finish(reqs)
    if hi <= lo:
        op.apply_planes(src_local, dst_owned, pb, pe)
    elif lo > pb or pe > hi:
        # both edge ranges in one launch (gdm_apply_planes2)
        op.apply_planes2(src_local, dst_owned, pb, lo, hi, pe)
    if bc_values is not None:
        op.add_boundary_data(bc_values, dst_owned)
    return dst_owned
