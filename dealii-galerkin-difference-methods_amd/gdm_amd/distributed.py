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
