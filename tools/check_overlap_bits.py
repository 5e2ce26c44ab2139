#!/usr/bin/env python3
"""Bitwise comparison of gdm_apply (one call) with gdm_apply_planes over the
overlapped ranges + gdm_add_boundary_data on one slab rank: reports the
planes where the two differ.  Debug tool."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))


def main():
    import torch
    import gdm_amd
    from gdm_amd.distributed import apply_overlapped

    for (p, n, R, r) in [(5, 30, 2, 0), (5, 30, 2, 1), (3, 20, 3, 1), (5, 14, 2, 0), (5, 60, 2, 1)]:
        op = gdm_amd.GdmOperator(3, p, n, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05), n_ranks=R, rank=r)
        L = op.layout
        g = torch.Generator(device="cuda").manual_seed(1)
        u = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=g)
        bc = torch.rand(max(op.n_bc_points, 1), dtype=torch.float64, device="cuda", generator=g)
        a = op.new_vector(local=False)
        b = op.new_vector(local=False)
        c = op.new_vector(local=False)
        op.apply(u, a, bc if op.n_bc_points else None)
        apply_overlapped(op, None, u, b, bc if op.n_bc_points else None)
        op.apply_planes(u, c, L["owned_plane_begin"], L["owned_plane_end"])
        if op.n_bc_points:
            op.add_boundary_data(bc, c)
        # without boundary data, and the boundary data alone (u = 0)
        a0, c0 = op.new_vector(local=False), op.new_vector(local=False)
        op.apply(u, a0)
        op.apply_planes(u, c0, L["owned_plane_begin"], L["owned_plane_end"])
        z = torch.zeros_like(u)
        a1, c1 = op.new_vector(local=False), op.new_vector(local=False)
        if op.n_bc_points:
            op.apply(z, a1, bc)
            op.apply_planes(z, c1, L["owned_plane_begin"], L["owned_plane_end"])
            op.add_boundary_data(bc, c1)
        torch.cuda.synchronize()
        print("  stencil only: %d entries differ; bc only: %d entries differ (max |d| %.3g)" % (
            int((a0 != c0).sum()), int((a1 != c1).sum()), float((a1 - c1).abs().max())), flush=True)
        ps = L["plane_size"]
        for name, x in (("overlapped", b), ("one range", c)):
            d = (a != x).cpu().numpy().reshape(-1, ps)
            bad = np.flatnonzero(d.any(axis=1)) + L["owned_plane_begin"]
            print("p=%d n=%d rank %d/%d %s: %d planes differ %s" % (p, n, r, R, name, len(bad), bad[:12].tolist()),
                  flush=True)


if __name__ == "__main__":
    main()
