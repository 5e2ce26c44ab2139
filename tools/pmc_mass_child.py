#!/usr/bin/env python3
"""PMC child for the C3 mass inverse (tools/pmc_mass.sh): one plain exact
inverse (gdm_mass_solve: z, y, x passes) and one with the RK stage update fused
into the x pass (gdm_mass_solve_rk, RKM 2: acc_in, y in; acc, Y out)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

import torch  # noqa: E402

import gdm_amd  # noqa: E402

op = gdm_amd.GdmOperator(3, 5, 511, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05))
g = torch.Generator(device="cuda").manual_seed(3)
r = torch.rand(op.n_owned, dtype=torch.float64, device="cuda", generator=g)
x = op.new_vector(False)
op.mass_solve(r, x)
acc, y, Y = torch.rand_like(r), torch.rand_like(r), torch.empty_like(r)
op.mass_solve_rk(r, 0.1, acc, acc, 0.05, y, Y)
torch.cuda.synchronize()
