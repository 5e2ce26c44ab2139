"""One C3 advection RK4 step (4 stages) under rocprofv3: which kernels a stage
launches and how long each takes (bench.py's rk4_stage_ms breakdown).
    rocprofv3 --kernel-trace --stats -d DIR -o ps --output-format csv -- python tools/profile_stage.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

import torch  # noqa: E402

import gdm_amd  # noqa: E402
from gdm_amd import AdvectionProblem  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 511
op = gdm_amd.GdmOperator(3, 5, n, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05))
prob = AdvectionProblem(op, op.FN_SINE_PRODUCT, [1.0, 0.15, -0.05, 1.0, 1.0, 1.0, 0.3, 0.0, 0.7])
g = torch.Generator(device="cuda").manual_seed(1)
prob.u.copy_(torch.rand(prob.u.numel(), dtype=torch.float64, device="cuda", generator=g))
prob.step(0.0, 1e-4)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(3):
    prob.step(i * 1e-4, 1e-4)
torch.cuda.synchronize()
print("stage_ms %.4f" % ((time.perf_counter() - t0) * 1e3 / 12))
