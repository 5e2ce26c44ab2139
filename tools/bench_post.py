"""Time gdm_error_norms (device postprocess) at C3 size: 3D p=5, 511^3 cells
(512^3 DoFs), sine-product exact solution.  Algorithmic traffic: 8 B/DoF."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dealii-galerkin-difference-methods_amd"))
import numpy as np
import torch
import gdm_amd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 511
p = int(sys.argv[2]) if len(sys.argv) > 2 else 5
op = gdm_amd.GdmOperator(3, p, n, 0.0, 1.0, "mass")
x = torch.linspace(0.0, 1.0, n + 1, dtype=torch.float64, device="cuda")
u = (torch.sin(2 * np.pi * x + 0.2)[:, None, None] * torch.sin(2 * np.pi * x + 0.1)[None, :, None]
     * torch.sin(2 * np.pi * x + 0.3)[None, None, :]).reshape(-1).contiguous()
prm = [0.0, 0.0, 0.0, 1.0, 1.0, 1.0, 0.3, 0.1, 0.2]
e = op.error_norms(u, 2, prm, 0.0)
torch.cuda.synchronize()
t0 = time.perf_counter()
K = 10
for _ in range(K):
    e = op.error_norms(u, 2, prm, 0.0)
dt = (time.perf_counter() - t0) / K
print("error_norms n=%d p=%d: %.3f ms/call (incl. D2H sync), %.2f GB/s algorithmic, norms %s"
      % (n, p, dt * 1e3, u.numel() * 8 / dt / 1e9, e))
