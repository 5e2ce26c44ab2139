#!/usr/bin/env python3
"""Stencil phase breakdown on the GPU: times the fused kernel with phases
disabled through the diagnostic build (make -C .../csrc diag; GDM_DBG bits:
1 consumer y-sweep, 2 consumer z-scatter, 4 producer x-sweep, 8 producer DMA,
16 barriers, 32 consumer global stores, 64 producer (A, B) LDS writes).  Results are wrong by design; timing only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GDM_HIP_LIB", os.path.join(ROOT, "dealii-galerkin-difference-methods_amd", "lib", "diag", "libgdm_hip.so"))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))
import torch  # noqa: E402
from gdm_amd import GdmOperator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 511
p = int(sys.argv[2]) if len(sys.argv) > 2 else 5
kind = sys.argv[3] if len(sys.argv) > 3 else "advection"
op = GdmOperator(3, p, n, 0.0, 1.0, kind, params=(1.0, 0.15, -0.05) if kind == "advection" else (), device=0)
src = torch.rand(op.n_local, dtype=torch.float64, device="cuda")
dst = op.new_vector(local=False)
BITS = [int(b) for b in os.environ.get("GDM_DIAG_BITS", "0,1,2,3,4,8,12,15,16,19,28,31").split(",")]
for bits in BITS:
    os.environ["GDM_DBG"] = str(bits)
    op.time_op(0, src, dst, None, 3)
    ms = op.time_op(0, src, dst, None, 10)
    print("dbg=%2d  %.3f ms  (%.0f GB/s algorithmic)" % (bits, ms, 16 * op.n_local / ms / 1e6), flush=True)
