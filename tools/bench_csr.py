#!/usr/bin/env python3
"""Config 5 matvec benchmark: device CSR SpMV and CG on the
full structural stencil of a 2D p=3 GDM matrix on 4096^2 vertices
(16.8 M rows, 823 M stored entries; prototypes/cut_poisson_01_gdm.cc:148-335
sparsity, system.h:586-599).  Values are a synthetic SPD Kronecker sum
(the cut quadrature that would produce the real values is out of scope);
SpMV cost depends on the structure only.

Algorithmic bytes per SpMV: 12 B per stored entry (u32 column + f64 value)
+ 24 B per row (int64 row pointer, x read once, y written once).
One JSON line on stdout.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))


def main():
    import numpy as np
    import torch
    from gdm_amd import sparse as sp

    n = int(os.environ.get("GDM_CSR_N", "4096"))
    p = 3
    m = np.array([1.0, 4.0, 9.0, 16.0, 9.0, 4.0, 1.0])
    lap = -np.ones(2 * p + 1)
    lap[p] = 2 * p + 1.0
    rp, ci, v = sp.stencil_csr_2d(n, p, [(lap, m), (m, lap)])
    A = sp.SparseMatrix(rp, ci, v)
    del rp, ci, v
    torch.cuda.empty_cache()
    rows, nnz = A.m(), A.n_nonzero_elements()
    gen = torch.Generator(device="cuda").manual_seed(20251010)
    x = torch.rand(rows, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    y = torch.empty_like(x)
    A.time_vmult(y, x, 3)
    ms = A.time_vmult(y, x, int(os.environ.get("GDM_CSR_ITERS", "20")))
    alg = 12.0 * nnz + 24.0 * rows
    b = torch.rand(rows, dtype=torch.float64, device="cuda", generator=gen)
    xs = torch.zeros_like(b)
    torch.cuda.synchronize()
    import time

    # SolverCG + PreconditionIdentity with the prototype's ReductionControl
    # (n, 1e-10, 1e-6) (cut_poisson_01_gdm.cc:332-335) on the synthetic system
    t0 = time.perf_counter()
    its, res = sp.solve_cg(A, xs, b, "identity", max_it=rows, abs_tol=1e-10, rel_tol=1e-6)
    torch.cuda.synchronize()
    cg_s = time.perf_counter() - t0
    r = torch.empty_like(b)
    A.vmult(r, xs)
    true_res = float(torch.linalg.norm(b - r))
    b_norm = float(torch.linalg.norm(b))
    out = {
        "metric": "CSR vmult (cut-Poisson CG matvec, config 5)",
        "n_rows": rows, "nnz": nnz, "lanes": os.environ.get("GDM_CSR_LANES", "auto"),
        "spmv_ms": ms, "rows_per_s": rows / (ms * 1e-3),
        "roofline": {"bound": "hbm", "achieved": alg / (ms * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": alg / (ms * 1e-3) / 1e9 / 8000.0, "algorithmic_bytes_per_launch": alg},
        "cg": {"iterations": its, "residual": res, "true_residual": true_res, "rhs_norm": b_norm, "seconds": cg_s,
               "ms_per_iteration": cg_s * 1e3 / max(its, 1),
               "setup": "SolverCG + PreconditionIdentity, ReductionControl(n, 1e-10, 1e-6) "
                        "(cut_poisson_01_gdm.cc:332-335), x0 = 0"},
        "data": "synthetic SPD Kronecker-sum values on the full structural stencil",
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
