#!/usr/bin/env python3
"""Config 5 with the reference's cut-cell values: the
2D p=3 cut Poisson system of prototypes/cut_poisson_01_gdm.cc on 4095^2 cells
(16.8 M DoFs) assembled by the library (gdm_amd.CutPoisson, host C++), moved
to HBM, then on the device: SpMV time (HIP events), one SpMV against the host
CSR product (oracle/gdm_oracle.c, test infrastructure), and a bounded
SolverCG run (identity, ReductionControl(max_it, 1e-10, 1e-6)) -- the
reference's iteration count at this size is O(10^4), so the run is capped
and reports the residual reduction reached and the time per iteration.
One JSON line on stdout.

    python tools/bench_cut_c5.py [--n 4095] [--max-it 1000] [--gp 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4095)
    ap.add_argument("--max-it", type=int, default=1000)
    ap.add_argument("--gp", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    import torch

    import gdm_amd
    import oracle as O

    t0 = time.time()
    S = gdm_amd.CutPoisson(3, a.n, ghost_penalty=bool(a.gp))
    t_asm = time.time() - t0
    A = S.matrix()
    b_h = S.rhs()
    b = torch.from_numpy(b_h).cuda()
    x = torch.zeros(S.n_rows, dtype=torch.float64, device="cuda")
    y = torch.zeros_like(x)
    u_h = np.random.default_rng(7).uniform(-1, 1, S.n_rows)
    u = torch.from_numpy(u_h).cuda()
    ms = A.time_vmult(y, u, 20)
    A.vmult(y, u)
    rp, c, v = S.csr()
    ref = O.csr_vmult(rp, c.astype(np.int64), v, u_h)
    spmv_rel = float(np.linalg.norm(y.cpu().numpy() - ref) / np.linalg.norm(ref))
    del rp, c, v, ref
    torch.cuda.synchronize()
    t1 = time.time()
    try:
        its, res = gdm_amd.solve_cg(A, x, b, "identity", a.max_it, 1e-10, 1e-6)
        conv = True
    except gdm_amd.GdmError:
        its, res, conv = a.max_it, float("nan"), False
    torch.cuda.synchronize()
    t_cg = time.time() - t1
    r = b - 0
    A.vmult(y, x)
    res_true = float(torch.linalg.norm(b - y)) / float(torch.linalg.norm(b))
    bytes_spmv = S.nnz * 12 + S.n_rows * 20
    print(json.dumps({"config": "C5 cut", "n_sub": a.n, "ghost_penalty": bool(a.gp), "n_rows": S.n_rows,
                      "nnz": S.nnz, "inside_cells": S.n_inside_cells, "intersected_cells": S.n_intersected_cells,
                      "assembly_s": t_asm, "spmv_ms": ms, "spmv_GBps": bytes_spmv / ms / 1e6,
                      "spmv_rel_vs_host": spmv_rel, "cg_its": its, "cg_converged": conv,
                      "cg_ms_per_it": t_cg * 1e3 / max(its, 1), "rel_residual": res_true,
                      "l2_error": S.l2_error(x) if conv else None}))


if __name__ == "__main__":
    main()
