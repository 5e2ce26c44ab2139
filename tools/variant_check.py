#!/usr/bin/env python3
"""Parity + timing of one stencil build (GDM_HIP_LIB selects a variant):
the v8 stencil on wall-touching 3D meshes against the oracle's Kronecker form
(the smoke test's check, any p / kind), then the timing of compute_rhs at a
BASELINE config.  Experiment tool, not product code.

    GDM_HIP_LIB=... python tools/variant_check.py --p 5 --kind advection --config C3
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=5)
    ap.add_argument("--kind", default="advection")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch
    import gdm_amd
    import oracle as O

    p = args.p
    a = (1.0, 0.15, -0.05) if args.kind == "advection" else ()
    rng = np.random.default_rng(0)
    worst = 0.0
    for n3 in ((90, 50, 40), (140, 75, 60)):
        op = gdm_amd.GdmOperator(3, p, n3, 0.0, 1.0, args.kind, params=a, device=0)
        m = O.Mesh(3, p, list(n3))
        u = rng.uniform(-1, 1, m.n_dofs)
        M = [m.matrices_1d(d)[0] for d in range(3)]
        if args.kind == "advection":
            B = [m.advection_outflow_B(d, a[d]) for d in range(3)]
        else:
            B = [-m.matrices_1d(d)[2] for d in range(3)]
        ref = m.kron_apply([(B[0], M[1], M[2]), (M[0], B[1], M[2]), (M[0], M[1], B[2])], u)
        y = op.new_vector(local=False)
        op.apply(torch.from_numpy(u).cuda(), y)
        torch.cuda.synchronize()
        err = float(np.linalg.norm(y.cpu().numpy() - ref) / np.linalg.norm(ref))
        worst = max(worst, err)
    ok = worst < 1e-12
    out = {"lib": os.environ.get("GDM_HIP_LIB", "main"), "p": p, "kind": args.kind, "parity_rel_err": worst,
           "parity_ok": ok}
    if ok:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_ops.py"), "--configs", args.config,
                            "--ops", "apply", "--iters", str(args.iters)], capture_output=True, text=True,
                           timeout=300)
        for line in r.stdout.splitlines():
            d = json.loads(line)
            out["ms"] = d["ms"]
            out["frac"] = d.get("frac_8TBps")
    print(json.dumps(out), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
