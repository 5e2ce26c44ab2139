#!/usr/bin/env python3
"""Per-operator timings of the device engine at the BASELINE configs
(HIP events around back-to-back applications on the operator's stream):

  C3  3D advection p=5, 512^3 DoFs: compute_rhs (stencil + inflow faces), mass solve
  C4  3D wave p=7, 256^3 DoFs:       compute_rhs, mass solve
  C2  2D advection p=5, 1024^2 DoFs: compute_rhs, mass solve

Algorithmic bytes: 16 B per DoF and application (read once, write once).
One JSON line per (config, operator) on stdout.

    python tools/bench_ops.py [--configs C3,C4,C2] [--iters 10] [--ops apply,mass_solve,rk_step]

rk_step: one device-resident RK4 step (gdm_amd.problem: 4 x (compute_rhs +
mass solve) + fused stage updates); C4 = the wave-rk stage of BASELINE C4.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

CONFIGS = {
    "C3": dict(dim=3, p=5, n=511, kind="advection", params=(1.0, 0.15, -0.05), lo=0.0, hi=1.0),
    "C4": dict(dim=3, p=7, n=255, kind="wave", params=(), lo=-1.21, hi=1.21),
    "C2": dict(dim=2, p=5, n=1023, kind="advection", params=(2 * 0.9063077870366499, 2 * 0.42261826174069944),
               lo=0.0, hi=1.0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3,C4,C2")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ops", default="apply,mass_solve")
    args = ap.parse_args()
    import torch
    from gdm_amd import GdmOperator

    for name in args.configs.split(","):
        c = CONFIGS[name]
        op = GdmOperator(c["dim"], c["p"], c["n"], c["lo"], c["hi"], c["kind"], params=c["params"], device=0)
        gen = torch.Generator(device="cuda").manual_seed(20251010)
        src = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
        dst = op.new_vector(local=False)
        bc = None
        if c["kind"] == "advection" and op.n_bc_points > 0:
            bc = torch.rand(op.n_bc_points, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
        n = op.n_owned
        for which, opname in ((0, "apply"), (2, "mass_solve")):
            if opname not in args.ops.split(","):
                continue
            op.time_op(which, src, dst, bc if which == 0 else None, 2)
            ms = op.time_op(which, src, dst, bc if which == 0 else None, args.iters)
            gbs = 16.0 * n / (ms * 1e-3) / 1e9
            print(json.dumps({"config": name, "op": opname, "kind": c["kind"], "dim": c["dim"], "p": c["p"],
                              "n_dofs": n, "ms": ms, "dof_per_s": n / (ms * 1e-3), "alg_GBps": gbs,
                              "frac_8TBps": gbs / 8000.0}), flush=True)
        if "rk_step" in args.ops.split(","):
            # one full RK4 step (4 x (compute_rhs + mass solve) + the fused stage updates), device-resident
            from gdm_amd import AdvectionProblem, WaveProblem

            if c["kind"] == "wave":
                prob = WaveProblem(op)
                prob.u.copy_(src[:n])
            else:
                prob = AdvectionProblem(op, op.FN_SINE_PRODUCT, [1.0, 0.15, -0.05, 1.0, 1.0, 1.0, 0.3, 0.0, 0.7])
                prob.u.copy_(src[:n])
            dt = 1e-4
            for _ in range(2):
                prob.step(0.0, dt)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(args.iters):
                prob.step(i * dt, dt)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            print(json.dumps({"config": name, "op": "rk_step", "kind": c["kind"], "dim": c["dim"], "p": c["p"],
                              "n_dofs": n, "ms": ms, "stage_ms": ms / 4, "dof_updates_per_s": 4 * n / (ms * 1e-3)}),
                  flush=True)
            del prob
        del op, src, dst, bc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
