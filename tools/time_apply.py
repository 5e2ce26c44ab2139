#!/usr/bin/env python3
"""Timing only (no parity) of compute_rhs without inflow data at C3 for the
libraries given as arguments (variant names under lib/ab, "main" = the
in-tree build), each in a child process.  Experiment tool for builds whose
results are wrong by design (phase-disable / role-only experiments).

    python tools/time_apply.py main onlycons onlyprod
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = os.path.join(ROOT, "dealii-galerkin-difference-methods_amd", "lib", "ab")
CHILD = r'''
import sys, torch
sys.path.insert(0, %r)
from gdm_amd import GdmOperator
n, p = %d, %d
op = GdmOperator(3, p, n, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05), device=0)
src = torch.rand(op.n_local, dtype=torch.float64, device="cuda")
dst = op.new_vector(local=False)
op.time_op(0, src, dst, None, 3)
print(min(op.time_op(0, src, dst, None, 20) for _ in range(3)))
'''


def main():
    n = int(os.environ.get("N", "511"))
    p = int(os.environ.get("P", "5"))
    for name in sys.argv[1:]:
        env = dict(os.environ)
        if name != "main":
            env["GDM_HIP_LIB"] = os.path.join(V, name, "libgdm_hip.so")
        r = subprocess.run([sys.executable, "-c", CHILD % (os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"), n, p)],
                           env=env, capture_output=True, text=True, timeout=240)
        if r.returncode != 0:
            print(json.dumps({"lib": name, "rc": r.returncode, "err": r.stderr[-400:]}), flush=True)
            if r.returncode < 0 or r.returncode > 1:
                sys.exit(r.returncode if r.returncode > 0 else 2)
            continue
        ms = float(r.stdout.strip().splitlines()[-1])
        print(json.dumps({"lib": name, "n": n, "p": p, "ms": ms, "frac": 16 * (n + 1) ** 3 / ms / 1e9 / 8000}),
              flush=True)


if __name__ == "__main__":
    main()
