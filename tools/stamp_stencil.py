#!/usr/bin/env python3
"""Where the fused stencil's waves spend a plane: s_memtime stamps of the
stamp build (tools/build_variant.sh stamp -DGDM_STAMP) at the phase
boundaries of planes 40..63 of every workgroup of the C3 interior launch.
Experiment tool, not product code; read the SHARES, not the absolute time
(the stamps' lgkmcnt waits change the kernel).

    GDM_HIP_LIB=.../lib/variants/stamp/libgdm_hip.so python tools/stamp_stencil.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

NI, NW, NS = 24, 16, 8
PROD = ["dma_wait", "xsweep+write", "dma_issue", "barrier"]
CONS = ["barrier", "ysweep", "z", "store+retire"]


def main():
    import torch
    from gdm_amd import GdmOperator

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 511
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    kind = sys.argv[3] if len(sys.argv) > 3 else "advection"
    op = GdmOperator(3, p, n, 0.0, 1.0, kind, params=(1.0, 0.15, -0.05) if kind == "advection" else (), device=0)
    src = torch.rand(op.n_local, dtype=torch.float64, device="cuda")
    dst = op.new_vector(local=False)
    nwg = 512
    st = torch.zeros(nwg * NI * NW * NS, dtype=torch.int64, device="cuda")
    for _ in range(3):
        op.apply(src, dst)
    torch.cuda.synchronize()
    os.environ["GDM_STAMP_PTR"] = str(st.data_ptr())
    op.apply(src, dst)
    torch.cuda.synchronize()
    del os.environ["GDM_STAMP_PTR"]
    S = st.cpu().numpy().reshape(nwg, NI, NW, NS).astype(np.float64)
    used = np.flatnonzero(S[:, :, 0, 0].min(axis=1) > 0)
    S = S[used]
    if os.environ.get("STAMP_V9"):
        # v9: every wave: 0 before B_i, 1 after, 2 after Y, 3 after Z, 4 after the stores, 5 after X(i+1)
        names = ["barrier", "ysweep", "z", "store", "xsweep"]
        d = {names[k]: float(np.median(S[:, :, :, k + 1] - S[:, :, :, k])) for k in range(5)}
        d["gap_to_next"] = float(np.median(S[:, 1:, :, 0] - S[:, :-1, :, 5]))
        per = np.diff(S[:, :, 0, 1], axis=1)
        out = {"workgroups": int(len(used)), "period_ticks_median": float(np.median(per)), "median_ticks": d,
               "barrier_by_wave": [float(np.median(S[:, :, w, 1] - S[:, :, w, 0])) for w in range(16)],
               "x_by_wave": [float(np.median(S[:, :, w, 5] - S[:, :, w, 4])) for w in range(16)],
               "yz_by_wave": [float(np.median(S[:, :, w, 3] - S[:, :, w, 1])) for w in range(16)]}
        print(json.dumps(out, indent=1))
        return
    prod, cons = S[:, :, :8, :], S[:, :, 8:, :]
    # plane period: producer barrier exits of consecutive planes
    per = np.diff(prod[:, :, :, 4], axis=1)
    out = {"workgroups": int(len(used)), "period_ticks_median": float(np.median(per))}
    pd = {PROD[k]: float(np.median(prod[:, :, :, k + 1] - prod[:, :, :, k])) for k in range(4)}
    cd = {CONS[k]: float(np.median(cons[:, :, :, k + 1] - cons[:, :, :, k])) for k in range(4)}
    cd["gap_to_next"] = float(np.median(cons[:, 1:, :, 0] - cons[:, :-1, :, 4]))
    pd["loop_to_next"] = float(np.median(prod[:, 1:, :, 0] - prod[:, :-1, :, 4]))
    out["producer_median_ticks"] = pd
    out["consumer_median_ticks"] = cd
    # per producer wave (waves 0-2 own two row groups at p = 5)
    out["producer_xsweep_by_wave"] = [float(np.median(prod[:, :, w, 2] - prod[:, :, w, 1])) for w in range(8)]
    out["producer_barrier_by_wave"] = [float(np.median(prod[:, :, w, 4] - prod[:, :, w, 3])) for w in range(8)]
    # who arrives last at the barrier: the last arrival's role
    arr_p = prod[:, :, :, 3].max(axis=2)
    arr_c = cons[:, :, :, 0].max(axis=2)
    out["last_arrival_consumer_frac"] = float(np.mean(arr_c > arr_p))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
