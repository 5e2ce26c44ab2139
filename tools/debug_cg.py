"""Debug aid: device SolverCG (gdm_csr_cg) vs a numpy CG on the failing
test_cg_vs_oracle systems, with GDM_CG_TRACE per-iteration invariants."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dealii-galerkin-difference-methods_amd")]
os.environ["GDM_CG_TRACE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from gdm_amd import sparse  # noqa: E402


def host_cg(rp, c, v, b, pc, n_it):
    import scipy.sparse as sp

    A = sp.csr_matrix((v, c, rp))
    dinv = 1.0 / A.diagonal() if pc else np.ones(len(b))
    x = np.zeros_like(b)
    r = b.copy()
    p = None
    gh_old = None
    for it in range(1, n_it + 1):
        z = dinv * r
        gh = r @ z
        p = z.copy() if it == 1 else z + gh / gh_old * p
        gh_old = gh
        q = A @ p
        pap = p @ q
        al = gh / pap
        x += al * p
        r -= al * q
        print("[host-cg ] it %d  rr %.6e gh %.6e pap %.6e alpha %.6e" % (it, r @ r, gh, pap, al))


for dim, p, n, pc, kind in [(1, 3, 64, 0, "lap_mass"), (1, 3, 64, 1, "mass"), (2, 5, 12, 0, "mass")]:
    m = O.Mesh(dim, p, n, 0.0, 1.0)
    b = np.random.default_rng(3).uniform(-1, 1, m.n_dofs)
    rp, c, v = m.matrix_csr(0)
    if kind == "lap_mass":
        v = v + m.matrix_csr(1)[2]
    tol = (1e-20, 1e-14) if kind == "mass" else (1e-10, 1e-6)
    x_ref, its_ref = O.cg(rp, c, v, b, precond=pc, max_it=5000, abs_tol=tol[0], rel_tol=tol[1])
    print("=== case", dim, p, n, "precond", pc, kind, "oracle its", its_ref, flush=True)
    host_cg(rp, c, v, b, pc, 6)
    for rep in range(3):
        A = sparse.SparseMatrix(rp, c.astype(np.uint32), v)
        x = torch.zeros(m.n_dofs, dtype=torch.float64, device="cuda")
        bd = torch.from_numpy(b).cuda()
        try:
            its, res = sparse.solve_cg(A, x, bd, preconditioner=["identity", "jacobi"][pc], max_it=60,
                                       abs_tol=tol[0], rel_tol=tol[1])
        except Exception as e:  # noqa: BLE001
            its, res = -1, str(e)
        print("--- rep", rep, "device its", its, "res", res, flush=True)
        A.close()
