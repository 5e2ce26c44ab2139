"""One process per rank (the reference's MPI model, advection-app.cc:160):
the C++ host mirror's MPI communicator (gdm/hip/mpi_communicator.h).

CPU: mpirun -np 2..4 of mpi_exchange_test -- the ghost-plane message pattern
over the gdm_halo_plan ranges on host buffers (every received entry holds
the global index of the vertex it stands for) and the MPI sum / max
reductions; no GPU involved.
GPU: advection_app_mpi under mpirun -np 2, 3 (MpiRank: host staging; all
ranks on the box's one GPU) reproduces the single-rank advection_app run
(rel 1e-10, exact SPIKE or Jacobi-CG mass solve as advection_app picks), and
the RCCL communicator (RcclRank) runs at one rank (RCCL admits one rank per
GPU; the 8-GPU exchange is unmeasured until an 8-GPU node runs it)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "dealii-galerkin-difference-methods_amd", "lib", "host")
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
HAVE_MPI = os.path.exists(MPIRUN) and os.path.exists(os.path.join(HOST, "mpi_exchange_test"))


def _mpirun(n, args, timeout=120):
    env = dict(os.environ, HYDRA_LAUNCHER="fork")
    return subprocess.run([MPIRUN, "-np", str(n)] + args, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.skipif(not HAVE_MPI, reason="MPI runtime or the MPI host programs missing")
@pytest.mark.parametrize("np_,dim,p,n", [(2, 3, 5, 40), (3, 3, 5, 40), (3, 2, 3, 31), (4, 1, 7, 120),
                                          (2, 3, 7, 15)])
def test_mpi_exchange_pattern(np_, dim, p, n):
    r = _mpirun(np_, [os.path.join(HOST, "mpi_exchange_test"), str(dim), str(p), str(n)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1] == "ok"


@pytest.mark.gpu
@pytest.mark.skipif(not HAVE_MPI, reason="MPI runtime or the MPI host programs missing")
@pytest.mark.parametrize("dim,p,n,steps,np_", [(3, 5, 14, 2, 2), (2, 5, 240, 2, 3), (2, 5, 30, 2, 2),
                                               (3, 3, 20, 2, 3)])
def test_mpi_driver_matches_single_rank(tmp_path, dim, p, n, steps, np_):
    out1, outn = tmp_path / "u1.bin", tmp_path / "un.bin"
    r1 = subprocess.run([os.path.join(HOST, "advection_app"), str(dim), str(p), str(n), str(steps), "0.1", str(out1),
                         "0", "1", "1"], capture_output=True, text=True, timeout=120)
    assert r1.returncode == 0, r1.stderr
    r = _mpirun(np_, [os.path.join(HOST, "advection_app_mpi"), str(dim), str(p), str(n), str(steps), "0.1", str(outn),
                      "1", "mpi"], timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    u1, un = np.fromfile(out1, dtype=np.float64), np.fromfile(outn, dtype=np.float64)
    assert u1.shape == un.shape
    assert np.linalg.norm(un - u1) / np.linalg.norm(u1) < 1e-10
    e1 = [float(v) for v in r1.stdout.strip().splitlines()[-1].split()[2:]]
    en = [float(v) for v in r.stdout.strip().splitlines()[-1].split()[2:]]
    np.testing.assert_allclose(en, e1, rtol=1e-7)


@pytest.mark.gpu
@pytest.mark.skipif(not HAVE_MPI, reason="MPI runtime or the MPI host programs missing")
@pytest.mark.parametrize("dim,p,n,np_", [(3, 5, 30, 2), (3, 3, 20, 3), (3, 5, 14, 2)])
def test_overlapped_exchange_bitwise_equals_blocking(tmp_path, dim, p, n, np_):
    """compute_rhs_overlapped (interior planes while MpiRank's messages are in
    flight, the slab-edge planes after them) gives the same bits as
    update_ghost_values + compute_rhs (advection/stiffness.h:343, 345-605)."""
    outs = []
    for kind in ("mpi", "mpi-blocking"):
        out = tmp_path / ("u_%s.bin" % kind)
        r = _mpirun(np_, [os.path.join(HOST, "advection_app_mpi"), str(dim), str(p), str(n), "2", "0.1", str(out),
                          "1", kind], timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert ("exchange blocking" in r.stdout) == kind.endswith("blocking")
        outs.append(np.fromfile(out, dtype=np.float64))
    assert outs[0].size > 0 and np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.skipif(not HAVE_MPI, reason="MPI runtime or the MPI host programs missing")
def test_rccl_communicator_one_rank(tmp_path):
    out1, outr = tmp_path / "u1.bin", tmp_path / "ur.bin"
    args = ["3", "5", "14", "2", "0.1"]
    r1 = subprocess.run([os.path.join(HOST, "advection_app")] + args + [str(out1), "0", "1", "1"],
                        capture_output=True, text=True, timeout=120)
    assert r1.returncode == 0, r1.stderr
    r = _mpirun(1, [os.path.join(HOST, "advection_app_mpi")] + args + [str(outr), "1", "rccl"], timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "comm: rccl" in r.stdout
    assert np.array_equal(np.fromfile(out1, dtype=np.float64), np.fromfile(outr, dtype=np.float64))
