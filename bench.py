#!/usr/bin/env python3
"""bench.py -- GDM operator application (vmult) throughput on MI355X.

Metric (BASELINE.json): DoF-updates/s of the 3D advection GDM stiffness action
(StiffnessMatrixOperator::compute_rhs, applications/advection/include/gdm/
advection/stiffness.h:196-606, uncut, alpha = 0) at p = 5 on 512^3 DoFs per
GPU, plus achieved HBM GB/s of the dominant kernel against the 8 TB/s roofline.

One step = ghost-plane exchange (N > 1) + fused Kronecker stencil kernel
(volume term + outflow traces) + inflow boundary-data kernels, on inputs that
are resident in HBM.  N = 1: 512^3 DoFs (BASELINE C3).  N > 1: strong scaling
on the same 512^3 global grid (C3 "512^3 DoFs, 8 x MI355X"), z-slabs of the
reference's formula (system.h:720-757); --weak gives every rank a 512-plane
slab of a 512 x 512 x 512N grid instead.

At N = 1 the line also carries the other two per-stage operations of the RK
loop, timed the same way (HIP events on the operator's stream): the exact
mass inverse (roofline.mass_solve) and one device-resident RK4 stage
(compute_rhs + mass solve + fused stage updates + device boundary data,
rk4_stage_ms).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment
starts the N ranks itself (one child process per GPU with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set; the parent never touches
the GPU) and exits with the first failing child's code.  Under torchrun the
launcher's WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dealii-galerkin-difference-methods_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
BYTES_PER_DOF = 16.0   # algorithmic: read u once + write v once, fp64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rank-timeout", type=float, default=1800.0,
                    help="--gpus N without a launcher: seconds before hung rank processes are terminated")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="before the W warm-up steps: untimed steps until this much wall time has passed (the "
                         "clock ramp of a fresh GPU: the first ~25 back-to-back launches run 5-40 %% slower, "
                         "profiles/r6k); reported as settle_steps; 0 = off")
    ap.add_argument("--n", type=int, default=511, help="cells per direction per GPU slab (vertices = n + 1)")
    ap.add_argument("--p", type=int, default=5)
    ap.add_argument("--kind", default="advection", choices=["advection", "wave", "mass"])
    ap.add_argument("--strong", action="store_true", help="(default for N > 1) fixed 512^3 global grid")
    ap.add_argument("--weak", action="store_true", help="one 512-plane slab per GPU instead of a fixed global grid")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: nproc, bounded by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-cells", type=int, default=24, help="cells per direction of the CPU-baseline sample")
    ap.add_argument("--pmc", default=os.environ.get("GDM_BENCH_PMC", "1"), help="collect HBM PMC traffic (1/0)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--metric-only", action="store_true",
                    help="time only the metric's compute_rhs (no mass / RK-stage / PMC / CPU legs): for per-config "
                         "rocprof kernel statistics")
    return ap.parse_args()


def _band_csr(O, mesh, d, which):
    """scipy CSR of the oracle's 1D band matrix (0 = M, 1 = C, 2 = L) along d"""
    import scipy.sparse as sps

    band = mesh.matrices_1d(d)[which]
    N, p = band.shape[0], mesh.p
    return sps.diags([band[max(0, -k + p):N - max(0, k - p) + max(0, -k + p), k][: N - abs(k - p)]
                      for k in range(2 * p + 1)], [k - p for k in range(2 * p + 1)], shape=(N, N))


def _timed(fn, budget):
    t0 = time.perf_counter()
    reps = 0
    while True:
        fn()
        reps += 1
        if time.perf_counter() - t0 > budget:
            break
    return (time.perf_counter() - t0) / reps, reps


def cpu_baseline(p, n_cells, threads, threads_source="--cpu-threads"):
    """Reference algorithms from the CPU restatement in oracle/ (test
    infrastructure, the checker -- never the measured product), on bounded
    samples of the benchmark's workloads:

    * C3 (the metric): the per-cell FEValues loop of advection/stiffness.h:
      345-532 on n_cells^3 cells; `threads` host threads, each running the cell
      loop over its own z-slab of cells into a private vector (ctypes releases
      the GIL; the reference's MPI ranks do the same with one slab each),
      summed; plus the 1-thread rate;
    * the per-stage mass solve of advection/problem.h:236-267 (CSR mass +
      SolverCG/Jacobi to rel 1e-14) at 24^3 cells, 1 thread;
    * C4: the wave stiffness cell loop of wave/stiffness.h:151-181 (p=7, 3D)
      on z-slabs over `threads` threads;
    * C5: cut_poisson_01_gdm.cc:332-335's SolverCG + PreconditionIdentity
      iterations over a CSR with the full (2p+1)^2 GDM sparsity of
      system.h:586-599 (the uncut Laplacian L(x)M + M(x)L, p=3), 1 thread.
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    import scipy.sparse as sps
    import oracle as O

    a = (1.0, 0.15, -0.05)
    O.Mesh(3, p, p + 1).advection_rhs(a, np.zeros((p + 2) ** 3), None)  # load the library
    # every thread gets at least one z-layer of cells (a larger sample on a larger host)
    n_cells = max(n_cells, threads)
    m = O.Mesh(3, p, n_cells, 0.0, 1.0)
    u = np.random.default_rng(20251010).uniform(-1, 1, m.n_dofs)
    bounds = [(n_cells * t // threads, n_cells * (t + 1) // threads) for t in range(threads)]
    bcs = [np.random.default_rng(1 + t).uniform(-1, 1, max(m.n_boundary_points(cb, ce), 1)) for t, (cb, ce) in
           enumerate(bounds)]
    outs = [np.zeros(m.n_dofs) for _ in range(threads)]

    def part(t):
        cb, ce = bounds[t]
        outs[t][:] = 0.0
        m.advection_rhs(a, u, bcs[t], cb=cb, ce=ce, rhs=outs[t])

    # C4 sample: wave p=7 cell loop, z-slabs over the same threads
    nw = max(12, threads)
    mw = O.Mesh(3, 7, nw, -1.21, 1.21)
    uw = np.random.default_rng(5).uniform(-1, 1, mw.n_dofs)
    wb = [(nw * t // threads, nw * (t + 1) // threads) for t in range(threads)]

    def wpart(t):
        cb, ce = wb[t]
        if ce > cb:
            mw.wave_rhs(uw, impl=True, cb=cb, ce=ce)

    with ThreadPoolExecutor(threads) as ex:
        def all_parts():
            list(ex.map(part, range(threads)))
            np.sum(outs, axis=0)

        dt_n, reps_n = _timed(all_parts, 10.0)
        dt_w, reps_w = _timed(lambda: list(ex.map(wpart, range(threads))), 5.0)
    bc1 = np.random.default_rng(3).uniform(-1, 1, m.n_boundary_points())
    dt_1, reps_1 = _timed(lambda: m.advection_rhs(a, u, bc1), 5.0)
    # mass solve: CSR + CG(Jacobi) to rel 1e-14 (the reference's per-stage solve).  The CSR matrix is
    # the Kronecker product of the oracle's 1D mass matrices (equal to the cell-assembled matrix up to
    # round-off; the oracle's cell assembly itself takes minutes at this size)
    mm = O.Mesh(3, p, 24, 0.0, 1.0)
    M1 = [_band_csr(O, mm, d, 0) for d in range(3)]
    A = sps.kron(M1[2], sps.kron(M1[1], M1[0])).tocsr()
    A.sort_indices()
    rp, cols, vals = A.indptr.astype(np.int64), A.indices.astype(np.int64), A.data
    r = np.random.default_rng(4).uniform(-1, 1, mm.n_dofs)
    t0 = time.perf_counter()
    _, its = O.cg(rp, cols, vals, r, precond=1, max_it=1000, abs_tol=1e-20, rel_tol=1e-14)
    dt_m = time.perf_counter() - t0
    # C5 sample: identity-preconditioned CG iterations (the reference's hot loop) on a 1024^2 GDM system
    n5, it5 = 1024, 40
    m5 = O.Mesh(2, 3, n5 - 1, -1.21, 1.21)
    Mx, Lx = _band_csr(O, m5, 0, 0), _band_csr(O, m5, 0, 2)
    A5 = (sps.kron(Lx, Mx) + sps.kron(Mx, Lx)).tocsr()
    A5.sort_indices()
    rp5, c5, v5 = A5.indptr.astype(np.int64), A5.indices.astype(np.int64), A5.data
    b5 = np.ones(n5 * n5)
    t0 = time.perf_counter()
    _, its5 = O.cg(rp5, c5, v5, b5, precond=0, max_it=it5, abs_tol=0.0, rel_tol=0.0)
    its5 = it5 if its5 < 0 else its5  # gdmo_cg returns -1 when max_it ends the solve (tolerance 0 here)
    dt5 = (time.perf_counter() - t0) / its5
    return {
        "value": m.n_dofs / dt_n,
        "unit": "DoF-updates/s",
        "cores": threads,
        "cores_source": threads_source,
        "cores_visible": os.cpu_count(),
        "cores_nproc": _nproc(),
        "kind": "port",
        "cpu": _cpu_model(),
        "sample": "3D p=%d advection compute_rhs, reference per-cell algorithm (oracle/gdm_oracle.c), %d^3 cells = "
                  "%d DoFs, %d z-slabs on %d threads, %d application(s) in %.1f s"
                  % (p, n_cells, m.n_dofs, threads, threads, reps_n, dt_n * reps_n),
        "value_1_thread": m.n_dofs / dt_1,
        "sample_1_thread": "same mesh, %d application(s), 1 thread" % reps_1,
        "mass_solve": {"value": mm.n_dofs / dt_m, "unit": "DoF/s (one M^-1 r)", "cores": 1, "cg_iterations": int(its),
                       "sample": "24^3 cells p=%d: CSR mass (%d nnz) + SolverCG/Jacobi rel 1e-14, 1 thread"
                                 % (p, len(vals))},
        "c4_wave": {"value": mw.n_dofs / dt_w, "unit": "DoF-updates/s (wave compute_rhs)", "cores": threads,
                    "sample": "3D p=7 wave stiffness cell loop (wave/stiffness.h:151-181), %d^3 cells, %d z-slabs, "
                              "%d application(s)" % (nw, threads, reps_w)},
        "c5_cg": {"value": (n5 * n5) / dt5, "unit": "row-updates/s (one CG iteration = SpMV + 2 dots + 3 axpys)",
                  "ms_per_iteration": dt5 * 1e3, "cores": 1,
                  # C5 is 4096^2: a CG iteration is linear in the rows (fixed (2p+1)^2 entries per row), so the
                  # 1024^2 sample's time per row is extrapolated x16 (the 4096^2 CSR would need ~13 GB of host
                  # memory and minutes of assembly inside the bench)
                  "ms_per_iteration_c5_extrapolated": dt5 * 1e3 * (4096 * 4096) / (n5 * n5),
                  "sample": "2D p=3 %d^2 DoFs, CSR %d nnz (full (2p+1)^2 GDM sparsity), SolverCG + "
                            "PreconditionIdentity, %d iterations, 1 thread" % (n5, len(v5), its5)},
    }


FP64_VALU_PEAK_TFS = 78.6  # MI355X FP64 vector peak (MI355X_MICROARCH.md chip table; FMA = 2 flop)
# minimum FP64 FMA per DoF of the factored p = 5 advection stencil: x sweep 11 (mass) + 10
# (derivative, zero centre tap), y sweep 11 + 21, z sweep 21, plus the x scale and the dint / z-mass folds
ADV5_MIN_FMA = 77


def c4_wave_stage(steps=10):
    """BASELINE config C4 on one GPU: applications/wave wave-rk, p = 7, 256^3
    vertices on [-1.21, 1.21]^3 (wave/problem.h:280-346): the stiffness
    compute_rhs (wave/stiffness.h:151-181), the exact mass inverse and one
    device-resident RK4 stage (WaveProblem.step / 4), HIP events on the
    operator stream.  The p = 7 stencil is FP64-ALU-bound: 105 FMA per DoF
    (x: 15 + 15, y: 15 + 30, z: 15 + 15) = 210 flop/DoF, reported against the
    78.6 TF/s FP64 vector peak; its HBM figure is 16 B/DoF."""
    import torch
    from gdm_amd import GdmOperator, WaveProblem

    n, p = 255, 7
    op = GdmOperator(3, p, n, -1.21, 1.21, "wave")
    N = op.n_owned
    gen = torch.Generator(device="cuda").manual_seed(20251011)
    u = torch.rand(N, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    v = op.new_vector(False)
    op.time_op(0, u, v, None, 3)
    st_ms = op.time_op(0, u, v, None, steps)
    op.time_op(2, v, u, None, 2)
    ms_ms = op.time_op(2, v, u, None, steps)
    prob = WaveProblem(op)
    prob.u.copy_(u)
    prob.step(0.0, 1e-4)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for i in range(3):
        prob.step(i * 1e-4, 1e-4)
    e1.record()
    torch.cuda.synchronize()
    stage = e0.elapsed_time(e1) / 12.0
    flops = 210.0 * N
    out = {
        "workload": "3D wave GDM p=7, 256^3 vertices (16.8 M DoFs), wave-rk",
        "stencil_ms": st_ms,
        "stencil_fp64_tflops": flops / (st_ms * 1e-3) / 1e12,
        "stencil_valu_frac": flops / (st_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFS,
        "stencil_hbm_frac": BYTES_PER_DOF * N / (st_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "mass_solve_ms": ms_ms,
        "rk4_stage_ms": stage,
        "dof_updates_per_s": N / (st_ms * 1e-3),
    }
    del prob, op, u, v
    torch.cuda.empty_cache()
    out["per_rank_8"] = c4_rank_slab(steps)
    return out


def c4_rank_slab(steps=10, n_ranks=8, rank=3):
    """C4 at its named 8-GPU size, one rank's share on this GPU: the 256^2 x
    32-plane slab of an interior rank (+ 2 x 7 ghost planes) of the reference's
    slab partition (system.h:720-757).  Device work per stage of that rank: the
    p = 7 wave stencil on the slab (wave/stiffness.h:151-181) and the
    distributed exact mass inverse (truncated SPIKE: slab solve, one
    refinement round, interface correction; wave/problem.h:457-502's solve).
    The ghost exchanges between them are not part of this single-GPU figure
    (2 x 7 planes x 0.5 MiB per exchange; xGMI point-to-point at N = 8)."""
    import torch
    from gdm_amd import GdmOperator

    from gdm_amd import _capi

    n, p = 255, 7
    op = GdmOperator(3, p, n, -1.21, 1.21, "wave", n_ranks=n_ranks, rank=rank)
    rounds = _capi.mesh_spike_rounds(op.mesh)
    gen = torch.Generator(device="cuda").manual_seed(20251012)
    u = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    v = op.new_vector(False)
    op.time_op(0, u, v, None, 3)
    st_ms = op.time_op(0, u, v, None, steps)
    x = op.new_vector(True)
    r = v.clone()

    def solve():
        op.mass_solve_slab(r, op.owned_view(x))
        for k in range(rounds):
            op.mass_solve_interface_round(x, k)
        op.mass_solve_interface(x)

    solve()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        solve()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    N = op.n_owned
    L = op.layout
    res = {
        "workload": "C4 rank %d of %d: 256^2 x %d owned planes + %d + %d ghost planes, p=7 wave"
                    % (rank, n_ranks, N // L["plane_size"], L["ghost_planes_below"], L["ghost_planes_above"]),
        "n_dofs_rank": N,
        "stencil_ms": st_ms,
        "stencil_valu_frac": 210.0 * N / (st_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFS,
        "stencil_hbm_frac": BYTES_PER_DOF * N / (st_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "spike_solve_ms": ms,
        "spike_rounds": rounds,
    }
    del op, u, v, x, r
    torch.cuda.empty_cache()
    return res


def c3_rank_slab(steps=10, n_ranks=8, rank=3):
    """C3 at its named 8-GPU split, one rank's share on this GPU: rank 3 of 8
    of the 512^3 p = 5 advection grid (system.h:720-757: 64 owned + 2 x 5
    ghost planes).  compute_rhs_ms: the stage's compute_rhs of the
    one-exchange RK (SlabRK4 / the C++ one_exchange_per_stage: the ghost
    planes are current, one launch over the owned planes with the inflow
    data); compute_rhs_overlapped_ms: as apply_overlapped runs it when the
    stage vector is exchanged first (advection/stiffness.h:343
    update_ghost_values overlapped with the planes that need no ghosts: the
    interior planes, the 2 x p edge planes, the inflow data).  The exchanges
    need a second GPU and are not part of these figures.  The mass inverse is
    the distributed exact one of that rank (truncated SPIKE: slab solve +
    interface correction with the ghost planes written, problem.h:236-267)."""
    import torch
    from gdm_amd import GdmOperator, _capi
    from gdm_amd.distributed import apply_overlapped

    op = GdmOperator(3, 5, 511, 0.0, 1.0, "advection", params=(1.0, 0.15, -0.05), n_ranks=n_ranks, rank=rank)
    L = op.layout
    gen = torch.Generator(device="cuda").manual_seed(20251013)
    u = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    v = op.new_vector(False)
    bc = torch.rand(max(op.n_bc_points, 1), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    p = L["halo_depth"]
    pb, pe = L["owned_plane_begin"], L["owned_plane_end"]
    lo = pb + (p if L["ghost_planes_below"] else 0)
    hi = pe - (p if L["ghost_planes_above"] else 0)

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    whole = timed(lambda: apply_overlapped(op, None, u, v, bc if op.n_bc_points else None))
    # the one-exchange RK stage (SlabRK4, C++ one_exchange_per_stage): the
    # stage vector's ghost planes are current when the stencil starts, so
    # compute_rhs is one launch over all owned planes (no overlap split)
    single = timed(lambda: op.apply(u, v, bc if op.n_bc_points else None))
    interior = timed(lambda: op.apply_planes(u, v, lo, hi))

    def edges():  # both edge ranges in one launch, as apply_overlapped runs them
        op.apply_planes2(u, v, pb, lo, hi, pe)

    edge = timed(edges)
    rounds = _capi.mesh_spike_rounds(op.mesh)
    x = op.new_vector(True)
    r = v.clone()

    def solve():
        op.mass_solve_slab(r, op.owned_view(x))
        for k in range(rounds):
            op.mass_solve_interface_round(x, k)
        op.mass_solve_interface_ghosts(x)

    spike = timed(solve)
    # the whole one-exchange RK stage of this rank without its exchanges
    # (SlabRK4 / the C++ one_exchange_per_stage): compute_rhs into k's owned
    # planes, the slab solve in place, the refinement rounds, then the
    # interface correction fused with the stage update over the local vectors
    # (gdm_mass_solve_interface_rk) -- or, unfused, interface_ghosts +
    # rk_update over n_local (the same bits)
    k = op.new_vector(True)
    acc, Y = op.new_vector(True), op.new_vector(True)
    kown = op.owned_view(k)

    def stage(fused):
        op.apply(u, kown, bc if op.n_bc_points else None)
        op.mass_solve_slab(kown, kown)
        for q in range(rounds):
            op.mass_solve_interface_round(k, q)
        if fused:
            op.mass_solve_interface_rk(k, 0.1, acc, acc, 0.05, u, Y)
        else:
            op.mass_solve_interface_ghosts(k)
            op.rk_update(0.1, k, acc, acc, 0.05, u, Y)

    stage_fused = timed(lambda: stage(True))
    stage_unfused = timed(lambda: stage(False))
    del k, acc, Y, kown
    N = op.n_owned
    n_int = (hi - lo) * L["plane_size"]
    res = {
        "workload": "C3 rank %d of %d: 512^2 x %d owned planes + %d + %d ghost planes, p=5 advection"
                    % (rank, n_ranks, pe - pb, L["ghost_planes_below"], L["ghost_planes_above"]),
        "n_dofs_rank": N,
        "compute_rhs_ms": single,
        "compute_rhs_overlapped_ms": whole,
        "interior_planes_ms": interior,
        "edge_planes_ms": edge,
        "stencil_frac": BYTES_PER_DOF * N / (single * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "stencil_frac_overlapped": BYTES_PER_DOF * N / (whole * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "interior_frac": BYTES_PER_DOF * n_int / (interior * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "spike_solve_ms": spike,
        "spike_rounds": rounds,
        "mass_solve_frac": BYTES_PER_DOF * N / (spike * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "rk_stage_ms": stage_fused,
        "rk_stage_unfused_ms": stage_unfused,
    }
    del op, u, v, x, r, bc
    torch.cuda.empty_cache()
    return res


def _nproc():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def _cgroup_cpus():
    """CPUs the cgroup's CFS quota allots this process (cgroup v2 cpu.max or
    v1 cpu.cfs_quota_us / cpu.cfs_period_us), with the file it came from;
    (None, None) when unlimited or unreadable."""
    import math

    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(per))), "/sys/fs/cgroup/cpu.max"
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, math.ceil(q / per)), "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
    except (OSError, ValueError):
        pass
    return None, None


def cpu_threads():
    """Threads of the CPU baseline: the affinity mask (nproc), bounded by the
    cgroup's CPU quota when there is one; returns (threads, source)."""
    n = _nproc()
    cg, src = _cgroup_cpus()
    if cg is not None and cg < n:
        return cg, "cgroup quota (%s)" % src
    return n, "sched_getaffinity (nproc)"


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def pmc_traffic(args):
    """HBM bytes per stencil launch from rocprofv3 PMC counters, collected in
    separate passes (FETCH_SIZE, WRITE_SIZE) by a child process; FETCH_SIZE is
    doubled per MI355X_MICROARCH.md 'HBM' (gfx950 reports half of a wide
    coalesced stream).  Returns bytes or None."""
    import csv
    import glob
    import shutil
    import tempfile

    if not shutil.which("rocprofv3"):
        return None
    res = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        out = tempfile.mkdtemp(prefix="gdm_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", out, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--n", str(args.n), "--p", str(args.p),
               "--kind", args.kind]
        try:
            subprocess.run(cmd, check=True, timeout=300, capture_output=True, cwd=ROOT)
        except Exception:
            return None
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        per_kernel = {}  # one application = one launch of each stencil kernel (interior-z + z-wall)
        for f in files:
            for row in csv.DictReader(open(f)):
                if "stencil" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                    per_kernel.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
        shutil.rmtree(out, ignore_errors=True)
        if not per_kernel:
            return None
        # median over launches per kernel, summed over the kernels of one application (KiB)
        res[ctr] = sum(sorted(v)[len(v) // 2] for v in per_kernel.values())
    return (2.0 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024.0


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n, cmd, env=None, poll_s=0.2, timeout_s=None):
    """Run `cmd` as n rank processes of one job on this node (one per GPU):
    each child gets RANK = LOCAL_RANK = r, WORLD_SIZE = n, MASTER_ADDR =
    127.0.0.1 and a free MASTER_PORT, and inherits stdout / stderr (rank 0
    prints the JSON line).  Returns 0 when every child exits 0, else the first
    non-zero exit code seen (a child killed by signal s gives 128 + s); the
    other children are then terminated by PID, so that none is left waiting in
    a collective.  timeout_s (None: no limit): past it every child still
    running is terminated and 124 returned (a rank hung in a collective never
    exits by itself).  An exception in the parent -- SIGINT, or SIGTERM, which
    is turned into one -- terminates the children too (try / finally), then
    kills any that ignore SIGTERM for 10 s.  The caller must not have touched
    the GPU.  (MASTER_PORT is probed free here and bound by rank 0's store a
    moment later; another process taking it in between fails the job's
    rendezvous loudly, it does not hang.)"""
    import signal

    base = dict(os.environ if env is None else env)
    base.update({"WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port())})
    procs = []

    def _term(signum, frame):
        raise KeyboardInterrupt("signal %d" % signum)

    old_term = signal.signal(signal.SIGTERM, _term)
    rc = 0
    try:
        for r in range(n):
            e = dict(base)
            e.update({"RANK": str(r), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(n)})
            procs.append(subprocess.Popen(cmd, env=e))
        t_end = None if timeout_s is None else time.monotonic() + timeout_s
        live = list(procs)
        while live:
            for pr in list(live):
                c = pr.poll()
                if c is None:
                    continue
                live.remove(pr)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    for other in live:
                        other.terminate()
            if live and t_end is not None and time.monotonic() > t_end:
                for pr in live:
                    pr.terminate()
                if rc == 0:
                    rc = 124
                t_end = None
            time.sleep(poll_s)
    finally:
        signal.signal(signal.SIGTERM, old_term)
        stragglers = [pr for pr in procs if pr.poll() is None]
        for pr in stragglers:
            pr.terminate()
        for pr in stragglers:
            try:
                pr.wait(10)
            except subprocess.TimeoutExpired:
                pr.kill()
                pr.wait()
    return rc


def rank_command(argv):
    """the command of one rank started by `bench.py --gpus N`: this script
    with the parent's arguments (the child sees WORLD_SIZE and runs its rank)"""
    return [sys.executable, os.path.abspath(__file__)] + list(argv)


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # no launcher: start the ranks here (before anything initialises the GPU)
        sys.exit(spawn_ranks(args.gpus, rank_command(sys.argv[1:]), timeout_s=args.rank_timeout))
    if world_env is not None and int(world_env) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (world_env, args.gpus), file=sys.stderr)
        sys.exit(2)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from gdm_amd import GdmOperator
    from gdm_amd.distributed import HaloExchange, apply_overlapped

    p, n = args.p, args.n
    weak = args.weak and not args.strong
    nz_cells = (n + 1) * world - 1 if (weak and world > 1) else n
    n_sub = (n, n, nz_cells)
    hi = (1.0, 1.0, nz_cells / n)  # uniform h = 1/n
    a = (1.0, 0.15, -0.05)        # advection_01_gdm.cc:37-41
    params = a if args.kind == "advection" else ()
    op = GdmOperator(3, p, n_sub, (0.0, 0.0, 0.0), hi, args.kind, params=params, rank=rank, n_ranks=world,
                     device=local_rank)
    lay = op.layout
    gen = torch.Generator(device="cuda").manual_seed(20251010 + rank)
    src = torch.rand(op.n_local, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    dst = op.new_vector(local=False)
    bc = None
    if args.kind == "advection" and op.n_bc_points > 0:
        bc = torch.rand(op.n_bc_points, dtype=torch.float64, device="cuda", generator=gen) * 2 - 1

    if args.pmc_child:
        for _ in range(3):
            op.apply(src, dst)
        torch.cuda.synchronize()
        return

    halo = HaloExchange(nz_cells, world, rank, lay["plane_size"], lay["halo_depth"]) if world > 1 else None
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        if halo is not None:
            # ghost-plane exchange overlapped with the planes that need no ghosts
            apply_overlapped(op, halo, src, dst)
            if bc is not None:
                op.add_boundary_data(bc, dst)
        else:
            # compute_rhs in one call: one stencil launch over all planes with the inflow faces' step 1 as its
            # tail work, then face step 2 fused with the ordered adds
            op.apply(src, dst, bc)
        if ev is not None:
            ev[1].record(stream)

    # settle: the GPU's clocks ramp over the first ~25 back-to-back launches of a fresh process
    # (profiles/r6k/README.md); untimed, before and in addition to the W warm-up steps
    settle_steps = 0
    if args.settle_ms > 0:
        torch.cuda.synchronize()
        ts = time.perf_counter()
        while True:
            for _ in range(10):
                step()
            settle_steps += 10
            torch.cuda.synchronize()
            done = (time.perf_counter() - ts) * 1e3 >= args.settle_ms or settle_steps >= 100000
            if dist is not None:  # every rank runs the same steps (the halo exchanges pair up)
                f = torch.tensor([1.0 if done else 0.0], device="cuda")
                dist.all_reduce(f, op=dist.ReduceOp.MAX)
                done = float(f) > 0.0
            if done:
                break
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(e0.elapsed_time(e1) for e0, e1 in events) / args.steps
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    total_dofs = lay["n_dofs_global"]
    ms_per_step = elapsed / args.steps * 1e3
    value = total_dofs * args.steps / elapsed

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    achieved = BYTES_PER_DOF * lay["n_owned"] / (kern_ms * 1e-3) / 1e9
    mass = stage_ms = None
    if world == 1 and not args.metric_only:
        # the exact mass inverse (gdm_mass_solve; HIP events on the op stream) and one device-resident RK4
        # stage of the advection problem (AdvectionProblem.step / 4)
        op.time_op(2, dst, src[:lay["n_owned"]], None, 2)  # warm-up (first launches of the line-solve kernels)
        ms = op.time_op(2, dst, src[:lay["n_owned"]], None, 10)
        mass = {"bound": "hbm", "kernel": "mass3_strided_kernel (z, y) + mass3_rows_kernel (x)",
                "achieved": BYTES_PER_DOF * lay["n_owned"] / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": BYTES_PER_DOF * lay["n_owned"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernel_ms": ms,
                "algorithmic_bytes_per_launch": BYTES_PER_DOF * lay["n_owned"]}
        if args.kind == "advection":
            from gdm_amd import AdvectionProblem

            prob = AdvectionProblem(op, op.FN_SINE_PRODUCT, [1.0, 0.15, -0.05, 1.0, 1.0, 1.0, 0.3, 0.0, 0.7])
            prob.u.copy_(src[:lay["n_owned"]])
            prob.step(0.0, 1e-4)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(3):
                prob.step(i * 1e-4, 1e-4)
            e1.record()
            torch.cuda.synchronize()
            stage_ms = e0.elapsed_time(e1) / 12.0
            del prob
    c4 = c3r = None
    if world == 1 and not args.metric_only:
        c3r = c3_rank_slab()
        c4 = c4_wave_stage()
    traffic = None
    if world == 1 and str(args.pmc) == "1" and not args.metric_only:
        traffic = pmc_traffic(args)
    cpu = None
    if world == 1 and not args.no_cpu_baseline and not args.metric_only:
        try:
            # every CPU this process may run on: the affinity mask (nproc), bounded by the cgroup's CPU quota
            th, src = (args.cpu_threads, "--cpu-threads") if args.cpu_threads else cpu_threads()
            cpu = cpu_baseline(p, args.cpu_cells, th, src)
        except Exception as e:  # the baseline never blocks the GPU line
            cpu = {"value": None, "error": str(e)}
    out = {
        "metric": "DoF-updates/sec (vmult) + achieved HBM GB/s, 3D advection p=5 at 1/2/4/8 GPUs",
        "value": value,
        "unit": "DoF-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_steps": settle_steps,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak" if (weak and world > 1) else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: u ~ U[-1,1) seeded, stage boundary values ~ U[-1,1); inputs resident in HBM",
        "config": {
            "workload": "3D %s GDM compute_rhs (uncut), p=%d, %dx%dx%d vertices global, %d vertex planes per rank"
                        % (args.kind, p, n + 1, n + 1, nz_cells + 1, lay["owned_plane_end"] - lay["owned_plane_begin"]),
            "fe_degree": p,
            "n_dofs_global": total_dofs,
            "n_dofs_per_gpu": lay["n_owned"],
            "advection": list(a) if args.kind == "advection" else None,
            "partition": "z-slabs, system.h:720-757 formula, %d ghost planes per side" % lay["halo_depth"],
            "parallelism": "slab%d" % world,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "compute_rhs = stencil8_kernel<p=%d> (fused Kronecker stencil, all planes, inflow face step 1 "
                      "as tail work) + face step 2 with the ordered adds; HIP events around the whole call" % p,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel_ms": kern_ms,
            "algorithmic_bytes_per_launch": BYTES_PER_DOF * lay["n_owned"],
            # the other bound of this kernel: FP64 VALU at the factored stencil's minimum FMA count
            "fp64_valu": None if args.kind != "advection" or p != 5 else {
                "fma_per_dof": ADV5_MIN_FMA, "achieved": 2.0 * ADV5_MIN_FMA * lay["n_owned"] / (kern_ms * 1e-3) / 1e12,
                "peak": FP64_VALU_PEAK_TFS, "unit": "TFLOP/s",
                "frac": 2.0 * ADV5_MIN_FMA * lay["n_owned"] / (kern_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFS},
            "mass_solve": mass,
        },
        "rk4_stage_ms": stage_ms,
        "c3_per_rank_8": c3r,
        "c4_wave": c4,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
