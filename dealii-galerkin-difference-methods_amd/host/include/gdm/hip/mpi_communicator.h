// gdm/hip/mpi_communicator.h -- Communicators for one process per GPU, the
// reference's own parallel model (MPI ranks, z-slabs of system.h:720-757):
//
//   MpiRank   ghost planes staged through host memory with MPI point-to-point
//             messages over the gdm_halo_plan ranges, reductions by
//             MPI_Allreduce (what LinearAlgebra::distributed::Vector::
//             update_ghost_values and Utilities::MPI::sum / max do for the
//             reference: advection/stiffness.h:343, problem.h:410-425)
//   RcclRank  (GDM_WITH_RCCL) the same exchange device to device with RCCL
//             ncclSend / ncclRecv inside ncclGroupStart / End on a comm
//             stream (xGMI peer-to-peer between the GPUs of a node; the
//             communicator is set up with ncclCommInitRank, the unique id
//             broadcast over MPI), ordered against the operator's stream by
//             events only (no host synchronisation); scalar reductions stay
//             on MPI
// Both implement the split-phase begin_ / end_update_ghost_values that
// StiffnessMatrixOperator::compute_rhs_overlapped brackets the interior
// planes with.
//
// Both exchange exactly the planes the owner-computes stencil reads: p planes
// from each z-neighbour (gdm_halo_plan), nothing is exported back (no
// compress(add)).
#pragma once

#include <gdm/hip/operators.h>
#include <mpi.h>

#include <vector>

#ifdef GDM_WITH_RCCL
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#endif

namespace GDM {
namespace HIP {

// The message pattern of one ghost exchange on host buffers: send the owned
// edge planes to the neighbours, receive their edge planes into the ghost
// ranges.  Tags: 1 = data moving up (to rank + 1), 2 = moving down.  Split
// phase: post_planes starts the four messages, Waitall on its requests ends
// them; exchange_planes does both.
struct PlaneRequests {
  MPI_Request req[4];
  int n = 0;
  void wait() {
    if (n) MPI_Waitall(n, req, MPI_STATUSES_IGNORE);
    n = 0;
  }
};

inline void post_planes(const gdm_halo &plan, MPI_Comm comm, const double *send_below, const double *send_above,
                        double *recv_below, double *recv_above, PlaneRequests &r) {
  r.n = 0;
  if (plan.rank_below >= 0 && plan.recv_below_count > 0)
    MPI_Irecv(recv_below, (int)plan.recv_below_count, MPI_DOUBLE, plan.rank_below, 1, comm, &r.req[r.n++]);
  if (plan.rank_above >= 0 && plan.recv_above_count > 0)
    MPI_Irecv(recv_above, (int)plan.recv_above_count, MPI_DOUBLE, plan.rank_above, 2, comm, &r.req[r.n++]);
  if (plan.rank_above >= 0 && plan.send_above_count > 0)
    MPI_Isend(send_above, (int)plan.send_above_count, MPI_DOUBLE, plan.rank_above, 1, comm, &r.req[r.n++]);
  if (plan.rank_below >= 0 && plan.send_below_count > 0)
    MPI_Isend(send_below, (int)plan.send_below_count, MPI_DOUBLE, plan.rank_below, 2, comm, &r.req[r.n++]);
}

inline void exchange_planes(const gdm_halo &plan, MPI_Comm comm, const double *send_below, const double *send_above,
                            double *recv_below, double *recv_above) {
  PlaneRequests r;
  post_planes(plan, comm, send_below, send_above, recv_below, recv_above, r);
  r.wait();
}

inline gdm_halo halo_plan_of(const gdm_mesh_desc &mesh, int rank) {
  gdm_mesh_desc m = mesh;
  m.rank = rank;
  gdm_halo plan{};
  check(gdm_halo_plan(&m, &plan), "gdm_halo_plan");
  return plan;
}

class MpiRank : public Communicator {
 public:
  MpiRank(MPI_Comm comm, const gdm_mesh_desc &mesh) : comm(comm) {
    int r = 0;
    MPI_Comm_rank(comm, &r);
    plan = halo_plan_of(mesh, r);
    sb.resize(plan.send_below_count);
    sa.resize(plan.send_above_count);
    rb.resize(plan.recv_below_count);
    ra.resize(plan.recv_above_count);
  }
  void update_ghost_values(gdm_op *op, DeviceVector &local) override {
    begin_update_ghost_values(op, local);
    end_update_ghost_values(op, local);
  }
  // begin: the edge planes to host (gdm_memcpy_d2h waits for the work queued
  // on op: the owned planes are final), the four messages posted.  end: wait
  // for them, the ghost planes to the device (ordered on op's stream after
  // whatever was queued in between, e.g. the interior planes of the stencil).
  void begin_update_ghost_values(gdm_op *op, DeviceVector &local) override {
    double *v = local.get_values();
    const size_t d = sizeof(double);
    if (!sb.empty()) check(gdm_memcpy_d2h(op, sb.data(), v + plan.send_below_offset, d * sb.size()), "d2h");
    if (!sa.empty()) check(gdm_memcpy_d2h(op, sa.data(), v + plan.send_above_offset, d * sa.size()), "d2h");
    post_planes(plan, comm, sb.data(), sa.data(), rb.data(), ra.data(), pending);
  }
  void end_update_ghost_values(gdm_op *op, DeviceVector &local) override {
    pending.wait();
    double *v = local.get_values();
    const size_t d = sizeof(double);
    if (!rb.empty()) check(gdm_memcpy_h2d(op, v + plan.recv_below_offset, rb.data(), d * rb.size()), "h2d");
    if (!ra.empty()) check(gdm_memcpy_h2d(op, v + plan.recv_above_offset, ra.data(), d * ra.size()), "h2d");
  }
  double sum(double v) override {
    double s = 0.0;
    MPI_Allreduce(&v, &s, 1, MPI_DOUBLE, MPI_SUM, comm);
    return s;
  }
  double max(double v) override {
    double s = 0.0;
    MPI_Allreduce(&v, &s, 1, MPI_DOUBLE, MPI_MAX, comm);
    return s;
  }
  const gdm_halo &get_plan() const { return plan; }

 private:
  MPI_Comm comm;
  gdm_halo plan{};
  std::vector<double> sb, sa, rb, ra;
  PlaneRequests pending;
};

#ifdef GDM_WITH_RCCL
class RcclRank : public Communicator {
 public:
  RcclRank(MPI_Comm comm, const gdm_mesh_desc &mesh, int device) : mpi(comm) {
    int r = 0, n = 1;
    MPI_Comm_rank(comm, &r);
    MPI_Comm_size(comm, &n);
    plan = halo_plan_of(mesh, r);
    ncclUniqueId id;
    if (r == 0 && ncclGetUniqueId(&id) != ncclSuccess) throw Error("ncclGetUniqueId failed");
    MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, comm);
    if (hipSetDevice(device) != hipSuccess) throw Error("hipSetDevice failed");
    if (ncclCommInitRank(&nccl, n, id, r) != ncclSuccess) throw Error("ncclCommInitRank failed");
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) throw Error("hipStreamCreate failed");
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess)
      throw Error("hipEventCreate failed");
  }
  ~RcclRank() override {
    ncclCommDestroy(nccl);
    (void)hipEventDestroy(ready);
    (void)hipEventDestroy(done);
    (void)hipStreamDestroy(stream);
  }
  void update_ghost_values(gdm_op *op, DeviceVector &local) override {
    begin_update_ghost_values(op, local);
    end_update_ghost_values(op, local);
  }
  // begin: the comm stream waits (device side, no host synchronisation) for
  // the work queued on op's stream so far, then runs the send / recv group;
  // end: op's stream waits for the group.  Between the two, op's stream runs
  // the interior planes concurrently with the xGMI transfers.
  void begin_update_ghost_values(gdm_op *op, DeviceVector &local) override {
    void *s = nullptr;
    check(gdm_op_get_stream(op, &s), "gdm_op_get_stream");
    op_stream = (hipStream_t)s;
    if (hipEventRecord(ready, op_stream) != hipSuccess || hipStreamWaitEvent(stream, ready, 0) != hipSuccess)
      throw Error("RcclRank: ordering the exchange after the owned planes failed");
    double *v = local.get_values();
    bool ok = ncclGroupStart() == ncclSuccess;
    if (plan.rank_below >= 0 && plan.recv_below_count > 0)
      ok &= ncclRecv(v + plan.recv_below_offset, plan.recv_below_count, ncclDouble, plan.rank_below, nccl, stream) ==
            ncclSuccess;
    if (plan.rank_above >= 0 && plan.recv_above_count > 0)
      ok &= ncclRecv(v + plan.recv_above_offset, plan.recv_above_count, ncclDouble, plan.rank_above, nccl, stream) ==
            ncclSuccess;
    if (plan.rank_above >= 0 && plan.send_above_count > 0)
      ok &= ncclSend(v + plan.send_above_offset, plan.send_above_count, ncclDouble, plan.rank_above, nccl, stream) ==
            ncclSuccess;
    if (plan.rank_below >= 0 && plan.send_below_count > 0)
      ok &= ncclSend(v + plan.send_below_offset, plan.send_below_count, ncclDouble, plan.rank_below, nccl, stream) ==
            ncclSuccess;
    ok &= ncclGroupEnd() == ncclSuccess;
    if (!ok || hipEventRecord(done, stream) != hipSuccess) throw Error("RCCL ghost exchange failed");
  }
  void end_update_ghost_values(gdm_op *op, DeviceVector &local) override {
    (void)op;
    (void)local;
    if (hipStreamWaitEvent(op_stream, done, 0) != hipSuccess) throw Error("RcclRank: waiting for the exchange failed");
  }
  double sum(double v) override {
    double s = 0.0;
    MPI_Allreduce(&v, &s, 1, MPI_DOUBLE, MPI_SUM, mpi);
    return s;
  }
  double max(double v) override {
    double s = 0.0;
    MPI_Allreduce(&v, &s, 1, MPI_DOUBLE, MPI_MAX, mpi);
    return s;
  }

 private:
  MPI_Comm mpi;
  gdm_halo plan{};
  ncclComm_t nccl{};
  hipStream_t stream{}, op_stream{};
  hipEvent_t ready{}, done{};
};
#endif

}  // namespace HIP
}  // namespace GDM
