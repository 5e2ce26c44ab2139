// gdm/hip/thread_communicator.h -- a Communicator whose ranks are threads of
// one process (all on one device): the multi-rank host path of the C++
// mirror (gdm/hip/operators.h) in tests, with MPI-like semantics.  Each
// update_ghost_values publishes the rank's vector, waits for every rank,
// copies the neighbours' planes named by gdm_halo_plan into its ghost ranges
// (device-to-device on its own stream) and waits again before returning;
// sum() is an all-reduce over the ranks.  An MPI rank implements the same
// interface with MPI_Isend / MPI_Irecv on those ranges.
#pragma once

#include <gdm/hip/operators.h>

#include <condition_variable>
#include <mutex>
#include <vector>

namespace GDM {
namespace HIP {

class ThreadGroup {
 public:
  explicit ThreadGroup(int n_ranks) : n(n_ranks), ptrs(n_ranks, nullptr), vals(n_ranks, 0.0) {}

  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const unsigned long gen = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }

  class Rank : public Communicator {
   public:
    Rank(ThreadGroup &g, int rank, const gdm_mesh_desc &mesh) : g(g), rank(rank) {
      gdm_mesh_desc m = mesh;
      m.rank = rank;
      check(gdm_halo_plan(&m, &plan), "gdm_halo_plan");
    }
    void update_ghost_values(gdm_op *op, DeviceVector &local) override {
      check(gdm_synchronize(op), "gdm_synchronize");
      g.ptrs[rank] = local.get_values();
      g.barrier();
      if (plan.rank_below >= 0 && plan.recv_below_count > 0) {
        // the lower neighbour's last planes (its send-above range)
        const gdm_halo &nb = g.plans_of(plan.rank_below);
        check(gdm_memcpy_d2d(op, local.get_values() + plan.recv_below_offset,
                             g.ptrs[plan.rank_below] + nb.send_above_offset, sizeof(double) * plan.recv_below_count),
              "gdm_memcpy_d2d");
      }
      if (plan.rank_above >= 0 && plan.recv_above_count > 0) {
        const gdm_halo &nb = g.plans_of(plan.rank_above);
        check(gdm_memcpy_d2d(op, local.get_values() + plan.recv_above_offset,
                             g.ptrs[plan.rank_above] + nb.send_below_offset, sizeof(double) * plan.recv_above_count),
              "gdm_memcpy_d2d");
      }
      check(gdm_synchronize(op), "gdm_synchronize");
      g.barrier();
    }
    double sum(double v) override {
      g.vals[rank] = v;
      g.barrier();
      double s = 0.0;
      for (double x : g.vals) s += x;  // same order on every rank
      g.barrier();
      return s;
    }
    double max(double v) override {
      g.vals[rank] = v;
      g.barrier();
      double s = g.vals[0];
      for (double x : g.vals) s = x > s ? x : s;
      g.barrier();
      return s;
    }
    const gdm_halo &get_plan() const { return plan; }

   private:
    ThreadGroup &g;
    int rank;
    gdm_halo plan{};
  };

  // ranks register their plans before the first exchange
  void set_plans(const std::vector<gdm_halo> &p) { plans = p; }
  const gdm_halo &plans_of(int r) const { return plans[r]; }

 private:
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long generation = 0;
  std::vector<double *> ptrs;
  std::vector<double> vals;
  std::vector<gdm_halo> plans;
};

}  // namespace HIP
}  // namespace GDM
