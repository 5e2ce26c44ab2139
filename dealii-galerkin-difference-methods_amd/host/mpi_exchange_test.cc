// mpi_exchange_test.cc -- CPU test of the MPI communicator's message pattern
// (gdm/hip/mpi_communicator.h exchange_planes over the gdm_halo_plan ranges,
// host buffers, no GPU) and of its reductions.
//
//   mpirun -np R mpi_exchange_test DIM P N
//
// Every rank fills its owned entries with their global DoF index, exchanges
// the ghost planes and checks that each received entry holds the global index
// of the vertex it stands for (the lower neighbour's last planes below, the
// upper neighbour's first planes above), repeats the exchange in split phase
// (post, work, wait) and compares bitwise, then checks MPI sum / max.  Prints
// "ok" on rank 0.
#include <gdm/hip/mpi_communicator.h>
#include <mpi.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 1, bad = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  const int dim = argc > 1 ? std::atoi(argv[1]) : 3, p = argc > 2 ? std::atoi(argv[2]) : 5,
            n = argc > 3 ? std::atoi(argv[3]) : 40;
  gdm_mesh_desc mesh{};
  mesh.dim = dim;
  mesh.fe_degree = p;
  for (int d = 0; d < 3; ++d) {
    mesh.n_subdivisions[d] = d < dim ? (d == dim - 1 ? n : 6) : 1;
    mesh.lo[d] = 0.0;
    mesh.hi[d] = 1.0;
  }
  mesh.n_ranks = size;
  try {
    const gdm_halo plan = GDM::HIP::halo_plan_of(mesh, rank);
    int64_t ps = 1;
    for (int d = 0; d < dim - 1; ++d) ps *= mesh.n_subdivisions[d] + 1;
    // the slab of system.h:729-737: stride = ceil(n / R), planes [r stride + (r > 0), (r + 1) stride + 1) cap n + 1
    const int stride = (n + size - 1) / size;
    const int pb = std::min(n + 1, rank * stride + (rank > 0 ? 1 : 0)), pe = std::min(n + 1, (rank + 1) * stride + 1);
    const int64_t owned = (int64_t)(pe - pb) * ps, g0 = (int64_t)pb * ps;
    std::vector<double> local(plan.owned_offset + owned + plan.recv_above_count, -1.0);
    for (int64_t i = 0; i < owned; ++i) local[plan.owned_offset + i] = (double)(g0 + i);
    GDM::HIP::exchange_planes(plan, MPI_COMM_WORLD, local.data() + plan.send_below_offset,
                              local.data() + plan.send_above_offset, local.data() + plan.recv_below_offset,
                              local.data() + plan.recv_above_offset);
    for (int64_t i = 0; i < plan.recv_below_count; ++i)
      bad += local[plan.recv_below_offset + i] != (double)(g0 - plan.recv_below_count + i);
    for (int64_t i = 0; i < plan.recv_above_count; ++i)
      bad += local[plan.recv_above_offset + i] != (double)(g0 + owned + i);
    if ((rank > 0) != (plan.recv_below_count > 0) || (rank + 1 < size && pe <= n) != (plan.recv_above_count > 0)) ++bad;
    // split phase (MpiRank::begin_ / end_update_ghost_values): post, work on
    // the owned interior meanwhile, wait -- the same ghost entries, bit for bit
    std::vector<double> split(local.size(), -1.0);
    for (int64_t i = 0; i < owned; ++i) split[plan.owned_offset + i] = (double)(g0 + i);
    GDM::HIP::PlaneRequests req;
    GDM::HIP::post_planes(plan, MPI_COMM_WORLD, split.data() + plan.send_below_offset,
                          split.data() + plan.send_above_offset, split.data() + plan.recv_below_offset,
                          split.data() + plan.recv_above_offset, req);
    double interior = 0.0;
    for (int64_t i = 0; i < owned; ++i) interior += split[plan.owned_offset + i];
    req.wait();
    bad += interior != interior;  // (keeps the overlapped work)
    for (std::size_t i = 0; i < local.size(); ++i) bad += split[i] != local[i];
    GDM::HIP::MpiRank comm(MPI_COMM_WORLD, mesh);
    const double s = comm.sum(rank + 1.0), m = comm.max(rank + 0.5);
    bad += s != size * (size + 1) / 2.0;
    bad += m != size - 0.5;
  } catch (const std::exception &e) {
    std::fprintf(stderr, "rank %d: %s\n", rank, e.what());
    bad = 1;
  }
  int total = 0;
  MPI_Allreduce(&bad, &total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  if (rank == 0) std::printf(total == 0 ? "ok\n" : "FAILED (%d)\n", total);
  MPI_Finalize();
  return total == 0 ? 0 : 1;
}
