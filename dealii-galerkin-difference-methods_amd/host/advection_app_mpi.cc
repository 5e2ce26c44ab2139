// advection_app_mpi.cc -- advection_app with one MPI process per rank (the
// reference's parallel model: MPI_InitFinalize, advection-app.cc:160; z-slabs
// of system.h:720-757), the ghost planes and reductions through
// GDM::HIP::MpiRank (host staging) or GDM::HIP::RcclRank (device to device,
// built with GDM_WITH_RCCL).
//
//   mpirun -np R advection_app_mpi DIM P N STEPS CFL OUT [DEVBC] [COMM]
//
// COMM = mpi (default) | rccl, each optionally suffixed -blocking (exchange,
// then apply; default: the exchange overlapped with the interior planes,
// StiffnessMatrixOperator::compute_rhs_overlapped).  Rank r uses device
// r % n_devices.  Same
// manufactured solution, output and printed lines as advection_app; OUT holds
// the ranks' owned values in rank order (gathered on rank 0).
#include <gdm/hip/mpi_communicator.h>
#include <gdm/hip/operators.h>
#include <mpi.h>

#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>

namespace {

const double kA[3] = {1.0, 0.15, -0.05};
const double kPi = 3.14159265358979323846;

template <int dim>
double g(const GDM::HIP::Point &x, double t) {
  double v = 1.0;
  for (int d = 0; d < dim; ++d) v *= std::sin(2 * kPi * (x[d] - kA[d] * t) + 0.3 * d);
  return v;
}

template <int dim>
double dg_dt(const GDM::HIP::Point &x, double t) {
  double s = 0.0;
  for (int d = 0; d < dim; ++d) {
    double v = -kA[d] * 2 * kPi * std::cos(2 * kPi * (x[d] - kA[d] * t) + 0.3 * d);
    for (int e = 0; e < dim; ++e)
      if (e != d) v *= std::sin(2 * kPi * (x[e] - kA[e] * t) + 0.3 * e);
    s += v;
  }
  return s;
}

double time_of(unsigned int steps, int n, double cfl) {
  GDM::HIP::DiscreteTime t(0.0, 1.0, (1.0 / n) * cfl);
  for (unsigned int i = 0; i < steps && !t.is_at_end(); ++i) t.advance_time();
  return t.get_current_time();
}

template <int dim>
int run(int p, int n, int steps, double cfl, const char *out, int devbc, const std::string &comm_kind) {
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  int n_dev = 0;
  GDM::HIP::check(gdm_get_device_count(&n_dev), "gdm_get_device_count");
  const int device = n_dev > 0 ? rank % n_dev : 0;
  GDM::HIP::Parameters<dim> params;
  params.fe_degree = p;
  params.n_subdivisions_1D = n;
  params.geometry_left = 0.0;
  params.geometry_right = 1.0;
  params.exact_solution = g<dim>;
  params.exact_solution_der = dg_dt<dim>;
  params.start_t = 0.0;
  params.end_t = 1.0;
  params.cfl = cfl;
  params.max_val = 1.0;
  for (int d = 0; d < dim; ++d) params.advection[d] = kA[d];
  params.device = device;
  if (devbc) {
    params.boundary_function = GDM_FN_SINE_PRODUCT;
    params.boundary_function_params = {kA[0], kA[1], kA[2], 1.0, 1.0, 1.0, 0.0, 0.3, 0.6};
  }
  params.n_ranks = size;
  params.rank = rank;
  const std::string blk = "-blocking";
  std::string kind = comm_kind;
  if (kind.size() > blk.size() && kind.compare(kind.size() - blk.size(), blk.size(), blk) == 0) {
    params.overlap_exchange = false;
    kind = kind.substr(0, kind.size() - blk.size());
  }
  gdm_mesh_desc mesh{};
  mesh.dim = dim;
  mesh.fe_degree = p;
  for (int d = 0; d < 3; ++d) {
    mesh.n_subdivisions[d] = d < dim ? n : 1;
    mesh.lo[d] = 0.0;
    mesh.hi[d] = 1.0;
  }
  mesh.n_ranks = size;
  std::unique_ptr<GDM::HIP::Communicator> comm;
  if (kind == "rccl") {
#ifdef GDM_WITH_RCCL
    comm = std::make_unique<GDM::HIP::RcclRank>(MPI_COMM_WORLD, mesh, device);
#else
    throw GDM::HIP::Error("built without RCCL (GDM_WITH_RCCL)");
#endif
  } else {
    comm = std::make_unique<GDM::HIP::MpiRank>(MPI_COMM_WORLD, mesh);
  }
  GDM::HIP::AdvectionProblem<dim> problem(params, comm.get());
  const unsigned int done = problem.run(steps);
  const std::vector<double> part = problem.get_solution();
  std::array<double, 6> norms{{-1.0, -1.0, -1.0, 0.0, 0.0, 0.0}};
  if (devbc) norms = problem.postprocess(time_of(done, n, cfl));
  // gather the owned parts on rank 0 (rank order = global order of the slabs)
  int mine = (int)part.size();
  std::vector<int> counts(size), displs(size);
  MPI_Gather(&mine, 1, MPI_INT, counts.data(), 1, MPI_INT, 0, MPI_COMM_WORLD);
  std::vector<double> u;
  if (rank == 0) {
    int off = 0;
    for (int r = 0; r < size; ++r) {
      displs[r] = off;
      off += counts[r];
    }
    u.resize(off);
  }
  MPI_Gatherv(part.data(), mine, MPI_DOUBLE, u.data(), counts.data(), displs.data(), MPI_DOUBLE, 0, MPI_COMM_WORLD);
  if (rank != 0) return 0;
  double s = 0.0;
  for (double v : u) s += v * v;
  std::printf("steps %u  |u|_2 %.15e\n", done, std::sqrt(s));
  std::printf("mass solve: %s, comm: %s, ranks %d, exchange %s\n", problem.used_spike_solve() ? "spike" : "cg",
              kind.c_str(), size, params.overlap_exchange ? "overlapped" : "blocking");
  if (devbc) std::printf("%5d %8.5f %14.8e %14.8e %14.8e\n", 0, time_of(done, n, cfl), norms[2], norms[1], norms[0]);
  std::ofstream f(out, std::ios::binary);
  f.write(reinterpret_cast<const char *>(u.data()), sizeof(double) * u.size());
  return f.good() ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rc = 2;
  if (argc < 7) {
    std::fprintf(stderr, "usage: %s DIM P N STEPS CFL OUT [DEVBC] [mpi|rccl][-blocking]\n", argv[0]);
  } else {
    const int dim = std::atoi(argv[1]), p = std::atoi(argv[2]), n = std::atoi(argv[3]), steps = std::atoi(argv[4]);
    const double cfl = std::atof(argv[5]);
    const int devbc = argc > 7 ? std::atoi(argv[7]) : 0;
    const std::string kind = argc > 8 ? argv[8] : "mpi";
    try {
      switch (dim) {
        case 1: rc = run<1>(p, n, steps, cfl, argv[6], devbc, kind); break;
        case 2: rc = run<2>(p, n, steps, cfl, argv[6], devbc, kind); break;
        case 3: rc = run<3>(p, n, steps, cfl, argv[6], devbc, kind); break;
        default: std::fprintf(stderr, "dim must be 1, 2 or 3\n");
      }
    } catch (const GDM::HIP::Error &e) {
      std::fprintf(stderr, "GDM::HIP::Error: %s\n", e.what());
      MPI_Abort(MPI_COMM_WORLD, 1);
    }
  }
  MPI_Finalize();
  return rc;
}
