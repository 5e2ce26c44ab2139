// advection_app.cc -- the uncut advection driver on the MI355X engine, written
// against the C++ mirror of the reference's operator surface
// (gdm/hip/operators.h), in the shape of
// applications/advection/advection-app.cc:86-154 + problem.h:31-102.
//
//   advection_app DIM P N STEPS CFL OUT [DEVICE] [DEVBC] [NRANKS] [EXCHANGES]
//
// Manufactured solution u(x, t) = prod_d sin(2 pi (x_d - a_d t) + 0.3 d) on
// [0, 1]^dim with a = (1, 0.15, -0.05) (prototypes/advection_01_gdm.cc:37-41);
// inflow data and block(0) evolution from u and du/dt.  Writes the owned DoF
// values after STEPS RK4 steps to OUT (raw little-endian doubles, reference
// global order) and prints one line per step with |u|_2.  DEVBC = 1 evaluates
// g and dg/dt on the device (GDM_FN_SINE_PRODUCT with the same parameters)
// instead of the host callbacks, with the stage values of block(0) evaluated
// by the engine per stage (Parameters::boundary_in_faces); DEVBC = 2 the same
// function with block(0) stored and RK-updated.  NRANKS > 1 runs the multi-rank path: one
// thread per rank (z-slabs of system.h:720-757, all on DEVICE), ghost planes
// and dots through GDM::HIP::ThreadGroup (an MPI communicator's role), the
// distributed exact mass inverse (SPIKE) when the slabs are thick enough, else
// the distributed Jacobi CG; OUT holds the ranks' owned values in rank order.
// EXCHANGES (SPIKE runs): 1 = one ghost exchange per RK stage (default,
// Parameters::one_exchange_per_stage), 2 = the reference's two.
// With DEVBC the final errors against the exact solution are computed on the
// device (AdvectionProblem::postprocess -> gdm_error_norms) and printed in the
// reference's postprocess format (time, L2, L1, Linf).
#include <gdm/hip/operators.h>
#include <gdm/hip/thread_communicator.h>

#include <array>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <thread>

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

// time after `steps` steps of DiscreteTime(0, 1, dx cfl / max_val), max_val = 1
double time_of(unsigned int steps, int n, double cfl) {
  GDM::HIP::DiscreteTime t(0.0, 1.0, (1.0 / n) * cfl);
  for (unsigned int i = 0; i < steps && !t.is_at_end(); ++i) t.advance_time();
  return t.get_current_time();
}

template <int dim>
GDM::HIP::Parameters<dim> make_params(int p, int n, double cfl, int device, int devbc) {
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
    params.boundary_in_faces = devbc != 2;
  }
  return params;
}

template <int dim>
int run(int p, int n, int steps, double cfl, const char *out, int device, int devbc, int n_ranks, int exchanges) {
  std::vector<double> u;
  unsigned int done = 0;
  std::array<double, 6> norms{{-1.0, -1.0, -1.0, 0.0, 0.0, 0.0}};
  bool spike = false, one_ex = false;
  if (n_ranks <= 1) {
    GDM::HIP::AdvectionProblem<dim> problem(make_params<dim>(p, n, cfl, device, devbc));
    done = problem.run(steps);
    u = problem.get_solution();
    if (devbc) norms = problem.postprocess(time_of(done, n, cfl));
  } else {
    gdm_mesh_desc mesh{};
    mesh.dim = dim;
    mesh.fe_degree = p;
    for (int d = 0; d < 3; ++d) {
      mesh.n_subdivisions[d] = d < dim ? n : 1;
      mesh.lo[d] = 0.0;
      mesh.hi[d] = 1.0;
    }
    mesh.n_ranks = n_ranks;
    GDM::HIP::ThreadGroup group(n_ranks);
    std::vector<gdm_halo> plans(n_ranks);
    for (int r = 0; r < n_ranks; ++r) {
      mesh.rank = r;
      GDM::HIP::check(gdm_halo_plan(&mesh, &plans[r]), "gdm_halo_plan");
    }
    group.set_plans(plans);
    std::vector<std::vector<double>> parts(n_ranks);
    std::vector<std::string> errors(n_ranks);
    std::vector<unsigned int> steps_done(n_ranks, 0);
    std::vector<std::thread> threads;
    for (int r = 0; r < n_ranks; ++r)
      threads.emplace_back([&, r] {
        try {
          GDM::HIP::Parameters<dim> params = make_params<dim>(p, n, cfl, device, devbc);
          params.n_ranks = n_ranks;
          params.rank = r;
          params.one_exchange_per_stage = exchanges != 2;
          GDM::HIP::ThreadGroup::Rank comm(group, r, mesh);
          GDM::HIP::AdvectionProblem<dim> problem(params, &comm);
          steps_done[r] = problem.run(steps);
          parts[r] = problem.get_solution();
          if (devbc) {
            const std::array<double, 6> e = problem.postprocess(time_of(steps_done[r], n, cfl));
            if (r == 0) norms = e;
          }
          if (r == 0) spike = problem.used_spike_solve();
          if (r == 0) one_ex = problem.used_one_exchange();
        } catch (const std::exception &e) {
          errors[r] = e.what();
          std::fprintf(stderr, "rank %d: %s\n", r, e.what());
          std::_Exit(1);  // a failed rank would leave the others blocked in a barrier
        }
      });
    for (auto &t : threads) t.join();
    for (int r = 0; r < n_ranks; ++r) u.insert(u.end(), parts[r].begin(), parts[r].end());
    done = steps_done[0];
  }
  double s = 0.0;
  for (double v : u) s += v * v;
  std::printf("steps %u  |u|_2 %.15e\n", done, std::sqrt(s));
  if (n_ranks > 1) std::printf("mass solve: %s\n", spike ? "spike" : "cg");
  if (n_ranks > 1) std::printf("exchanges per stage: %d\n", one_ex ? 1 : 2);
  if (devbc)  // the reference's postprocess line (problem.h:427-433): counter, time, L2, L1, Linf
    std::printf("%5d %8.5f %14.8e %14.8e %14.8e\n", 0, time_of(done, n, cfl), norms[2], norms[1], norms[0]);
  std::ofstream f(out, std::ios::binary);
  f.write(reinterpret_cast<const char *>(u.data()), sizeof(double) * u.size());
  return f.good() ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: %s DIM P N STEPS CFL OUT [DEVICE]\n", argv[0]);
    return 2;
  }
  const int dim = std::atoi(argv[1]), p = std::atoi(argv[2]), n = std::atoi(argv[3]), steps = std::atoi(argv[4]);
  const double cfl = std::atof(argv[5]);
  const int device = argc > 7 ? std::atoi(argv[7]) : 0;
  const int devbc = argc > 8 ? std::atoi(argv[8]) : 0;
  const int n_ranks = argc > 9 ? std::atoi(argv[9]) : 1;
  const int exchanges = argc > 10 ? std::atoi(argv[10]) : 1;
  try {
    switch (dim) {
      case 1: return run<1>(p, n, steps, cfl, argv[6], device, devbc, n_ranks, exchanges);
      case 2: return run<2>(p, n, steps, cfl, argv[6], device, devbc, n_ranks, exchanges);
      case 3: return run<3>(p, n, steps, cfl, argv[6], device, devbc, n_ranks, exchanges);
      default: std::fprintf(stderr, "dim must be 1, 2 or 3\n"); return 2;
    }
  } catch (const GDM::HIP::Error &e) {
    std::fprintf(stderr, "GDM::HIP::Error: %s\n", e.what());
    return 1;
  }
}
