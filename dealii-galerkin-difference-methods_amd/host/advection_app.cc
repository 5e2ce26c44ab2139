// advection_app.cc -- the uncut advection driver on the MI355X engine, written
// against the C++ mirror of the reference's operator surface
// (gdm/hip/operators.h), in the shape of
// applications/advection/advection-app.cc:86-154 + problem.h:31-102.
//
//   advection_app DIM P N STEPS CFL OUT [DEVICE] [DEVBC]
//
// Manufactured solution u(x, t) = prod_d sin(2 pi (x_d - a_d t) + 0.3 d) on
// [0, 1]^dim with a = (1, 0.15, -0.05) (prototypes/advection_01_gdm.cc:37-41);
// inflow data and block(0) evolution from u and du/dt.  Writes the owned DoF
// values after STEPS RK4 steps to OUT (raw little-endian doubles, reference
// global order) and prints one line per step with |u|_2.  DEVBC = 1 evaluates
// g and dg/dt on the device (GDM_FN_SINE_PRODUCT with the same parameters)
// instead of the host callbacks.
#include <gdm/hip/operators.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>

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

template <int dim>
int run(int p, int n, int steps, double cfl, const char *out, int device, int devbc) {
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
  GDM::HIP::AdvectionProblem<dim> problem(params);
  const unsigned int done = problem.run(steps);
  const std::vector<double> u = problem.get_solution();
  double s = 0.0;
  for (double v : u) s += v * v;
  std::printf("steps %u  |u|_2 %.15e\n", done, std::sqrt(s));
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
  try {
    switch (dim) {
      case 1: return run<1>(p, n, steps, cfl, argv[6], device, devbc);
      case 2: return run<2>(p, n, steps, cfl, argv[6], device, devbc);
      case 3: return run<3>(p, n, steps, cfl, argv[6], device, devbc);
      default: std::fprintf(stderr, "dim must be 1, 2 or 3\n"); return 2;
    }
  } catch (const GDM::HIP::Error &e) {
    std::fprintf(stderr, "GDM::HIP::Error: %s\n", e.what());
    return 1;
  }
}
