// wave_app.cc -- the uncut wave-rk driver on the MI355X engine, written against
// the C++ mirror of the reference's wave operator surface (gdm/hip/wave.h), in
// the shape of applications/wave/wave-app.cc:222-285 + problem.h:280-346.
//
//   wave_app DIM P N STEPS CFL OUT [NITSCHE] [DEVICE]
//
// Box [-1.21, 1.21]^dim, initial displacement u0 = prod_d cos(0.75 pi x_d /
// 1.21 + 0.2 d), v0 = 0, natural boundary (NITSCHE = 0) or box Nitsche with
// gamma_D = NITSCHE.  Writes u then v after STEPS RK4 steps to OUT (raw
// little-endian doubles, reference global order).
#include <gdm/hip/wave.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>

namespace {

const double kPi = 3.14159265358979323846;

template <int dim>
int run(int p, int n, int steps, double cfl, const char *out, double nitsche, int device) {
  GDM::HIP::Wave::Parameters<dim> params;
  params.fe_degree = p;
  params.n_subdivisions_1D = n;
  params.nitsche_parameter = nitsche;
  params.exact_solution = [](const GDM::HIP::Point &x, double) {
    double v = 1.0;
    for (int d = 0; d < dim; ++d) v *= std::cos(0.75 * kPi * x[d] / 1.21 + 0.2 * d);
    return v;
  };
  params.cfl = cfl;
  params.end_t = 1e9;
  params.device = device;
  GDM::HIP::Wave::WaveProblem<dim> problem(params);
  const unsigned int done = problem.run(steps);
  std::vector<double> u = problem.get_solution();
  const std::vector<double> v = problem.get_velocity();
  double s = 0.0;
  for (double x : u) s += x * x;
  std::printf("steps %u  |u|_2 %.15e\n", done, std::sqrt(s));
  u.insert(u.end(), v.begin(), v.end());
  std::ofstream f(out, std::ios::binary);
  f.write(reinterpret_cast<const char *>(u.data()), sizeof(double) * u.size());
  return f.good() ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: %s DIM P N STEPS CFL OUT [NITSCHE] [DEVICE]\n", argv[0]);
    return 2;
  }
  const int dim = std::atoi(argv[1]), p = std::atoi(argv[2]), n = std::atoi(argv[3]), steps = std::atoi(argv[4]);
  const double cfl = std::atof(argv[5]);
  const double nitsche = argc > 7 ? std::atof(argv[7]) : 0.0;
  const int device = argc > 8 ? std::atoi(argv[8]) : 0;
  try {
    switch (dim) {
      case 1: return run<1>(p, n, steps, cfl, argv[6], nitsche, device);
      case 2: return run<2>(p, n, steps, cfl, argv[6], nitsche, device);
      case 3: return run<3>(p, n, steps, cfl, argv[6], nitsche, device);
      default: std::fprintf(stderr, "dim must be 1, 2 or 3\n"); return 2;
    }
  } catch (const GDM::HIP::Error &e) {
    std::fprintf(stderr, "GDM::HIP::Error: %s\n", e.what());
    return 1;
  }
}
