// gdm/hip/cut_wave.h -- C++ host mirror of the reference's wave application
// (applications/wave) over the "Cut-cell wave" entry points of the C ABI
// (include/gdm_hip.h): the same parameter sets, simulation types and
// postprocess table, every operator in libgdm_hip.so.
//
//   Parameters<dim>       applications/wave/include/gdm/wave/parameters.h:7-52
//   fill_parameters       applications/wave/wave-app.cc:9-347 (step85, heat /
//                         heat-rk / heat-impl, heat-composite, wave,
//                         wave-composite)
//   WaveProblem<dim>::run .../wave/problem.h:39-440: poisson (one stiffness
//                         solve), heat-rk / wave-rk (RK_CLASSIC_FOURTH_ORDER +
//                         DiscreteTime, composite or not), heat-impl (backward
//                         Euler), postprocess (:504-615, the reference's printf)
//
// Level set, right-hand side, interface / domain Dirichlet data and exact
// solution are host functions (the reference's Function objects), evaluated
// at the points the library reports and uploaded per stage; the FE_Q(k)
// level set is handed over as its values at each cell's Gauss-Lobatto points.
// The reference's "[L] solved in N" lines (iteration counts of its AMG / ILU
// preconditioned CG) have no counterpart: the library's solves are exact
// banded Cholesky solves.  Errors throw GDM::HIP::Error; no CPU fallback.
#pragma once

#include <gdm/hip/operators.h>

#include <cmath>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace GDM {
namespace HIP {
namespace CutWave {

// f(x, t) with x[dim]
using Function = std::function<double(const double *, double)>;

template <int dim>
struct Parameters {
  std::string simulation_type;
  unsigned int fe_degree = 3;
  bool composite = false;
  unsigned int n_subdivisions_1D = 40;
  double geometry_left = -1.21, geometry_right = 1.21;
  double ghost_parameter_M = -1.0, ghost_parameter_A = -1.0, nitsche_parameter = -1.0;
  Function function_domain_dbc, function_interface_dbc, function_rhs, exact_solution;
  double start_t = 0.0, end_t = 0.0, cfl = 0.0, cfl_pow = 1.0;
  unsigned int level_set_fe_degree = 3;
  std::function<double(const double *)> level_set_function;
};

template <int dim>
double norm(const double *x) {
  double s = 0.0;
  for (int d = 0; d < dim; ++d) s += x[d] * x[d];
  return std::sqrt(s);
}

// wave-app.cc fill_parameters
template <int dim>
void fill_parameters(Parameters<dim> &params, const std::string &name) {
  static_assert(dim == 1 || dim == 2, "the reference's wave application runs dim 1 and 2");
  params.level_set_function = [](const double *x) { return norm<dim>(x) - 1.0; };  // SignedDistance::Sphere
  params.fe_degree = params.level_set_fe_degree = 3;
  params.n_subdivisions_1D = 40;
  params.geometry_left = -1.21;
  params.geometry_right = 1.21;
  params.nitsche_parameter = 5.0 * params.fe_degree;
  auto heat_exact = [](const double *x, double t) {
    return dim == 1 ? std::pow(x[0], 9.0) * std::exp(-t) : std::pow(x[0], 9.0) * std::pow(x[1], 8.0) * std::exp(-t);
  };
  auto heat_rhs = [](const double *x, double t) {
    if (dim == 1) return -std::pow(x[0], 7.0) * std::exp(-t) * (std::pow(x[0], 2.0) + 72);
    return -std::pow(x[0], 7.0) * std::pow(x[1], 6.0) * std::exp(-t) *
           (std::pow(x[0], 2.0) * std::pow(x[1], 2.0) + 72 * std::pow(x[1], 2.0) + 56 * std::pow(x[0], 2.0));
  };
  auto wave_exact = [](const double *x, double t) {
    const double r = norm<dim>(x);
    if (dim == 1) {
      const double k = 1.5 * M_PI;
      return std::cos(k * r) * std::cos(k * t);
    }
    const double k = 3.0 * M_PI;
    return std::cyl_bessel_j(0.0, k * r) * std::cos(k * t);
  };
  if (name == "step85") {
    params.simulation_type = "poisson";
    params.ghost_parameter_M = -1.0;
    params.ghost_parameter_A = 0.5;
    params.function_interface_dbc = [](const double *, double) { return 1.0; };
    params.function_rhs = [](const double *, double) { return 4.0; };
    params.exact_solution = [](const double *x, double) { return 1. - 2. / dim * (norm<dim>(x) * norm<dim>(x) - 1.); };
    params.start_t = 0.0;
    params.end_t = 0.1;
    params.cfl = 0.3;
    params.cfl_pow = 1.0;
  } else if (name == "heat" || name == "heat-rk" || name == "heat-impl" || name == "heat-composite") {
    const bool composite = name == "heat-composite";
    params.simulation_type = (name == "heat") ? std::string("heat-impl") : composite ? "heat-rk" : name;
    params.composite = composite;
    params.ghost_parameter_M = 0.75;
    params.ghost_parameter_A = 1.5;
    (composite ? params.function_domain_dbc : params.function_interface_dbc) = heat_exact;
    params.function_rhs = heat_rhs;
    params.exact_solution = heat_exact;
    params.start_t = 0.0;
    params.end_t = 0.1;
    if (params.simulation_type == "heat-rk") {
      params.cfl = 0.3 / params.fe_degree / params.fe_degree;
      params.cfl_pow = 2.0;
    } else {
      params.cfl = 0.3;
      params.cfl_pow = 1.0;
    }
  } else if (name == "wave" || name == "wave-composite") {
    const bool composite = name == "wave-composite";
    params.simulation_type = "wave-rk";
    params.composite = composite;
    params.ghost_parameter_M = 0.25 * std::sqrt(3.0);
    params.ghost_parameter_A = 0.50 * std::sqrt(3.0);
    (composite ? params.function_domain_dbc : params.function_interface_dbc) = wave_exact;
    params.function_rhs = {};
    params.exact_solution = wave_exact;
    params.start_t = 0.0;
    params.end_t = 2.0;
    params.cfl = 0.3;
    params.cfl_pow = 1.0;
  } else {
    throw Error("fill_parameters: unknown simulation " + name);
  }
}

// Gauss-Lobatto points of n >= 2 points on [0, 1] (the FE_Q support points)
inline std::vector<double> gauss_lobatto(int n) {
  std::vector<double> x(n);
  x[0] = 0.0;
  x[n - 1] = 1.0;
  const int m = n - 1;
  for (int i = 1; i < m; ++i) {
    double t = -std::cos(M_PI * i / m);
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = t;
      for (int j = 2; j <= m; ++j) {
        const double p2 = ((2 * j - 1) * t * p1 - (j - 1) * p0) / j;
        p0 = p1;
        p1 = p2;
      }
      const double dp = m * (t * p1 - p0) / (t * t - 1.0), d2p = (2.0 * t * dp - m * (m + 1) * p1) / (1.0 - t * t);
      t -= dp / d2p;
      if (std::fabs(dp / d2p) < 1e-16) break;
    }
    x[i] = 0.5 * (t + 1.0);
  }
  return x;
}

// one field (location inside / outside) of the problem: the device handle and its points
template <int dim>
class Field {
 public:
  Field(const Parameters<dim> &P, int location, int flags, int device) {
    const int n = (int)P.n_subdivisions_1D, k = (int)P.level_set_fe_degree;
    const double h = (P.geometry_right - P.geometry_left) / n;
    const std::vector<double> gl = gauss_lobatto(k + 1);
    std::vector<double> ls;
    double x[2] = {0.0, 0.0};
    if (dim == 1) {
      for (int c = 0; c < n; ++c)
        for (int a = 0; a <= k; ++a) {
          x[0] = (P.geometry_left + c * h) + gl[a] * h;
          ls.push_back(P.level_set_function(x));
        }
    } else {
      for (int cy = 0; cy < n; ++cy)
        for (int cx = 0; cx < n; ++cx)
          for (int b = 0; b <= k; ++b)
            for (int a = 0; a <= k; ++a) {
              x[0] = (P.geometry_left + cx * h) + gl[a] * h;
              x[1] = (P.geometry_left + cy * h) + gl[b] * h;
              ls.push_back(P.level_set_function(x));
            }
    }
    check(gdm_cut_wave_create(dim, (int)P.fe_degree, n, P.geometry_left, P.geometry_right, k, ls.data(), location,
                              flags, P.ghost_parameter_M, P.ghost_parameter_A, P.nitsche_parameter, device, &c_),
          "gdm_cut_wave_create");
    int64_t cells[3];
    check(gdm_cut_wave_info(c_, &n_dofs, &n_quad, &n_data, cells), "gdm_cut_wave_info");
    qx.resize((size_t)std::max<int64_t>(n_quad, 1) * dim);
    qw.resize((size_t)std::max<int64_t>(n_quad, 1));
    sx.resize((size_t)std::max<int64_t>(n_data, 1) * dim);
    std::vector<double> sn(sx.size());
    check(gdm_cut_wave_points(c_, qx.data(), qw.data(), sx.data(), sn.data()), "gdm_cut_wave_points");
    check(gdm_cut_wave_op(c_, &op_), "gdm_cut_wave_op");
    fq.reinit(op_, (size_t)std::max<int64_t>(n_quad, 1));
    gs.reinit(op_, (size_t)std::max<int64_t>(n_data, 1));
    vals.reinit(op_, (size_t)std::max<int64_t>(n_quad, 1));
    h_ = h;
  }
  ~Field() {
    fq = DeviceVector();
    gs = DeviceVector();
    vals = DeviceVector();
    gdm_cut_wave_destroy(c_);
  }
  Field(const Field &) = delete;
  Field &operator=(const Field &) = delete;

  gdm_op *op() const { return op_; }
  gdm_cut_wave *handle() const { return c_; }
  double h() const { return h_; }

  // upload f at the quadrature points / g at the data points; NULL pointers when absent
  const double *rhs_data(const Function &f, double t) {
    if (!f || n_quad == 0) return nullptr;
    std::vector<double> v((size_t)n_quad);
    for (int64_t q = 0; q < n_quad; ++q) v[(size_t)q] = f(&qx[(size_t)q * dim], t);
    upload_prefix(fq, v);
    return fq.get_values();
  }
  const double *dirichlet_data(const Function &g, double t) {
    if (!g || n_data == 0) return nullptr;
    std::vector<double> v((size_t)n_data);
    for (int64_t q = 0; q < n_data; ++q) v[(size_t)q] = g(&sx[(size_t)q * dim], t);
    upload_prefix(gs, v);
    return gs.get_values();
  }
  // (L2, L1, Linf) of u_h - exact over the field's quadrature (problem.h:504-615)
  std::array<double, 3> errors(const DeviceVector &u, const Function &exact, double t) {
    check(gdm_cut_wave_eval(c_, u.get_values(), vals.get_values()), "gdm_cut_wave_eval");
    const std::vector<double> uh = vals.download();
    double l2 = 0.0, l1 = 0.0, linf = 0.0;
    for (int64_t q = 0; q < n_quad; ++q) {
      const double e = uh[(size_t)q] - exact(&qx[(size_t)q * dim], t);
      l2 += e * e * qw[(size_t)q];
      l1 += std::fabs(e) * qw[(size_t)q];
      linf = std::max(linf, std::fabs(e));
    }
    return {std::sqrt(l2), l1, linf};
  }

  int64_t n_dofs = 0, n_quad = 0, n_data = 0;

 private:
  void upload_prefix(DeviceVector &d, const std::vector<double> &v) {
    if (!v.empty()) check(gdm_memcpy_h2d(op_, d.get_values(), v.data(), sizeof(double) * v.size()), "gdm_memcpy_h2d");
  }
  gdm_cut_wave *c_ = nullptr;
  gdm_op *op_ = nullptr;
  std::vector<double> qx, qw, sx;
  DeviceVector fq, gs, vals;
  double h_ = 0.0;
};

struct Row {
  int counter;
  double time, l2, l1, linf;
};

template <int dim>
class WaveProblem {
 public:
  explicit WaveProblem(const Parameters<dim> &params, int device = 0, bool print = true)
      : P(params), device_(device), print_(print) {}

  std::vector<Row> run() {
    const bool comp = P.composite;
    const int flags = comp ? (GDM_CUT_WAVE_DOMAIN_DATA | GDM_CUT_WAVE_COUPLED) : GDM_CUT_WAVE_INTERFACE_DATA;
    std::vector<std::unique_ptr<Field<dim>>> F;
    F.emplace_back(new Field<dim>(P, GDM_CUT_INSIDE, flags, device_));
    if (comp) {
      F.emplace_back(new Field<dim>(P, GDM_CUT_OUTSIDE, flags, device_));
      // both fields' operators and the block updates on one stream (the HIP null stream): the coupling reads the
      // partner's stage vector
      for (auto &f : F) check(gdm_op_set_stream(f->op(), nullptr), "gdm_op_set_stream");
    }
    gdm_op *op = F[0]->op();
    const size_t N = (size_t)F[0]->n_dofs;
    const Function &dbc = comp ? P.function_domain_dbc : P.function_interface_dbc;
    rows_.clear();
    counter_[0] = counter_[1] = 0;
    DeviceVector r(op, N);

    // compute_rhs (+ coupling) and the mass solve of field i at time t
    auto accel = [&](size_t i, double t, const DeviceVector &u, const DeviceVector *u_other, DeviceVector &k) {
      Field<dim> &f = *F[i];
      check(gdm_cut_wave_compute_rhs(f.handle(), u.get_values(), f.rhs_data(P.function_rhs, t),
                                     f.dirichlet_data(dbc, t), k.get_values()),
            "gdm_cut_wave_compute_rhs");
      if (u_other) check(gdm_cut_wave_couple(f.handle(), u_other->get_values(), k.get_values()), "gdm_cut_wave_couple");
      check(gdm_cut_wave_mass_solve(f.handle(), k.get_values(), k.get_values()), "gdm_cut_wave_mass_solve");
    };

    if (P.simulation_type == "poisson") {
      DeviceVector u(op, N);
      Field<dim> &f = *F[0];
      check(gdm_cut_wave_compute_rhs(f.handle(), nullptr, f.rhs_data(P.function_rhs, 0.0),
                                     f.dirichlet_data(dbc, 0.0), r.get_values()),
            "gdm_cut_wave_compute_rhs");
      check(gdm_cut_wave_stiffness_solve(f.handle(), r.get_values(), u.get_values()), "gdm_cut_wave_stiffness_solve");
      postprocess(f, 0.0, u, 0);
      return rows_;
    }

    const double h = F[0]->h(), dt = P.cfl * std::pow(h, P.cfl_pow);
    DiscreteTime time(P.start_t, P.end_t, dt);
    // blocks: (u_0 [, u_1]) for heat, (u_0 [, u_1], v_0 [, v_1]) for wave
    const size_t nf = F.size(), nb = P.simulation_type == "wave-rk" ? 2 * nf : nf;
    std::vector<DeviceVector> y(nb), acc(nb), Y(nb), k(nb);
    for (size_t b = 0; b < nb; ++b) {
      y[b].reinit(op, N);
      acc[b].reinit(op, N);
      Y[b].reinit(op, N);
      k[b].reinit(op, N);
    }
    {
      // GDM::VectorTools::interpolate: vertex values
      const int n1 = (int)P.n_subdivisions_1D + 1;
      std::vector<double> u0(N);
      double x[2] = {0.0, 0.0};
      for (size_t i = 0; i < N; ++i) {
        x[0] = P.geometry_left + (double)(i % n1) * h;
        if (dim == 2) x[1] = P.geometry_left + (double)(i / n1) * h;
        u0[i] = P.exact_solution(x, P.start_t);
      }
      for (size_t i = 0; i < nf; ++i) y[i].upload(u0);
    }
    for (size_t i = 0; i < nf; ++i) postprocess(*F[i], 0.0, y[i], i);

    static constexpr double A[3] = {0.5, 0.5, 1.0}, B[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6},
                            C[4] = {0.0, 0.5, 0.5, 1.0};
    while (!time.is_at_end()) {
      const double t0 = time.get_current_time(), hs = time.get_next_step_size();
      if (P.simulation_type == "heat-impl") {
        // u <- (M + dt K)^-1 (M u + dt F(t + dt))  (problem.h:218-268)
        Field<dim> &f = *F[0];
        check(gdm_cut_wave_compute_rhs(f.handle(), nullptr, f.rhs_data(P.function_rhs, t0 + hs),
                                       f.dirichlet_data(dbc, t0 + hs), r.get_values()),
              "gdm_cut_wave_compute_rhs");
        check(gdm_cut_wave_mass_apply(f.handle(), y[0].get_values(), k[0].get_values()), "gdm_cut_wave_mass_apply");
        k[0].sadd(1.0, hs, r);
        check(gdm_cut_wave_system_solve(f.handle(), hs, k[0].get_values(), y[0].get_values()),
              "gdm_cut_wave_system_solve");
      } else {
        // TimeStepping::ExplicitRungeKutta, RK_CLASSIC_FOURTH_ORDER, low-storage form
        for (int s = 0; s < 4; ++s) {
          const std::vector<DeviceVector> &st = s == 0 ? y : Y;
          const double ts = t0 + C[s] * hs;
          std::vector<const DeviceVector *> ks(nb);
          for (size_t i = 0; i < nf; ++i) {
            if (nb == nf) {  // heat: du/dt = M^-1 f(u)
              accel(i, ts, st[i], nf == 2 ? &st[1 - i] : nullptr, k[i]);
              ks[i] = &k[i];
            } else {  // wave: du/dt = v, dv/dt = M^-1 f(u)
              accel(i, ts, st[i], nf == 2 ? &st[1 - i] : nullptr, k[nf + i]);
              ks[i] = &st[nf + i];
              ks[nf + i] = &k[nf + i];
            }
          }
          const bool last = s == 3;
          // u blocks first: they read the stage v before the v blocks overwrite Y_v
          for (size_t b = 0; b < nb; ++b)
            check(gdm_vec_rk_update(op, (int64_t)N, hs * B[s], ks[b]->get_values(),
                                    (s == 0 ? y : acc)[b].get_values(), (last ? y : acc)[b].get_values(),
                                    last ? 0.0 : hs * A[s], last ? nullptr : y[b].get_values(),
                                    last ? nullptr : Y[b].get_values()),
                  "gdm_vec_rk_update");
        }
      }
      for (size_t i = 0; i < nf; ++i) postprocess(*F[i], t0 + hs, y[i], i);
      time.advance_time();
    }
    check(gdm_synchronize(op), "gdm_synchronize");
    return rows_;
  }

 private:
  void postprocess(Field<dim> &f, double t, const DeviceVector &u, size_t location) {
    const auto e = f.errors(u, P.exact_solution, t);
    const int c = counter_[location]++;
    rows_.push_back({c, t, e[0], e[1], e[2]});
    if (print_) std::printf("%5d %8.5f %14.8e %14.8e %14.8e\n", c, t, e[0], e[1], e[2]);
  }

  Parameters<dim> P;
  int device_;
  bool print_;
  std::vector<Row> rows_;
  int counter_[2] = {0, 0};
};

}  // namespace CutWave
}  // namespace HIP
}  // namespace GDM
