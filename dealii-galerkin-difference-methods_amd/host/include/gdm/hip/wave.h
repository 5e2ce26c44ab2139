// gdm/hip/wave.h -- C++ host mirror of the reference's wave application
// operator surface over the C ABI (include/gdm_hip.h), uncut configuration.
//
// Same class and method names, argument meaning and error behaviour as the
// reference (paths relative to peterrum/dealii-galerkin-difference-methods):
//   Parameters<dim>              applications/wave/include/gdm/wave/parameters.h:7-52
//   StiffnessMatrixOperator<dim> .../wave/stiffness.h:18-420
//     compute_rhs(dst, src, compute_impl_part, time)   :409-420
//   MassMatrixOperator<dim>      .../wave/mass.h:18-250 (get_sparse_matrix / solve)
//   WaveProblem<dim>             .../wave/problem.h:22-346, "wave-rk" branch :280-346
// The level set contains the box (no cut cells): the volume term
// -(grad v, grad u), and with function_domain_dbc the box Nitsche terms
// (gamma_D / h, :261-330); the right-hand-side function and the Dirichlet
// data are zero (the uncut C4 configuration of BASELINE.json).
#pragma once

#include <gdm/hip/operators.h>

namespace GDM {
namespace HIP {
namespace Wave {

template <int dim>
struct Parameters {
  unsigned int fe_degree = 3;
  unsigned int n_subdivisions_1D = 40;
  double geometry_left = -1.21;
  double geometry_right = 1.21;
  double nitsche_parameter = 0.0;  // > 0: box Nitsche (function_domain_dbc with g = 0)
  Function exact_solution;         // initial condition u(x, 0)
  double start_t = 0.0;
  double end_t = 2.0;
  double cfl = 0.3;
  double cfl_pow = 1.0;
  int device = 0;
  int n_ranks = 1, rank = 0;
};

template <int dim>
class Discretization {
 public:
  void reinit(const Parameters<dim> &params) {
    desc = gdm_mesh_desc{};
    desc.dim = dim;
    desc.fe_degree = (int)params.fe_degree;
    for (int d = 0; d < 3; ++d) {
      desc.n_subdivisions[d] = d < dim ? (int)params.n_subdivisions_1D : 1;
      desc.lo[d] = d < dim ? params.geometry_left : 0.0;
      desc.hi[d] = d < dim ? params.geometry_right : 1.0;
    }
    desc.n_ranks = params.n_ranks;
    desc.rank = params.rank;
    device = params.device;
  }
  double get_dx() const { return (desc.hi[0] - desc.lo[0]) / desc.n_subdivisions[0]; }  // discretization.h:53
  const gdm_mesh_desc &get_mesh() const { return desc; }
  int get_device() const { return device; }

 private:
  gdm_mesh_desc desc{};
  int device = 0;
};

using VectorType = DeviceVector;  // LinearAlgebra::distributed::Vector<double>, local layout

template <int dim>
class StiffnessMatrixOperator {
 public:
  explicit StiffnessMatrixOperator(const Discretization<dim> &discretization) : discretization(discretization) {}
  StiffnessMatrixOperator(const StiffnessMatrixOperator &) = delete;
  ~StiffnessMatrixOperator() { gdm_op_destroy(op); }

  void reinit(const Parameters<dim> &params) {
    gdm_op_destroy(op);
    op = nullptr;
    const double nitsche = params.nitsche_parameter;
    check(gdm_op_create(&discretization.get_mesh(), GDM_OP_WAVE, nitsche > 0 ? &nitsche : nullptr,
                        nitsche > 0 ? 1 : 0, discretization.get_device(), &op),
          "gdm_op_create");
    check(gdm_op_layout(op, &layout), "gdm_op_layout");
    check(gdm_op_set_stream(op, nullptr), "gdm_op_set_stream");
  }

  void initialize_dof_vector(VectorType &vec) const { vec.reinit(op, layout.n_local); }

  // vec_rhs (owned entries) = -(grad v, grad u) [+ box Nitsche] if
  // compute_impl_part; the right-hand-side and Dirichlet-data terms vanish
  // (f = 0, g = 0), so the explicit part is zero (stiffness.h:409-420)
  void compute_rhs(VectorType &vec_rhs, const VectorType &solution, const bool compute_impl_part,
                   const double /*time*/) const {
    if (compute_impl_part)
      check(gdm_apply(op, solution.get_values(), owned(vec_rhs), nullptr), "gdm_apply");
    else
      check(gdm_vec_axpby(op, layout.n_owned, 0.0, owned(vec_rhs), 0.0, owned(vec_rhs)), "gdm_vec_axpby");
  }

  gdm_op *handle() const { return op; }
  const gdm_layout &get_layout() const { return layout; }
  double *owned(VectorType &v) const { return v.get_values() + layout.ghost_planes_below * layout.plane_size; }
  const double *owned(const VectorType &v) const {
    return v.get_values() + layout.ghost_planes_below * layout.plane_size;
  }

 private:
  const Discretization<dim> &discretization;
  gdm_op *op = nullptr;
  gdm_layout layout{};
};

template <int dim>
class MassMatrixOperator {
 public:
  explicit MassMatrixOperator(const Discretization<dim> &discretization) : discretization(discretization) {}
  MassMatrixOperator(const MassMatrixOperator &) = delete;
  ~MassMatrixOperator() { gdm_op_destroy(op); }
  void reinit(const Parameters<dim> &) {
    gdm_op_destroy(op);
    op = nullptr;
    check(gdm_op_create(&discretization.get_mesh(), GDM_OP_MASS, nullptr, 0, discretization.get_device(), &op),
          "gdm_op_create");
    check(gdm_op_layout(op, &layout), "gdm_op_layout");
    check(gdm_op_set_stream(op, nullptr), "gdm_op_set_stream");
  }
  // WaveProblem::solve (problem.h:471-502): the AMG / ILU CG replaced by the
  // exact Kronecker inverse
  void solve(double *x_owned, const double *rhs_owned) const {
    check(gdm_mass_solve(op, rhs_owned, x_owned), "gdm_mass_solve");
  }
  void vmult(double *dst_owned, const double *src_local) const {
    check(gdm_mass_apply(op, src_local, dst_owned), "gdm_mass_apply");
  }
  std::size_t m() const { return (std::size_t)layout.n_dofs_global; }

 private:
  const Discretization<dim> &discretization;
  gdm_op *op = nullptr;
  gdm_layout layout{};
};

// WaveProblem<dim>::run, "wave-rk" (problem.h:280-346): y = (u, v),
// du/dt = v, dv/dt = M^-1 compute_rhs(u, true, t), RK_CLASSIC_FOURTH_ORDER,
// DiscreteTime(start, end, cfl dx^cfl_pow), device-resident in low-storage
// form (gdm_vec_rk_update).
template <int dim>
class WaveProblem {
 public:
  explicit WaveProblem(const Parameters<dim> &params)
      : params(params), mass_matrix_operator(discretization), stiffness_matrix_operator(discretization) {}

  unsigned int run(unsigned int max_steps = ~0u) {
    if (params.n_ranks != 1) throw Error("WaveProblem: the host RK driver is single-rank");
    discretization.reinit(params);
    mass_matrix_operator.reinit(params);
    stiffness_matrix_operator.reinit(params);
    const double delta_t = params.cfl * std::pow(discretization.get_dx(), params.cfl_pow);  // problem.h:284
    for (auto *v : {&u, &v_, &acc_u, &acc_v, &Yu, &Yv, &kv}) stiffness_matrix_operator.initialize_dof_vector(*v);
    set_initial_condition(u);
    DiscreteTime time(params.start_t, params.end_t, delta_t);
    unsigned int n = 0;
    while (!time.is_at_end() && n < max_steps) {
      const double t0 = time.get_current_time(), h = time.get_next_step_size();
      const DeviceVector *su = &u, *sv = &v_;
      for (int s = 0; s < 4; ++s) {
        // k = (stage v, M^-1 compute_rhs(stage u))   (problem.h:303-318)
        stiffness_matrix_operator.compute_rhs(kv, *su, true, t0 + ClassicRK4::c[s] * h);
        double *r = stiffness_matrix_operator.owned(kv);
        mass_matrix_operator.solve(r, r);
        // u block first: its k is the stage v, which the v update overwrites
        rk4_stage_update(s, h, *sv, u, acc_u, Yu);
        rk4_stage_update(s, h, kv, v_, acc_v, Yv);
        su = &Yu;
        sv = &Yv;
      }
      time.advance_time();
      ++n;
    }
    return n;
  }

  std::vector<double> get_solution() const { return u.download(); }
  std::vector<double> get_velocity() const { return v_.download(); }

 private:
  void set_initial_condition(DeviceVector &vec) const {  // VectorTools::interpolate: vertex values
    const gdm_mesh_desc &m = discretization.get_mesh();
    const gdm_layout &L = stiffness_matrix_operator.get_layout();
    std::vector<double> h(L.n_local);
    const int64_t N0 = m.n_subdivisions[0] + 1, N1 = dim > 1 ? m.n_subdivisions[1] + 1 : 1;
    const int64_t first_plane = L.owned_plane_begin - L.ghost_planes_below;
    for (int64_t i = 0; i < L.n_local; ++i) {
      const int64_t g = first_plane * L.plane_size + i;
      const int64_t id[3] = {g % N0, (g / N0) % N1, g / (N0 * N1)};
      Point x{0.0, 0.0, 0.0};
      for (int d = 0; d < dim; ++d) {
        const int64_t k = dim == 1 ? g : (dim == 2 ? (d == 0 ? g % N0 : g / N0) : id[d]);
        x[d] = m.lo[d] + k * (m.hi[d] - m.lo[d]) / m.n_subdivisions[d];
      }
      h[i] = params.exact_solution ? params.exact_solution(x, params.start_t) : 0.0;
    }
    vec.upload(h);
  }

  Parameters<dim> params;
  Discretization<dim> discretization;
  MassMatrixOperator<dim> mass_matrix_operator;
  StiffnessMatrixOperator<dim> stiffness_matrix_operator;
  DeviceVector u, v_, acc_u, acc_v, Yu, Yv, kv;
};

}  // namespace Wave
}  // namespace HIP
}  // namespace GDM
