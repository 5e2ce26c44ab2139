// gdm/hip/operators.h -- C++ host mirror of the reference's operator surface
// over the C ABI of libgdm_hip.so (include/gdm_hip.h).
//
// Same class and method names, argument meaning and error behaviour as the
// reference (paths relative to peterrum/dealii-galerkin-difference-methods):
//   Parameters<dim>              applications/advection/include/gdm/advection/parameters.h:5-47
//   Discretization<dim>          .../advection/discretization.h:21-177
//   StiffnessMatrixOperator<dim> .../advection/stiffness.h:18-606
//     initialize_dof_vector      :162-179   (block(0) = boundary points, block(1) = solution)
//     initialize_time_step       :181-194   (block(0) <- g(t_n))
//     compute_rhs                :196-606   (block(0) = dg/dt, block(1) = K u + inflow data)
//   MassMatrixOperator<dim>      .../advection/mass.h:18-243 (vmult on the matrix-free mass)
//   AdvectionProblem<dim>        .../advection/problem.h:13-205 (RK4 + DiscreteTime + solve)
// deal.II is not needed: vectors are device buffers owned by DeviceVector, the
// mesh is the uncut subdivided hyper cube, the advection field is constant and
// the level set cuts nothing (the uncut configuration of BASELINE.json).
// Errors: every ABI failure throws GDM::HIP::Error (the reference's
// AssertThrow); there is no CPU fallback.
#pragma once

#include <gdm_hip.h>

#include <array>
#include <cmath>
#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace GDM {
namespace HIP {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void check(int rc, const char *what) {
  if (rc != GDM_OK) {
    char buf[1024];
    gdm_last_error(buf, sizeof(buf));
    throw Error(std::string(what) + ": " + buf);
  }
}

using Point = std::array<double, 3>;
using Function = std::function<double(const Point &, double)>;  // (x, t) -> value

// applications/advection/include/gdm/advection/parameters.h (uncut subset)
template <int dim>
struct Parameters {
  unsigned int fe_degree = 5;
  unsigned int n_subdivisions_1D = 40;
  double geometry_left = 0.0;
  double geometry_right = 1.0;
  Function exact_solution;      // g(x, t): initial condition and inflow data
  Function exact_solution_der;  // dg/dt(x, t): evolves block(0) (stiffness.h:286-289)
  double start_t = 0.0;
  double end_t = 0.1;
  double cfl = 0.1;
  double max_val = 1.0;                 // max |a| for the time step (problem.h:45)
  std::array<double, dim> advection{};  // constant field a
  int device = 0;
  int n_ranks = 1, rank = 0;            // z-slab partition (system.h:720-757)
  // n_ranks > 1: overlap the stage's ghost exchange with the interior planes
  // (Communicator::begin_ / end_update_ghost_values); false: exchange, then apply
  bool overlap_exchange = true;
  // Device evaluation of g / dg/dt at the boundary points (gdm_eval_boundary):
  // a gdm_fn_kind (GDM_FN_CONE = the advection app's ExactSolution,
  // advection-app.cc:51-79; GDM_FN_SINE_PRODUCT = a transported product of
  // sines) and its parameters.  -1: evaluate the host callbacks above and
  // upload (the reference's behaviour, a PCIe copy per stage).
  int boundary_function = -1;
  std::vector<double> boundary_function_params;
  // with a built-in boundary function: evaluate the stage values of block(0)
  // (g(t_n) + h a_{s,s-1} dg/dt) in the engine, per stage (gdm_apply_bc_fn /
  // gdm_add_boundary_fn) instead of storing and RK-updating block(0); the
  // same bits for block(1); block(0) of the solution is then not maintained
  // (initialize_time_step overwrites it every step, problem.h:88-90)
  bool boundary_in_faces = true;
  // n_ranks > 1 with the exact SPIKE mass inverse: ONE exchange per RK stage.
  // The interface systems give each rank the neighbours' edge planes of k
  // (gdm_mass_solve_interface_ghosts), the stage updates run over the local
  // vectors, so y / acc / Y keep valid ghost planes and the stencil needs no
  // update_ghost_values (advection/stiffness.h:343); the solve's exchange is
  // the one left.  Ghost values then follow the neighbours' to the interface
  // truncation (<= 1e-15 relative per stage); ghost_resync_steps > 0
  // re-exchanges the solution's ghost planes every that many steps.  false:
  // the reference's two exchanges per stage.
  bool one_exchange_per_stage = true;
  unsigned int ghost_resync_steps = 0;
};

// A device buffer of doubles allocated through the engine (gdm_malloc).
class DeviceVector {
 public:
  DeviceVector() = default;
  DeviceVector(gdm_op *op, std::size_t n) { reinit(op, n); }
  DeviceVector(const DeviceVector &) = delete;
  DeviceVector &operator=(const DeviceVector &) = delete;
  DeviceVector(DeviceVector &&o) noexcept { swap(o); }
  DeviceVector &operator=(DeviceVector &&o) noexcept {
    swap(o);
    return *this;
  }
  ~DeviceVector() {
    if (ptr_) gdm_free(op_, ptr_);
  }
  void reinit(gdm_op *op, std::size_t n) {
    if (ptr_) gdm_free(op_, ptr_);
    op_ = op;
    n_ = n;
    void *p = nullptr;
    check(gdm_malloc(op_, sizeof(double) * std::max<std::size_t>(n, 1), &p), "gdm_malloc");
    ptr_ = static_cast<double *>(p);
    *this = 0.0;
  }
  DeviceVector &operator=(double s) {  // only 0 is meaningful, like deal.II
    if (n_) check(gdm_vec_axpby(op_, (int64_t)n_, 0.0, ptr_, 0.0, ptr_), "gdm_vec_axpby");
    (void)s;
    return *this;
  }
  void upload(const std::vector<double> &h) {
    if (h.size() != n_) throw Error("DeviceVector::upload: size mismatch");
    if (n_) check(gdm_memcpy_h2d(op_, ptr_, h.data(), sizeof(double) * n_), "gdm_memcpy_h2d");
  }
  std::vector<double> download() const {
    std::vector<double> h(n_);
    if (n_) check(gdm_memcpy_d2h(op_, h.data(), ptr_, sizeof(double) * n_), "gdm_memcpy_d2h");
    return h;
  }
  // this = a x + b this
  void sadd(double b, double a, const DeviceVector &x) {
    if (x.n_ != n_) throw Error("DeviceVector::sadd: size mismatch");
    if (n_) check(gdm_vec_axpby(op_, (int64_t)n_, a, x.ptr_, b, ptr_), "gdm_vec_axpby");
  }
  // this = acc_in + beta k and, when Y != nullptr, *Y = y + alpha k (one pass, gdm_vec_rk_update)
  void rk_update(double beta, const DeviceVector &k, const DeviceVector &acc_in, double alpha = 0.0,
                 const DeviceVector *y = nullptr, DeviceVector *Y = nullptr) {
    if (k.n_ != n_ || acc_in.n_ != n_ || (Y && (Y->n_ != n_ || !y || y->n_ != n_)))
      throw Error("DeviceVector::rk_update: size mismatch");
    if (n_)
      check(gdm_vec_rk_update(op_, (int64_t)n_, beta, k.ptr_, acc_in.ptr_, ptr_, alpha, Y ? y->ptr_ : nullptr,
                              Y ? Y->ptr_ : nullptr),
            "gdm_vec_rk_update");
  }
  double operator*(const DeviceVector &x) const {
    double r = 0.0;
    check(gdm_vec_dot(op_, (int64_t)n_, ptr_, x.ptr_, &r), "gdm_vec_dot");
    return r;
  }
  std::size_t size() const { return n_; }
  double *get_values() { return ptr_; }
  const double *get_values() const { return ptr_; }

 private:
  void swap(DeviceVector &o) noexcept {
    std::swap(op_, o.op_);
    std::swap(ptr_, o.ptr_);
    std::swap(n_, o.n_);
  }
  gdm_op *op_ = nullptr;
  double *ptr_ = nullptr;
  std::size_t n_ = 0;
};

// LinearAlgebra::distributed::BlockVector with the two blocks the advection
// operator uses: block(0) = stage boundary values, block(1) = DoF values in the
// local layout [ghost planes | owned planes | ghost planes].
struct BlockVector {
  DeviceVector b0, b1;
  DeviceVector &block(unsigned int i) { return i == 0 ? b0 : b1; }
  const DeviceVector &block(unsigned int i) const { return i == 0 ? b0 : b1; }
  void sadd(double b, double a, const BlockVector &x) {
    b0.sadd(b, a, x.b0);
    b1.sadd(b, a, x.b1);
  }
};

// What a multi-rank problem needs from its communicator (MPI_COMM_WORLD in
// the reference): the ghost-plane exchange of update_ghost_values
// (advection/stiffness.h:343) over the ranges of gdm_halo_plan, and
// Utilities::MPI::sum for the dots of the distributed CG.  An MPI rank
// implements it with MPI_Isend / MPI_Irecv (GPU-aware) or ncclSend / ncclRecv
// on those ranges; gdm/hip/thread_communicator.h runs ranks
// as threads of one process for the tests.
class Communicator {
 public:
  virtual ~Communicator() = default;
  // fill the ghost planes of `local` (engine-local layout of `op`) from the slab neighbours
  virtual void update_ghost_values(gdm_op *op, DeviceVector &local) = 0;
  // Split-phase form, for overlapping the exchange with work that reads no
  // ghost plane (the interior planes of the stencil, advection/stiffness.h:343
  // update_ghost_values before the cell loop): begin_ starts the exchange once
  // the owned planes queued on `op` are final; after end_ the ghost planes are
  // visible to everything queued on `op` later.  The default runs the whole
  // exchange in begin_.
  virtual void begin_update_ghost_values(gdm_op *op, DeviceVector &local) { update_ghost_values(op, local); }
  virtual void end_update_ghost_values(gdm_op *op, DeviceVector &local) {
    (void)op;
    (void)local;
  }
  virtual double sum(double local_value) = 0;
  // Utilities::MPI::max (the Linf reduction of the postprocess, problem.h:410-411)
  virtual double max(double local_value) = 0;
};

// RK_CLASSIC_FOURTH_ORDER (deal.II TimeStepping): c_i, a_{i,i-1}, b_i
struct ClassicRK4 {
  static constexpr double c[4] = {0.0, 0.5, 0.5, 1.0};
  static constexpr double a[4] = {0.0, 0.5, 0.5, 1.0};  // a[s] = a_{s,s-1}
  static constexpr double b[4] = {1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0};
};

// One RK stage update in low-storage form (the b-sum accumulated as the stages
// are produced, in the order of deal.II's final sadd loop): acc = (s == 0 ? y
// : acc) + h b_s k; Y = y + h a_{s+1} k; the last stage writes y itself.
inline void rk4_stage_update(int s, double h, const DeviceVector &k, DeviceVector &y, DeviceVector &acc,
                             DeviceVector &Y) {
  if (s == 3)
    y.rk_update(h * ClassicRK4::b[3], k, acc);
  else
    acc.rk_update(h * ClassicRK4::b[s], k, s == 0 ? y : acc, h * ClassicRK4::a[s + 1], &y, &Y);
}

// .../advection/discretization.h: the mesh, categories and partition (held by
// the engine) plus the quantities the problem driver reads.
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
  double get_dx() const { return (desc.hi[0] - desc.lo[0]) / desc.n_subdivisions[0]; }  // discretization.h:50
  const gdm_mesh_desc &get_mesh() const { return desc; }
  int get_device() const { return device; }

 private:
  gdm_mesh_desc desc{};
  int device = 0;
};

template <int dim>
class StiffnessMatrixOperator {
 public:
  explicit StiffnessMatrixOperator(const Discretization<dim> &discretization) : discretization(discretization) {}
  StiffnessMatrixOperator(const StiffnessMatrixOperator &) = delete;
  ~StiffnessMatrixOperator() { gdm_op_destroy(op); }

  void reinit(const Parameters<dim> &params) {
    gdm_op_destroy(op);
    op = nullptr;
    check(gdm_op_create(&discretization.get_mesh(), GDM_OP_ADVECTION, params.advection.data(), dim,
                        discretization.get_device(), &op),
          "gdm_op_create");
    check(gdm_op_layout(op, &layout), "gdm_op_layout");
    // every operator of a problem launches on the HIP null stream, so calls on
    // different operators stay ordered like the reference's serial calls
    check(gdm_op_set_stream(op, nullptr), "gdm_op_set_stream");
    exact_solution = params.exact_solution;
    exact_solution_der = params.exact_solution_der;
    bc_fn = params.boundary_function;
    bc_fn_params = params.boundary_function_params;
    // boundary points of the owned cells (device order), collect_boundary_points (:40-160)
    std::vector<double> xyz(3 * std::max<int64_t>(layout.n_bc_points, 1));
    check(gdm_bc_points(op, xyz.data()), "gdm_bc_points");
    all_points_0.resize(layout.n_bc_points);
    for (int64_t i = 0; i < layout.n_bc_points; ++i) all_points_0[i] = {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
  }

  // boundary_block = false: block(0) is left empty (size 0), for drivers that
  // let the engine compute the stage boundary values (boundary_in_faces)
  void initialize_dof_vector(BlockVector &vec, bool boundary_block = true) const {
    vec.b0.reinit(op, boundary_block ? layout.n_bc_points : 0);
    vec.b1.reinit(op, layout.n_local);
  }

  void initialize_time_step(BlockVector &stage_bc_and_solution, const double time) const {
    set_boundary(stage_bc_and_solution.block(0), time, 0);
  }

  // vec_rhs.block(1) (owned entries of its local layout) = K u + inflow
  // data; vec_rhs.block(0) = dg/dt at the boundary points.  The ghost planes of
  // src.block(1) must be current (update_ghost_values, stiffness.h:343).
  void compute_rhs(BlockVector &vec_rhs, const BlockVector &stage_bc_and_solution, const double time) const {
    set_boundary(vec_rhs.block(0), time, 1);
    check(gdm_apply(op, stage_bc_and_solution.block(1).get_values(), owned(vec_rhs.block(1)),
                    stage_bc_and_solution.block(0).get_values()),
          "gdm_apply");
  }

  // compute_rhs of one slab rank with the ghost exchange of `src`'s block(1)
  // overlapped (stiffness.h:343 + :345-605): the output planes whose 2p+1
  // input planes are all owned run while the exchange is in flight, the p
  // planes next to each slab edge after it, then the inflow boundary data.
  // Same additions in the same order as update_ghost_values + compute_rhs.
  // Plane ranges exist in 3D (gdm_apply_planes); other dims exchange first.
  void compute_rhs_overlapped(BlockVector &vec_rhs, BlockVector &src, const double time, Communicator &comm) const {
    if (dim != 3) {
      comm.update_ghost_values(op, src.block(1));
      compute_rhs(vec_rhs, src, time);
      return;
    }
    set_boundary(vec_rhs.block(0), time, 1);
    apply_planes_overlapped(vec_rhs.block(1), src.block(1), comm);
    if (layout.n_bc_points > 0)
      check(gdm_add_boundary_data(op, src.block(0).get_values(), owned(vec_rhs.block(1))), "gdm_add_boundary_data");
  }
  // the volume term of every owned plane, the planes that need no ghosts while
  // the exchange of u's ghost planes is in flight
  void apply_planes_overlapped(DeviceVector &rhs_block1, DeviceVector &u_vec, Communicator &comm) const {
    const int p = layout.halo_depth, pb = (int)layout.owned_plane_begin, pe = (int)layout.owned_plane_end;
    const int lo = pb + (layout.ghost_planes_below ? p : 0), hi = pe - (layout.ghost_planes_above ? p : 0);
    const double *u = u_vec.get_values();
    double *dst = owned(rhs_block1);
    comm.begin_update_ghost_values(op, u_vec);
    if (hi > lo) check(gdm_apply_planes(op, u, dst, lo, hi), "gdm_apply_planes");
    comm.end_update_ghost_values(op, u_vec);
    if (hi <= lo) {
      check(gdm_apply_planes(op, u, dst, pb, pe), "gdm_apply_planes");
    } else {
      // both edge ranges in one launch
      if (lo > pb || pe > hi) check(gdm_apply_planes2(op, u, dst, pb, lo, hi, pe), "gdm_apply_planes2");
    }
  }

  // block(0) from the built-in function, computed by the engine per stage
  bool boundary_in_faces() const { return bc_fn >= 0 && layout.n_bc_points > 0; }
  // compute_rhs's block(1) with the stage boundary values g(t_g) + alpha
  // dg/dt(t_k) computed by the engine per stage (gdm_apply_bc_fn)
  void compute_rhs_fn(DeviceVector &rhs_block1, const DeviceVector &u, double t_g, double alpha, double t_k) const {
    check(gdm_apply_bc_fn(op, u.get_values(), owned(rhs_block1), bc_fn, bc_fn_params.data(),
                          (int)bc_fn_params.size(), t_g, alpha, t_k),
          "gdm_apply_bc_fn");
  }
  // compute_rhs_overlapped with the boundary values of compute_rhs_fn
  void compute_rhs_fn_overlapped(DeviceVector &rhs_block1, DeviceVector &u, double t_g, double alpha, double t_k,
                                 Communicator &comm) const {
    if (dim != 3) {
      comm.update_ghost_values(op, u);
      compute_rhs_fn(rhs_block1, u, t_g, alpha, t_k);
      return;
    }
    apply_planes_overlapped(rhs_block1, u, comm);
    check(gdm_add_boundary_fn(op, owned(rhs_block1), bc_fn, bc_fn_params.data(), (int)bc_fn_params.size(), t_g,
                              alpha, t_k),
          "gdm_add_boundary_fn");
  }

  gdm_op *handle() const { return op; }
  const gdm_layout &get_layout() const { return layout; }
  double *owned(DeviceVector &v) const { return v.get_values() + layout.ghost_planes_below * layout.plane_size; }
  const double *owned(const DeviceVector &v) const {
    return v.get_values() + layout.ghost_planes_below * layout.plane_size;
  }

 private:
  std::vector<double> evaluate(const Function &f, double t) const {
    std::vector<double> v(all_points_0.size());
    for (std::size_t i = 0; i < v.size(); ++i) v[i] = f ? f(all_points_0[i], t) : 0.0;
    return v;
  }
  // block(0) <- g(t) (derivative 0) or dg/dt(t) (1): on the device for a
  // built-in function, else host callbacks + upload
  void set_boundary(DeviceVector &b0, double t, int derivative) const {
    if (layout.n_bc_points == 0) return;
    if (bc_fn >= 0)
      check(gdm_eval_boundary(op, bc_fn, bc_fn_params.data(), (int)bc_fn_params.size(), t, derivative,
                              b0.get_values()),
            "gdm_eval_boundary");
    else
      b0.upload(evaluate(derivative ? exact_solution_der : exact_solution, t));
  }
  int bc_fn = -1;
  std::vector<double> bc_fn_params;
  const Discretization<dim> &discretization;
  gdm_op *op = nullptr;
  gdm_layout layout{};
  Function exact_solution, exact_solution_der;
  std::vector<Point> all_points_0;
};

// .../advection/mass.h: the matrix-free mass operator models deal.II's
// MatrixType (vmult); solve() replaces the CG + ILU solve of problem.h:236-267
// by the exact Kronecker inverse.
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
    check(gdm_op_set_stream(op, nullptr), "gdm_op_set_stream");  // ordered with the stiffness operator
  }
  // dst (owned) = M src (local layout, ghosts current)
  void vmult(double *dst_owned, const double *src_local) const { check(gdm_mass_apply(op, src_local, dst_owned), "gdm_mass_apply"); }
  // x = M^-1 rhs (owned vectors)
  void solve(double *x_owned, const double *rhs_owned) const { check(gdm_mass_solve(op, rhs_owned, x_owned), "gdm_mass_solve"); }

  // MassMatrixOperator::get_sparse_matrix (advection/mass.h:30-36): an object
  // modelling deal.II's MatrixType -- vmult / Tvmult (M is symmetric) and
  // m() / n() -- over the matrix-free mass; SolverCG and the solve() call
  // sites take it where the reference takes the Trilinos matrix.
  class SparseMatrix {
   public:
    explicit SparseMatrix(const MassMatrixOperator &M) : M(M) {}
    // dst (owned entries) = M src (local layout, ghost planes current)
    void vmult(DeviceVector &dst, const DeviceVector &src) const {
      M.vmult(dst.get_values() + M.layout.ghost_planes_below * M.layout.plane_size, src.get_values());
    }
    void Tvmult(DeviceVector &dst, const DeviceVector &src) const { vmult(dst, src); }
    std::size_t m() const { return (std::size_t)M.layout.n_dofs_global; }
    std::size_t n() const { return (std::size_t)M.layout.n_dofs_global; }

   private:
    const MassMatrixOperator &M;
  };
  SparseMatrix get_sparse_matrix() const { return SparseMatrix(*this); }

  // Multi-rank solve(M, x, b) (problem.h:251-261): SolverCG with
  // ReductionControl(max_it, abs_tol, rel_tol) and the Jacobi preconditioner
  // on the matrix-free mass, ghost planes and dots through `comm`; x (owned)
  // starts from zero like the reference's fresh result vector.  Returns the
  // number of iterations (SolverControl::last_step).
  unsigned int solve_distributed(double *x_owned, const double *b_owned, Communicator &comm, double rel_tol = 1e-14,
                                 double abs_tol = 1e-20, unsigned int max_it = 1000) const {
    const int64_t n = layout.n_owned;
    if (cg_p.size() != (std::size_t)layout.n_local) {
      cg_p.reinit(op, layout.n_local);
      for (auto *v : {&cg_r, &cg_z, &cg_Ap, &cg_invdiag}) v->reinit(op, n);
      check(gdm_mass_diagonal(op, cg_invdiag.get_values()), "gdm_mass_diagonal");
      std::vector<double> d = cg_invdiag.download();
      for (double &v : d) v = 1.0 / v;
      cg_invdiag.upload(d);
    }
    const int64_t o = layout.ghost_planes_below * layout.plane_size;
    double *p_owned = cg_p.get_values() + o;
    auto dot = [&](const double *a, const double *b) {
      double r = 0.0;
      check(gdm_vec_dot(op, n, a, b, &r), "gdm_vec_dot");
      return comm.sum(r);
    };
    check(gdm_vec_axpby(op, n, 0.0, b_owned, 0.0, x_owned), "gdm_vec_axpby");            // x = 0
    check(gdm_vec_axpby(op, n, 1.0, b_owned, 0.0, cg_r.get_values()), "gdm_vec_axpby");  // r = b
    double res = std::sqrt(dot(cg_r.get_values(), cg_r.get_values()));
    const double tol = std::max(abs_tol, rel_tol * res);
    unsigned int it = 0;
    if (res <= tol) return 0;
    check(gdm_vec_pointwise_mult(op, n, cg_invdiag.get_values(), cg_r.get_values(), cg_z.get_values()), "jacobi");
    check(gdm_vec_axpby(op, n, 1.0, cg_z.get_values(), 0.0, p_owned), "gdm_vec_axpby");
    double rz = dot(cg_r.get_values(), cg_z.get_values());
    while (true) {
      if (it >= max_it) throw Error("MassMatrixOperator::solve_distributed: SolverControl::NoConvergence");
      ++it;
      comm.update_ghost_values(op, cg_p);
      check(gdm_mass_apply(op, cg_p.get_values(), cg_Ap.get_values()), "gdm_mass_apply");
      const double alpha = rz / dot(p_owned, cg_Ap.get_values());
      check(gdm_vec_axpby(op, n, alpha, p_owned, 1.0, x_owned), "gdm_vec_axpby");
      check(gdm_vec_axpby(op, n, -alpha, cg_Ap.get_values(), 1.0, cg_r.get_values()), "gdm_vec_axpby");
      res = std::sqrt(dot(cg_r.get_values(), cg_r.get_values()));
      if (res <= tol) break;
      check(gdm_vec_pointwise_mult(op, n, cg_invdiag.get_values(), cg_r.get_values(), cg_z.get_values()), "jacobi");
      const double rz_new = dot(cg_r.get_values(), cg_z.get_values());
      check(gdm_vec_axpby(op, n, 1.0, cg_z.get_values(), rz_new / rz, p_owned), "gdm_vec_axpby");
      rz = rz_new;
    }
    return it;
  }
  // Multi-rank exact solve (the SPIKE scheme of gdm_mass_solve_slab /
  // gdm_mass_solve_interface): slab-local solve, one ghost-plane exchange
  // through `comm`, spike_rounds() refinement rounds of one more exchange
  // each (slabs too thin for the truncated interface systems, e.g. C4 at 8
  // ranks), interface correction.  Usable when spike_available() (every slab
  // has >= 2p planes and the rounds reach 1e-15); x_owned may alias b_owned.
  int spike_rounds() const {
    int rounds = -1;
    return gdm_mass_spike_rounds(&discretization.get_mesh(), &rounds) == GDM_OK ? rounds : -1;
  }
  bool spike_available() const { return spike_rounds() >= 0; }
  void solve_spike(double *x_owned, const double *b_owned, Communicator &comm) const {
    if (sp_x.size() != (std::size_t)layout.n_local) sp_x.reinit(op, layout.n_local);
    if (sp_rounds < 0) sp_rounds = spike_rounds();
    double *own = sp_x.get_values() + layout.ghost_planes_below * layout.plane_size;
    check(gdm_mass_solve_slab(op, b_owned, own), "gdm_mass_solve_slab");
    comm.update_ghost_values(op, sp_x);
    for (int k = 0; k < sp_rounds; ++k) {
      check(gdm_mass_solve_interface_round(op, sp_x.get_values(), k), "gdm_mass_solve_interface_round");
      comm.update_ghost_values(op, sp_x);
    }
    check(gdm_mass_solve_interface(op, sp_x.get_values()), "gdm_mass_solve_interface");
    check(gdm_memcpy_d2d(op, x_owned, own, sizeof(double) * layout.n_owned), "gdm_memcpy_d2d");
  }
  // x_local (engine-local layout) = M^-1 of its owned part, in place, with
  // its ghost planes set to the neighbours' edge planes of the result from
  // the interface systems (gdm_mass_solve_interface_ghosts): one exchange
  // (+ the refinement rounds of thin slabs), no copy
  void solve_spike_local(DeviceVector &x_local, Communicator &comm) const {
    solve_spike_local_pending(x_local, comm);
    check(gdm_mass_solve_interface_ghosts(op, x_local.get_values()), "gdm_mass_solve_interface_ghosts");
  }
  // solve_spike_local up to (not including) the interface correction: the
  // slab solve, its exchange and the refinement rounds; finish with
  // spike_stage_update (the correction fused with the RK stage update)
  void solve_spike_local_pending(DeviceVector &x_local, Communicator &comm) const {
    if (x_local.size() != (std::size_t)layout.n_local) throw Error("solve_spike_local: x must be a local vector");
    if (sp_rounds < 0) sp_rounds = spike_rounds();
    double *own = x_local.get_values() + layout.ghost_planes_below * layout.plane_size;
    check(gdm_mass_solve_slab(op, own, own), "gdm_mass_solve_slab");
    comm.update_ghost_values(op, x_local);
    for (int k = 0; k < sp_rounds; ++k) {
      check(gdm_mass_solve_interface_round(op, x_local.get_values(), k), "gdm_mass_solve_interface_round");
      comm.update_ghost_values(op, x_local);
    }
  }
  // rk4_stage_update of local vectors with k = the interface-corrected solve
  // pending in x_local (gdm_mass_solve_interface_rk: one launch, k not stored;
  // the bits of solve_spike_local + rk4_stage_update)
  void spike_stage_update(int s, double h, const DeviceVector &x_local, DeviceVector &y, DeviceVector &acc,
                          DeviceVector &Y) const {
    if (s == 3)
      check(gdm_mass_solve_interface_rk(op, x_local.get_values(), h * ClassicRK4::b[3], acc.get_values(),
                                        y.get_values(), 0.0, nullptr, nullptr),
            "gdm_mass_solve_interface_rk");
    else
      check(gdm_mass_solve_interface_rk(op, x_local.get_values(), h * ClassicRK4::b[s],
                                        (s == 0 ? y : acc).get_values(), acc.get_values(), h * ClassicRK4::a[s + 1],
                                        y.get_values(), Y.get_values()),
            "gdm_mass_solve_interface_rk");
  }
  gdm_op *handle() const { return op; }

 private:
  const Discretization<dim> &discretization;
  gdm_op *op = nullptr;
  gdm_layout layout{};
  mutable DeviceVector cg_p, cg_r, cg_z, cg_Ap, cg_invdiag;  // solve_distributed work vectors
  mutable DeviceVector sp_x;                                  // solve_spike local vector
  mutable int sp_rounds = -1;                                 // solve_spike refinement rounds (cached)
};

// deal.II DiscreteTime (base/discrete_time.cc): the next time is the current
// one plus the last step, the step itself recomputed as the difference of the
// two times (so round-off accumulates exactly as in the reference), snapped to
// the end time when within 5 % of a step of it.
class DiscreteTime {
 public:
  DiscreteTime(double start, double end, double dt) : t(start), end(end), next(next_time(start, dt, end)) {}
  bool is_at_end() const { return t == end; }
  double get_current_time() const { return t; }
  double get_next_step_size() const { return next - t; }
  void advance_time() {
    const double step = next - t;
    t = next;
    next = next_time(t, step, end);
    ++steps;
  }
  unsigned int get_step_number() const { return steps; }

 private:
  static double next_time(double current, double step, double end) {
    double n = current + step;
    if (step > 0.0 && n > end - 0.05 * step) n = end;
    return n;
  }
  double t, end, next;
  unsigned int steps = 0;
};

// .../advection/problem.h:31-102 (non-composite branch): explicit RK4
// (RK_CLASSIC_FOURTH_ORDER) on (block(0), block(1)) with
// f(t, y) = (dg/dt, M^-1 (K u + inflow data)).
template <int dim>
class AdvectionProblem {
 public:
  // comm: required for n_ranks > 1 (MPI_COMM_WORLD of the reference)
  explicit AdvectionProblem(const Parameters<dim> &params, Communicator *comm = nullptr)
      : params(params), comm(comm), mass_matrix_operator(discretization), stiffness_matrix_operator(discretization) {}

  // Runs to end_t (or max_steps); returns the number of steps.  The solution
  // is available through get_solution() (owned DoFs, reference global order).
  unsigned int run(unsigned int max_steps = ~0u) {
    if (params.n_ranks != 1 && !comm) throw Error("AdvectionProblem: n_ranks > 1 needs a Communicator");
    discretization.reinit(params);
    mass_matrix_operator.reinit(params);
    stiffness_matrix_operator.reinit(params);
    const double delta_t = discretization.get_dx() * params.cfl / params.max_val;  // problem.h:45
    // in_faces: the engine computes the stage boundary values itself, block(0)
    // is never read or updated and stays empty (28 M points at C3)
    const bool in_faces = params.boundary_in_faces && stiffness_matrix_operator.boundary_in_faces();
    stiffness_matrix_operator.initialize_dof_vector(solution, !in_faces);
    set_initial_condition(solution.block(1));
    // device-resident low-storage RK4: k (stage derivative), acc (b-sum), Y
    // (next stage) -- no per-stage allocation (problem.h:64-65) and, with a
    // device boundary function, no host evaluation or upload in the loop
    BlockVector k, acc, stage;
    stiffness_matrix_operator.initialize_dof_vector(k, !in_faces);
    stiffness_matrix_operator.initialize_dof_vector(acc, !in_faces);
    stiffness_matrix_operator.initialize_dof_vector(stage, !in_faces);
    if (params.n_ranks != 1) rhs_tmp.reinit(stiffness_matrix_operator.handle(), stiffness_matrix_operator.get_layout().n_owned);
    use_spike = params.n_ranks != 1 && mass_matrix_operator.spike_available();
    one_exchange = use_spike && params.one_exchange_per_stage;
    // the ghost planes of the solution once at the start (set_initial_condition
    // interpolates them too); with one_exchange they are kept current by the
    // local-vector updates from then on
    if (one_exchange) comm->update_ghost_values(stiffness_matrix_operator.handle(), solution.block(1));
    // stage boundary values computed by the engine: g(t0) + alpha dg/dt(t_k)
    double t0 = 0.0, bc_alpha = 0.0, bc_tk = 0.0;
    const auto fu_rhs = [&](double time, BlockVector &y, BlockVector &result) {
      if (one_exchange) {
        // the stage vector's ghost planes are current: no update_ghost_values
        if (in_faces)
          stiffness_matrix_operator.compute_rhs_fn(result.block(1), y.block(1), t0, bc_alpha, bc_tk);
        else
          stiffness_matrix_operator.compute_rhs(result, y, time);
        // the interface correction runs fused with the stage update below
        mass_matrix_operator.solve_spike_local_pending(result.block(1), *comm);
        return;
      }
      if (in_faces) {
        if (params.n_ranks != 1 && params.overlap_exchange) {
          stiffness_matrix_operator.compute_rhs_fn_overlapped(result.block(1), y.block(1), t0, bc_alpha, bc_tk,
                                                              *comm);
        } else {
          if (params.n_ranks != 1) comm->update_ghost_values(stiffness_matrix_operator.handle(), y.block(1));
          stiffness_matrix_operator.compute_rhs_fn(result.block(1), y.block(1), t0, bc_alpha, bc_tk);
        }
      } else if (params.n_ranks != 1 && params.overlap_exchange) {
        stiffness_matrix_operator.compute_rhs_overlapped(result, y, time, *comm);
      } else {
        if (params.n_ranks != 1) comm->update_ghost_values(stiffness_matrix_operator.handle(), y.block(1));
        stiffness_matrix_operator.compute_rhs(result, y, time);
      }
      double *r = stiffness_matrix_operator.owned(result.block(1));
      if (params.n_ranks == 1) {
        mass_matrix_operator.solve(r, r);
      } else if (use_spike) {
        mass_matrix_operator.solve_spike(r, r, *comm);
      } else {
        check(gdm_memcpy_d2d(stiffness_matrix_operator.handle(), rhs_tmp.get_values(), r,
                             sizeof(double) * rhs_tmp.size()),
              "gdm_memcpy_d2d");
        mass_matrix_operator.solve_distributed(r, rhs_tmp.get_values(), *comm);
      }
    };
    DiscreteTime time(params.start_t, params.end_t, delta_t);
    unsigned int n = 0;
    while (!time.is_at_end() && n < max_steps) {
      t0 = time.get_current_time();
      const double h = time.get_next_step_size();
      if (!in_faces) stiffness_matrix_operator.initialize_time_step(solution, t0);  // evaluate bc
      for (int s = 0; s < 4; ++s) {
        // stage s reads block(0) = g(t0) + h a_{s,s-1} dg/dt(t0 + c_{s-1} h)
        bc_alpha = s == 0 ? 0.0 : h * ClassicRK4::a[s];
        bc_tk = s == 0 ? t0 : t0 + ClassicRK4::c[s - 1] * h;
        fu_rhs(t0 + ClassicRK4::c[s] * h, s == 0 ? solution : stage, k);  // ghosts of the stage exchanged
        for (unsigned int bl = in_faces ? 1 : 0; bl < 2; ++bl)
          if (one_exchange && bl == 1)
            mass_matrix_operator.spike_stage_update(s, h, k.block(1), solution.block(1), acc.block(1),
                                                    stage.block(1));
          else
            rk4_stage_update(s, h, k.block(bl), solution.block(bl), acc.block(bl), stage.block(bl));
      }
      time.advance_time();
      ++n;
      if (one_exchange && params.ghost_resync_steps > 0 && n % params.ghost_resync_steps == 0)
        comm->update_ghost_values(stiffness_matrix_operator.handle(), solution.block(1));
    }
    return n;
  }

  // owned DoF values (reference global order of the owned planes)
  std::vector<double> get_solution() const {
    const gdm_layout &L = stiffness_matrix_operator.get_layout();
    std::vector<double> v = solution.block(1).download();
    const int64_t o = L.ghost_planes_below * L.plane_size;
    return std::vector<double>(v.begin() + o, v.begin() + o + L.n_owned);
  }
  const BlockVector &get_solution_vector() const { return solution; }
  // which multi-rank mass solve run() used: exact SPIKE or the Jacobi CG
  bool used_spike_solve() const { return use_spike; }
  // whether run() did one exchange per stage (Parameters::one_exchange_per_stage)
  bool used_one_exchange() const { return one_exchange; }

  // postprocess(time, solution) (problem.h:269-485), error part on the device:
  // {Linf, L1, L2, Linf_face, L1_face, L2_face} of u - exact_solution(time)
  // over QGauss(p+1) on the owned cells, reduced over the ranks like the
  // reference (max, sum, sqrt of the summed squares).  The uncut box has no
  // immersed surface, so the face norms are 0.  The exact solution must be a
  // built-in device function (Parameters::boundary_function).
  std::array<double, 6> postprocess(const double time) {
    if (params.boundary_function < 0)
      throw Error("AdvectionProblem::postprocess: needs a built-in exact solution (boundary_function)");
    if (params.n_ranks != 1) comm->update_ghost_values(stiffness_matrix_operator.handle(), solution.block(1));
    double e[3];
    check(gdm_error_norms(stiffness_matrix_operator.handle(), solution.block(1).get_values(), params.boundary_function,
                          params.boundary_function_params.data(), (int)params.boundary_function_params.size(), time,
                          nullptr, e),
          "gdm_error_norms");
    if (params.n_ranks != 1) {
      e[0] = comm->max(e[0]);
      e[1] = comm->sum(e[1]);
      e[2] = std::sqrt(comm->sum(e[2] * e[2]));
    }
    return {{e[0], e[1], e[2], 0.0, 0.0, 0.0}};
  }

 private:
  // VectorTools::interpolate of the GDM vertex basis = vertex values (vector_tools.h:11-23)
  void set_initial_condition(DeviceVector &u) const {
    const gdm_mesh_desc &m = discretization.get_mesh();
    const gdm_layout &L = stiffness_matrix_operator.get_layout();
    std::vector<double> h(L.n_local);
    const int N0 = m.n_subdivisions[0] + 1, N1 = dim > 1 ? m.n_subdivisions[1] + 1 : 1;
    const int64_t first_plane = L.owned_plane_begin - L.ghost_planes_below;
    for (int64_t i = 0; i < L.n_local; ++i) {
      const int64_t g = first_plane * L.plane_size + i;  // global lexicographic index
      Point x{0.0, 0.0, 0.0};
      int64_t r = g;
      const int64_t n[3] = {N0, N1, 0};
      for (int d = 0; d < dim; ++d) {
        const int64_t id = d + 1 < dim ? r % n[d] : r;
        if (d + 1 < dim) r /= n[d];
        x[d] = m.lo[d] + id * (m.hi[d] - m.lo[d]) / m.n_subdivisions[d];
      }
      h[i] = params.exact_solution(x, params.start_t);
    }
    u.upload(h);
  }

  Parameters<dim> params;
  Communicator *comm = nullptr;
  Discretization<dim> discretization;
  MassMatrixOperator<dim> mass_matrix_operator;
  StiffnessMatrixOperator<dim> stiffness_matrix_operator;
  BlockVector solution;
  DeviceVector rhs_tmp;
  bool use_spike = false, one_exchange = false;
};

}  // namespace HIP
}  // namespace GDM
