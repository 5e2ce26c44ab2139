/*
 * gdm_hip.h -- C ABI of libgdm_hip.so, the MI355X (gfx950) operator engine for
 * the Galerkin-difference-method (GDM) hot path of
 * peterrum/dealii-galerkin-difference-methods.
 *
 * The reference has no formal FFI: its drop-in surface is the operator classes
 * the RK drivers call plus deal.II's MatrixType concept (vmult).  Each entry
 * point below replaces one of those reference interfaces (paths relative to
 * the reference root):
 *
 *   gdm_op_create        GDM::System<dim>(comm, p, n_comp, ghost) +
 *                        subdivided_hyper_cube + categorize
 *                        (include/gdm/system.h:355-424) and
 *                        Discretization::reinit
 *                        (applications/advection/include/gdm/advection/
 *                        discretization.h:27-89) and
 *                        StiffnessMatrixOperator::reinit (advection/stiffness.h:23-38,
 *                        wave/stiffness.h:23-31) / MassMatrixOperator::reinit
 *                        (advection/mass.h:25-28)
 *   gdm_op_layout        System::locally_owned_dofs / locally_active_dofs and the
 *                        Partitioner (system.h:634-688, 720-757;
 *                        advection/discretization.h:85-88), plus
 *                        StiffnessMatrixOperator::initialize_dof_vector's block(0)
 *                        size (advection/stiffness.h:162-179)
 *   gdm_apply            StiffnessMatrixOperator::compute_rhs (advection:
 *                        advection/stiffness.h:196-606; wave:
 *                        wave/stiffness.h:409-420 -> :42-407), volume + box-face
 *                        terms of the uncut path
 *   gdm_mass_apply       TrilinosWrappers::SparseMatrix::vmult on the matrix of
 *                        MassMatrixOperator::get_sparse_matrix (advection/mass.h:30-36)
 *   gdm_mass_solve       *Problem::solve(mass_matrix, result, rhs)
 *                        (advection/problem.h:236-267, wave/problem.h:471-502):
 *                        the CG + ILU/AMG solve is replaced by the exact
 *                        Kronecker inverse of the uncut mass matrix
 *   gdm_vec_axpby/dot    the vector updates of TimeStepping::ExplicitRungeKutta
 *                        (advection/problem.h:91-94) / SolverCG inner products
 *   gdm_bc_points        StiffnessMatrixOperator::collect_boundary_points
 *                        (advection/stiffness.h:40-160): coordinates of the
 *                        boundary quadrature points (device order)
 *   gdm_bc_reference_order  permutation between the reference's block(0)
 *                        order (cell, face, q) and the device order
 *
 * Conventions: plain pointers and sizes only; every function returns GDM_OK (0)
 * or a negative error code, never throws across the ABI; the message of the
 * last error on the calling thread is available from gdm_last_error.  Vector
 * arguments are DEVICE pointers (hipMalloc'ed or torch CUDA tensors) unless
 * the name says _host.  Calls are ordered on the operator's stream; results
 * that reach host memory are synchronous on return.
 */
#ifndef GDM_HIP_H
#define GDM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GDM_HIP_ABI_VERSION 15

enum gdm_status {
  GDM_OK = 0,
  GDM_ERR_ARG = -1,         /* invalid argument (AssertThrow in the reference) */
  GDM_ERR_HIP = -2,         /* HIP runtime error */
  GDM_ERR_UNSUPPORTED = -3, /* ExcNotImplemented in the reference */
  GDM_ERR_NOMEM = -4,
  GDM_ERR_STATE = -5
};

/* operator kinds */
enum gdm_op_kind {
  GDM_OP_MASS = 0,       /* (v, u)                                  mass.h:144-156   */
  GDM_OP_ADVECTION = 1,  /* (a u, grad v) - <(a.n) u_up, v>_box     stiffness.h:345-532 */
  GDM_OP_WAVE = 2,       /* -(grad v, grad u) [+ Nitsche on the box] wave/stiffness.h:151-330 */
  GDM_OP_CONVECTIVE = 3  /* -(a . grad u, v)  prototypes/advection_01_gdm.cc:164-206 */
};

typedef struct gdm_op gdm_op;

typedef struct {
  int32_t dim;               /* 1, 2 or 3                                   */
  int32_t fe_degree;         /* odd, 1..9 (fe.h:321-323)                     */
  int32_t n_subdivisions[3]; /* cells per direction                          */
  double lo[3], hi[3];       /* box (subdivided_hyper_cube/_rectangle)       */
  int32_t n_ranks, rank;     /* slab partition along the last coordinate     */
  int32_t periodic;          /* bit d: periodic constraints in direction d
                                (System::make_periodicity_constraints, system.h:427-463:
                                vertex N_d - 1 := vertex 0; gdm_apply / gdm_mass_apply
                                distribute the input and condense the result, the
                                constrained rows are zero; single rank; not with the
                                advection face terms or box Nitsche) */
} gdm_mesh_desc;

/* Local vector layout of one rank.  Device vectors are stored
 * [ghost planes below | owned planes | ghost planes above], each plane
 * lexicographic (x fastest), i.e. the reference's global DoF order
 * (system.h:238-244) restricted to a plane range. */
typedef struct {
  int64_t n_dofs_global;
  int64_t plane_size;             /* DoFs per vertex plane of the last coordinate */
  int32_t n_planes_global;
  int32_t owned_plane_begin;      /* global vertex planes [begin, end) owned   */
  int32_t owned_plane_end;
  int32_t ghost_planes_below;     /* halo depth actually present (<= p)         */
  int32_t ghost_planes_above;
  int32_t cell_plane_begin;       /* owned cell planes (system.h:747-757)       */
  int32_t cell_plane_end;
  int32_t halo_depth;             /* = fe_degree                                */
  int64_t n_owned;                /* owned DoFs                                 */
  int64_t n_local;                /* owned + ghost DoFs                         */
  int64_t n_bc_points;            /* device block(0) size: boundary points of the owned
                                     cells plus, on a multi-rank mesh, those of the
                                     neighbour cells whose DoF boxes reach owned DoFs
                                     (owner-computes replaces compress(add)) */
  int64_t n_bc_points_ref;        /* the reference's block(0) size: points of the owned
                                     cells only (stiffness.h:40-160)                  */
} gdm_layout;

/* Ghost-plane exchange of one rank: owner-computes needs the
 * p vertex planes next to the slab from each z-neighbour (the reference's
 * update_ghost_values + compress(add), advection/stiffness.h:343, 605).  All
 * ranges are in elements of the rank's engine-local vector (gdm_layout);
 * every range is contiguous.  The caller moves them with its own
 * communicator (MPI_Isend/Irecv on device pointers with a GPU-aware MPI,
 * ncclSend/ncclRecv, or torch.distributed, gdm_amd/distributed.py):
 *   send [send_below_offset, + send_below_count) to rank_below, which
 *   receives it into its [recv_above_offset, + recv_above_count), and the
 *   mirror image towards rank_above.
 * deal.II's LinearAlgebra::distributed::Vector stores [owned | ghosts sorted]
 * with the reference's ghost layer (one ghost cell layer: dealii_ghost_planes_
 * below / _above planes, system.h:657-688, 767-771) -- fewer than the p planes
 * owner-computes reads -- so the engine vector is a separate buffer: its owned
 * block starts at owned_offset and equals deal.II's owned block element for
 * element (the reference's global lexicographic order). */
typedef struct {
  int32_t rank_below, rank_above; /* -1: none */
  int64_t owned_offset;           /* = ghost_planes_below * plane_size */
  int64_t send_below_offset, send_below_count;
  int64_t recv_below_offset, recv_below_count;
  int64_t send_above_offset, send_above_count;
  int64_t recv_above_offset, recv_above_count;
  int32_t dealii_ghost_planes_below, dealii_ghost_planes_above;
} gdm_halo;

/* params (n_params):
 *   GDM_OP_MASS        : none
 *   GDM_OP_ADVECTION   : a_x, a_y, a_z               (constant field, see below)
 *   GDM_OP_CONVECTIVE  : a_x, a_y, a_z
 *   The reference evaluates advection->value(x_q, d) at every quadrature point
 *   (advection/stiffness.h:395-406, 443, 510); the engine's Kronecker form
 *   holds for a CONSTANT field only, which is what every reference preset uses
 *   (ConstantFunction, advection-app.cc:131-139).  A spatially varying field
 *   cannot be expressed through these params: a caller with one must keep the
 *   reference's cell loop (the engine cannot detect it, it only sees a[]).
 *   GDM_OP_WAVE        : [nitsche_parameter]         (> 0 enables box Nitsche,
 *                        function_domain_dbc; absent / <= 0 = natural BC) */
int gdm_last_error(char *buf, size_t len);
int gdm_abi_version(void);
int gdm_get_device_count(int *n);

int gdm_op_create(const gdm_mesh_desc *mesh, int kind, const double *params, int n_params, int device,
                  gdm_op **out);
int gdm_op_destroy(gdm_op *op);
/* the exchange plan of mesh->rank (pure host function: no device, no op) */
int gdm_halo_plan(const gdm_mesh_desc *mesh, gdm_halo *out);
int gdm_op_layout(const gdm_op *op, gdm_layout *out);
/* launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream;
 * NULL is the HIP null stream); gdm_op_use_own_stream restores the operator's
 * private non-blocking stream.  An operator's calls must stay ordered (one
 * stream at a time, or the caller orders the streams): they share the
 * operator's face scratch and the stencil's tail-work counter.  Each call is
 * self-contained otherwise, so it may be captured in a hipGraph and replayed. */
int gdm_op_set_stream(gdm_op *op, void *hip_stream);
int gdm_op_use_own_stream(gdm_op *op);
/* the hipStream_t the operator launches on now (set or own): a communicator
 * orders a device-side ghost exchange after the operator's work on it and
 * makes later work wait for the exchange (RcclRank's split-phase
 * update_ghost_values, advection/stiffness.h:343) -- ABI v10 */
int gdm_op_get_stream(const gdm_op *op, void **hip_stream);

/* dst_owned = K src_local (+ inflow boundary-data term when bc_values != NULL,
 * advection only: bc_values are the stage boundary values, device order, size
 * n_bc_points).  src_local has the full local layout (ghost planes filled). */
int gdm_apply(gdm_op *op, const double *src_local, double *dst_owned, const double *bc_values);
/* The volume part of gdm_apply for the owned output planes [plane_begin,
 * plane_end) of the last coordinate only (global plane indices; 3D).  Lets a
 * multi-rank caller compute the planes that need no ghost data while the
 * ghost-plane exchange is in flight, then the p planes next to each slab edge
 * (the overlap of update_ghost_values, advection/stiffness.h:343, with the cell
 * loop).  Boundary data: gdm_add_boundary_data afterwards. */
int gdm_apply_planes(gdm_op *op, const double *src_local, double *dst_owned, int plane_begin, int plane_end);
/* gdm_apply_planes of two plane ranges [b0, e0) and [b1, e1) in ONE launch
 * (ABI 13): the p planes next to both slab edges after the exchange, so the
 * thin edge ranges share the GPU instead of running one after the other.  The
 * same bits as two gdm_apply_planes calls.  Both ranges are clipped to the
 * owned planes first; an empty (or wholly unowned) range is allowed. */
int gdm_apply_planes2(gdm_op *op, const double *src_local, double *dst_owned, int b0, int e0, int b1, int e1);
/* dst_owned += inflow boundary-data term only (the bc part of gdm_apply,
 * advection/stiffness.h:520-529 with a.n < 0); no-op for other kinds */
int gdm_add_boundary_data(gdm_op *op, const double *bc_values, double *dst_owned);
/* dst_owned = M src_local */
int gdm_mass_apply(gdm_op *op, const double *src_local, double *dst_owned);
/* x_owned = M^-1 rhs_owned (exact Kronecker inverse; single rank; not with
 * periodic constraints: gdm_mass_solve_cg) */
int gdm_mass_solve(gdm_op *op, const double *rhs_owned, double *x_owned);
/* gdm_mass_solve_rk: k = M^-1 rhs, then gdm_vec_rk_update's acc_out = acc_in +
 * beta k and, when Y != NULL, Y = y + alpha k -- one RK stage's solve and
 * update (advection/problem.h:62-94 + the solve of :236-267) with the update
 * fused into the last line-solve pass, so k never reaches HBM.  rhs_owned is
 * overwritten (scratch).  Aliasing (GDM_ERR_ARG otherwise): rhs_owned overlaps
 * none of acc_in / acc_out / y / Y; acc_out and Y are distinct; a written
 * vector (acc_out, Y) may equal a read one (acc_in, y) but not partially
 * overlap it.  Same bits as gdm_mass_solve(rhs, rhs) + gdm_vec_rk_update.
 * Single rank, non-periodic. */
int gdm_mass_solve_rk(gdm_op *op, double *rhs_owned, double beta, const double *acc_in, double *acc_out,
                      double alpha, const double *y, double *Y);

/* Distributed exact mass inverse (n_ranks > 1; replaces the CG + ILU/AMG
 * solve of advection/problem.h:236-267 / wave/problem.h:457-502 across MPI
 * ranks).  M^-1 = M_q^-1 (x) ... (x) M_0^-1; the in-slab directions are
 * solved locally; the partitioned direction q = dim - 1 by a truncated SPIKE
 * scheme: each slab solves with its own diagonal block A_r of M_q, the ranks
 * exchange p planes with each slab neighbour (exactly the ghost planes of the
 * stencil's update_ghost_values), and a 2p x 2p interface system per slab
 * boundary (the same for every line) corrects the slab:
 *   gdm_mass_solve_slab(op, rhs_owned, x_owned)   x = (A_r^-1 (x) M_y^-1 (x) M_x^-1) rhs
 *   <copy x_owned into the owned part of a local vector; ghost exchange>
 *   for round in [0, rounds):                        (thin slabs only)
 *     gdm_mass_solve_interface_round(op, x_local, round); <ghost exchange>
 *   gdm_mass_solve_interface(op, x_local)          owned part of x_local = M^-1 rhs
 * The truncated interface systems drop the far-spike couplings (entries
 * <= gdm_mass_spike_eps, pure host; decays geometrically with the slab
 * thickness).  When that exceeds 1e-15 (slabs thinner than ~48 planes at p = 5,
 * e.g. C4 at 8 ranks: 32 planes, p = 7, eps 2e-8) gdm_mass_spike_rounds
 * (pure host) returns the number m of refinement rounds: each evaluates the
 * dropped couplings at the current interface values, moves them into the
 * slab's edge planes (the right-hand sides of the next interface systems) and
 * needs one more ghost exchange of the same p planes; the error after m rounds
 * is ~eps^(m+1).  rounds = -1: refused (GDM_ERR_UNSUPPORTED from the slab
 * solve; a slab with fewer than 2p planes or eps too large).  n_ranks == 1:
 * the slab solve is gdm_mass_solve and the interface call a no-op. */
int gdm_mass_spike_eps(const gdm_mesh_desc *mesh, double *eps_host);
int gdm_mass_spike_rounds(const gdm_mesh_desc *mesh, int *rounds);
int gdm_mass_solve_slab(gdm_op *op, const double *rhs_owned, double *x_owned);
int gdm_mass_solve_interface_round(gdm_op *op, double *x_local, int round);
int gdm_mass_solve_interface(gdm_op *op, double *x_local);
/* gdm_mass_solve_interface, and the ghost planes of x_local are overwritten
 * with the interface solution -- the lower neighbour's last p planes and the
 * upper neighbour's first p planes of M^-1 rhs, which each interface system
 * yields on both ranks of the pair (ABI 14).  x_local is then a valid local
 * vector of M^-1 rhs (ghosts equal to the neighbours' owned values to the
 * truncation tolerance, <= 1e-15 relative): an RK stage that updates its
 * local vectors over the ghost planes too (k, acc, y, Y in local layout)
 * needs no update_ghost_values before the next stage's stencil
 * (advection/stiffness.h:343) -- one exchange per stage, the SPIKE one. */
int gdm_mass_solve_interface_ghosts(gdm_op *op, double *x_local);
/* The interface step of the one-exchange stage fused with its RK update
 * (ABI 15): k = M^-1 rhs on every plane of the local layout (the owned planes
 * corrected as gdm_mass_solve_interface does, the ghost planes the interface
 * solution as gdm_mass_solve_interface_ghosts writes them) goes straight into
 * acc_out = acc_in + beta k and, when Y != NULL, Y = y + alpha k -- local
 * vectors (n_local entries), the arithmetic and the bits of
 * gdm_mass_solve_interface_ghosts + gdm_vec_rk_update over n_local; k is not
 * stored (x_local, holding the slab solve and the exchanged planes, is only
 * read).  acc_out may equal acc_in (not partially overlap it), y may equal
 * acc_in; x_local must not overlap an output.  Multi-rank only. */
int gdm_mass_solve_interface_rk(gdm_op *op, const double *x_local, double beta, const double *acc_in, double *acc_out,
                                double alpha, const double *y, double *Y);

/* x_owned = M^-1 rhs_owned by SolverCG on the matrix-free mass operator with
 * ReductionControl(max_it, abs_tol, rel_tol) semantics, the solve of
 * prototypes/advection_01_gdm.cc:208-217 (PreconditionJacobi, rel 1e-8) and of
 * *Problem::solve (advection/problem.h:251-261); precond 0 = identity,
 * 1 = Jacobi (diagonal of the condensed mass).  x_owned is the initial guess
 * (the reference starts from zero); *its_host = SolverControl::last_step();
 * GDM_ERR_STATE when max_it is reached.  Works with periodic constraints (the
 * condensed operator: constrained rows zero).  Single rank. */
int gdm_mass_solve_cg(gdm_op *op, const double *rhs_owned, double *x_owned, double rel_tol, double abs_tol,
                      int max_it, int precond, int *its_host, double *res_host);

/* diag_owned (device) = the diagonal of the (condensed) mass matrix on the
 * owned DoFs: the PreconditionJacobi of prototypes/advection_01_gdm.cc:211
 * and the diagonal a distributed CG preconditions with (constrained rows 1). */
int gdm_mass_diagonal(gdm_op *op, double *diag_owned);
/* y = w .* x elementwise (a diagonal preconditioner application) */
int gdm_vec_pointwise_mult(gdm_op *op, int64_t n, const double *w, const double *x, double *y);
/* device-to-device copy on the operator's stream */
int gdm_memcpy_d2d(gdm_op *op, void *dst, const void *src, size_t bytes);

/* AffineConstraints::distribute of the periodicity constraints
 * (advection_01_gdm.cc:158, 268): v[last vertex of d] = v[first] for every
 * periodic direction d; no-op without periodic constraints. */
int gdm_constraints_distribute(gdm_op *op, double *v_owned);

/* In-place banded-Cholesky solve with the 1D mass matrix of reference
 * direction `axis` (0 = x, 1 = y, 2 = z) along n_lines lines of full length
 * N[axis]: line l starts at v + (l / A) * B + (l % A) * C and its entries are
 * `stride` apart.  The building block of the distributed mass inverse (the
 * slab-local directions are solved in place, the partitioned one after a
 * transpose; gdm_amd/distributed.py), replacing the CG of
 * advection/problem.h:236-267 on a multi-rank mesh. */
int gdm_mass_solve_lines(gdm_op *op, int axis, double *v, int64_t n_lines, int64_t stride, int64_t A, int64_t B,
                         int64_t C);

/* y = a x + b y ; *result_host = x . y */
int gdm_vec_axpby(gdm_op *op, int64_t n, double a, const double *x, double b, double *y);
int gdm_vec_dot(gdm_op *op, int64_t n, const double *x, const double *y, double *result_host);
int gdm_synchronize(gdm_op *op);

/* ------------------------------------------------------------------------
 * Device-resident explicit Runge-Kutta: replaces the per-stage
 * BlockVector allocation and vector updates of TimeStepping::
 * ExplicitRungeKutta (advection/problem.h:62-94, wave/problem.h:296-338) and
 * the host evaluation of block(0) in initialize_time_step / compute_rhs
 * (advection/stiffness.h:181-194, 286-289).
 *
 *   gdm_vec_rk_update   acc_out = acc_in + beta k and, when Y != NULL,
 *                       Y = y + alpha k, in one pass (low-storage form of a
 *                       Butcher table with one nonzero a_ij per stage, e.g.
 *                       RK_CLASSIC_FOURTH_ORDER; acc_in may equal acc_out)
 *   gdm_eval_boundary   bc_values (device order, n_bc_points) = g(t)
 *                       (derivative 0) or dg/dt(t) (derivative 1) at the
 *                       boundary points for a built-in function:
 *     GDM_FN_CONSTANT      params: c
 *     GDM_FN_CONE          params: r0, center[dim] -- max(0, r0 - |x - c|)
 *                          (the advection app's ExactSolution,
 *                          applications/advection/advection-app.cc:51-79;
 *                          dg/dt = 0, its ExactSolutionDerivative)
 *     GDM_FN_SINE_PRODUCT  params: a[3], k[3], phi[3] --
 *                          prod_d sin(2 pi k_d (x_d - a_d t) + phi_d)
 *                          (a solution transported with velocity a)
 * ---------------------------------------------------------------------- */
enum gdm_fn_kind { GDM_FN_CONSTANT = 0, GDM_FN_CONE = 1, GDM_FN_SINE_PRODUCT = 2 };
int gdm_vec_rk_update(gdm_op *op, int64_t n, double beta, const double *k, const double *acc_in, double *acc_out,
                      double alpha, const double *y, double *Y);
int gdm_eval_boundary(gdm_op *op, int fn_kind, const double *params, int n_params, double t, int derivative,
                      double *bc_values);
/* gdm_apply_bc_fn: gdm_apply (stencil + inflow boundary term) with the stage
 * boundary values computed by the engine (into its own scratch, inflow faces
 * only, one launch before the stencil) instead of read from a caller's
 * bc_values vector: BC = g(t_g) + alpha dg/dt(t_k) (alpha = 0: g(t_g)), the
 * same bits as gdm_eval_boundary(g, t_g) / (dg/dt, t_k) followed by
 * gdm_vec_rk_update's Y = y + alpha k.  This is block(0) of the reference's
 * RK stages (advection/problem.h:62-94 with initialize_time_step,
 * stiffness.h:181-194, and the dg/dt stage block, stiffness.h:286-289) for
 * the classic RK4 tableau, where stage s >= 1 reads y0 + h a_{s,s-1} k_{s-1}:
 * the block(0) vectors and their stage updates disappear (block(0) after a
 * step is never read: initialize_time_step overwrites it, problem.h:88-90).
 * Advection operators; fn_kind / params as gdm_eval_boundary. */
int gdm_apply_bc_fn(gdm_op *op, const double *src_local, double *dst_owned, int fn_kind, const double *params,
                    int n_params, double t_g, double alpha, double t_k);
/* gdm_add_boundary_fn: gdm_add_boundary_data with the stage boundary values
 * of gdm_apply_bc_fn (the inflow term alone, after gdm_apply_planes) */
int gdm_add_boundary_fn(gdm_op *op, double *dst_owned, int fn_kind, const double *params, int n_params, double t_g,
                        double alpha, double t_k);

/* ----------------------------------------------------------------------
 * Postprocess on the device
 *   gdm_error_norms     the volume error norms of the reference's
 *                       postprocess (applications/advection/include/gdm/
 *                       advection/problem.h:269-425, the uncut mesh has no
 *                       immersed surface, so its *_face norms are 0):
 *                       norms_host = {Linf, L1, L2} of u - f(t) over
 *                       QGauss(p+1) on this rank's locally owned cells, f a
 *                       built-in function (gdm_fn_kind, same params as
 *                       gdm_eval_boundary).  u_local: engine-local vector
 *                       (ghost planes filled).  The caller reduces across
 *                       ranks as the reference does: Linf max, L1 sum,
 *                       L2 = sqrt(sum L2^2) (problem.h:410-425).
 *                       cell_errors (device, optional, n_owned_cells =
 *                       product of the owned cell counts, lexicographic
 *                       x fastest) = integrate_difference's per-cell L2
 *                       errors (include/gdm/vector_tools.h:25-86).
 * ---------------------------------------------------------------------- */
int gdm_error_norms(gdm_op *op, const double *u_local, int fn_kind, const double *params, int n_params, double t,
                    double *cell_errors, double *norms_host);

/* memory helpers for callers without their own device allocator */
int gdm_malloc(gdm_op *op, size_t bytes, void **ptr);
int gdm_free(gdm_op *op, void *ptr);
int gdm_memcpy_h2d(gdm_op *op, void *dst, const void *src_host, size_t bytes);
int gdm_memcpy_d2h(gdm_op *op, void *dst_host, const void *src, size_t bytes);

/* boundary points: coordinates of all n_bc_points device points (device
 * order; the caller evaluates its boundary data there, ghost-cell points
 * included) and ref_to_dev[i] = device index of the i-th point in the
 * reference's block(0) order (owned cells lexicographic, faces 0..2dim-1, q;
 * n_bc_points_ref entries). */
int gdm_bc_points(const gdm_op *op, double *xyz_host);
int gdm_bc_reference_order(const gdm_op *op, int64_t *ref_to_dev_host);

/* time n_iter back-to-back applications with HIP events on the operator's
 * stream; which: 0 = gdm_apply, 1 = gdm_mass_apply, 2 = gdm_mass_solve.
 * avg_ms_host receives the mean time per application. */
int gdm_time_op(gdm_op *op, int which, const double *src, double *dst, const double *bc_values, int n_iter,
                double *avg_ms_host);

/* ------------------------------------------------------------------------
 * Assembled sparse matrices: the irregular-stencil CG of
 * the cut-cell Poisson prototype and the on-disk triplet format.
 *
 *   gdm_csr_create       dealii::SparseMatrix<double>::reinit(sparsity) + the
 *                        assembled values (prototypes/cut_poisson_01_gdm.cc:
 *                        148-163, 327-336; full structural stencil of
 *                        System::create_sparsity_pattern, system.h:586-599).
 *                        Arrays are copied into device memory owned by the
 *                        handle; row_ptr int64 (n_rows+1), cols uint32 (the
 *                        reference's unsigned int indices), vals fp64.
 *                        src_is_device: 1 = the three arrays are device
 *                        pointers, 0 = host pointers.
 *   gdm_csr_vmult        SparseMatrix::vmult(dst, src) -- the matvec SolverCG
 *                        calls (cut_poisson_01_gdm.cc:335)
 *   gdm_csr_cg           SolverCG<>(ReductionControl(max_it, abs_tol, rel_tol))
 *                        .solve(A, x, b, P) with P = PreconditionIdentity
 *                        (precond 0, cut_poisson_01_gdm.cc:332-335) or
 *                        PreconditionJacobi (precond 1, omega = 1); x is the
 *                        initial guess; *its_host = last_step, *res_host = final
 *                        residual norm; GDM_ERR_STATE when max_it is reached.
 *   gdm_csr_read_triplets / gdm_csr_write_triplets
 *                        the binary / text triplet files of write_matrix_to_file
 *                        (applications/wave/wave-ev.cc:93-127): per entry u32
 *                        row, u32 column, f64 value (binary) or "row col value"
 *                        lines (text), rows ascending, diagonal first in each
 *                        square-matrix row (deal.II SparsityPattern order).
 *                        Reading sums duplicate (row, col) entries.
 * ---------------------------------------------------------------------- */
typedef struct gdm_csr gdm_csr;

int gdm_csr_create(int device, int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *row_ptr,
                   const uint32_t *cols, const double *vals, int src_is_device, gdm_csr **out);
int gdm_csr_destroy(gdm_csr *A);
int gdm_csr_info(const gdm_csr *A, int64_t *n_rows, int64_t *n_cols, int64_t *nnz);
int gdm_csr_set_stream(gdm_csr *A, void *hip_stream);
/* host copies of the three arrays (caller-allocated, sizes from gdm_csr_info) */
int gdm_csr_download(const gdm_csr *A, int64_t *row_ptr_host, uint32_t *cols_host, double *vals_host);
/* dst = A src (device pointers, dst of n_rows, src of n_cols entries) */
int gdm_csr_vmult(gdm_csr *A, const double *src, double *dst);
int gdm_csr_cg(gdm_csr *A, const double *b, double *x, int precond, int max_it, double abs_tol, double rel_tol,
               int *its_host, double *res_host);
int gdm_csr_read_triplets(int device, const char *path, int binary, gdm_csr **out);
int gdm_csr_write_triplets(const gdm_csr *A, const char *path, int binary);
/* mean time of n_iter back-to-back gdm_csr_vmult calls (HIP events, ms) */
int gdm_csr_time_vmult(gdm_csr *A, const double *src, double *dst, int n_iter, double *avg_ms_host);

/* ------------------------------------------------------------------------
 * Cut-cell systems: the 2D cut Poisson problem of
 * prototypes/cut_poisson_01_gdm.cc:57-405 assembled on the host
 * (csrc/gdm_cut.cpp) and solved by the device SpMV + SolverCG above.
 *
 *   gdm_cut_poisson_create   the reference's test<2>(ghost_penalty) system:
 *                            GDM degree p, n_sub^2 cells on [lo, hi]^2,
 *                            level set = FE_Q(1) interpolant of
 *                            |x - center| - radius (SignedDistance::Sphere),
 *                            NonMatching::MeshClassifier, the deal.II
 *                            QuadratureGenerator (Saye) on each intersected
 *                            cell, (grad v, grad u)_inside + Nitsche
 *                            (gamma = 5 (p+1) p) + ghost penalty (0.5 * 0.5 h
 *                            [d_n v][d_n u]) if ghost_penalty, rhs
 *                            rhs_value v + Nitsche data bc_value, zero
 *                            diagonals -> 1 (:148-323).  2D only.
 *   gdm_cut_poisson_matrix   the system matrix as a device CSR (gdm_csr_*)
 *   gdm_cut_poisson_csr      host copy of the CSR arrays (caller-allocated,
 *                            sizes from gdm_cut_poisson_info; ascending
 *                            columns, the entries cell assembly touches plus
 *                            every diagonal)
 *   gdm_cut_poisson_rhs      the right-hand side (host copy, n_rows values)
 *   gdm_cut_poisson_solve    SolverCG<>(ReductionControl(max_it, abs_tol,
 *                            rel_tol)).solve(A, u, rhs, PreconditionIdentity())
 *                            from u = 0 on the device (:332-335); A from
 *                            gdm_cut_poisson_matrix; u_host receives the
 *                            solution; GDM_ERR_STATE when max_it is reached
 *   gdm_cut_poisson_l2_error L2 error over the inside quadrature against the
 *                            manufactured solution bc + rhs/4 (r^2 - |x-c|^2)
 *                            (:349-405); u_host in the global DoF order
 * ------------------------------------------------------------------------ */
typedef struct gdm_cut_system gdm_cut_system;
int gdm_cut_poisson_create(int p, int n_sub, double lo, double hi, const double *center /* [2] or NULL */,
                           double radius, int ghost_penalty, double rhs_value, double bc_value, gdm_cut_system **out);
int gdm_cut_poisson_info(const gdm_cut_system *S, int64_t *n_rows, int64_t *nnz, int64_t *n_inside_cells,
                         int64_t *n_intersected_cells);
int gdm_cut_poisson_matrix(const gdm_cut_system *S, int device, gdm_csr **A);
int gdm_cut_poisson_csr(const gdm_cut_system *S, int64_t *row_ptr_host, uint32_t *cols_host, double *vals_host);
int gdm_cut_poisson_rhs(const gdm_cut_system *S, double *rhs_host);
int gdm_cut_poisson_solve(const gdm_cut_system *S, gdm_csr *A, double rel_tol, double abs_tol, int max_it,
                          double *u_host, int *its_host, double *res_host);
int gdm_cut_poisson_l2_error(const gdm_cut_system *S, const double *u_host, double *err);
int gdm_cut_poisson_destroy(gdm_cut_system *S);

/* ------------------------------------------------------------------------
 * Cut-cell advection (applications/advection, non-composite,
 * alpha = 0, 2D): the device compute_rhs / mass solve of the reference's
 * advection application on a mesh cut by an FE_Q(1) level set.
 *
 *   compute_rhs   rhs = Z S u + C u + F bc  (advection/stiffness.h:196-606):
 *                 S = the uncut fused Kronecker stencil of the box (the
 *                 advection operator of gdm_op_create with the box outflow
 *                 traces, no inflow data), Z zeroes the rows of the DoFs in
 *                 the box of a cell that is not fully inside, C =
 *                 those rows of the cut operator in full (volume and
 *                 outflow box-face terms of the inside cells, their cut
 *                 versions on intersected cells, outflow part of the
 *                 cut-surface term (II) :420-471) plus the ghost penalty
 *                 -0.5 gamma_A h^2 [d_n v][d_n u] (IV) :534-598, F = the
 *                 inflow data of (II) and (III) :473-532 (one column per
 *                 stage boundary point); C and F assembled on the host
 *                 (csrc/gdm_cut_advection.cpp), device CSR products.
 *   mass_solve    x = M_cut^-1 rhs exactly: banded Cholesky of the cut mass
 *                 (v, u)_inside + 0.5 gamma_M h^3 [d_n v][d_n u], zero
 *                 diagonals -> 1 (advection/mass.h:47-243), factored on the
 *                 host, triangular solves on the device (the SolverDirect
 *                 branch of advection/problem.h:262-265).  Up to 2^22 DoFs.
 *   bc_points     the stage boundary points (x, y) in the reference's
 *                 point_counter order (stiffness.h:40-160: per cell in
 *                 lexicographic order, its cut-surface points, then the inside
 *                 parts of its box faces in face order); block(0) of the
 *                 reference's BlockVector = the caller's values at them.
 *   op            the inner gdm_op (its stream; vector ops such as
 *                 gdm_vec_rk_update on these vectors).
 * level_set: the (n_sub + 1)^2 vertex values of the level set (x fastest);
 * cells with all values < 0 are inside, all > 0 outside (MeshClassifier).
 * u, bc, rhs, x: device pointers (n_dofs / n_bc_points doubles).
 * ------------------------------------------------------------------------ */
typedef struct gdm_cut_advection gdm_cut_advection;
int gdm_cut_advection_create(int fe_degree, int n_subdivisions, double left, double right, const double *level_set,
                             const double *advection /* [2] */, double ghost_parameter_A, double ghost_parameter_M,
                             int device, gdm_cut_advection **out);
/* cells[3] = inside, intersected, outside */
int gdm_cut_advection_info(const gdm_cut_advection *c, int64_t *n_dofs, int64_t *n_bc_points, int64_t *cells,
                           int64_t *mass_bandwidth);
int gdm_cut_advection_bc_points(const gdm_cut_advection *c, double *xy_host /* [n_bc_points][2] */);
int gdm_cut_advection_op(gdm_cut_advection *c, gdm_op **op);
int gdm_cut_advection_compute_rhs(gdm_cut_advection *c, const double *u, const double *bc, double *rhs);
int gdm_cut_advection_mass_solve(gdm_cut_advection *c, const double *rhs, double *x);
int gdm_cut_advection_destroy(gdm_cut_advection *c);
/* Composite advection (advection-app.cc's preset: params.composite, problem.h
 * :103-181; ABI v10): one handle per field.  location GDM_CUT_INSIDE (phi < 0,
 * params.advection) or GDM_CUT_OUTSIDE (phi > 0, params.advection_1; the
 * region, its box-face parts, the surface normal (stiffness.h:437), the ghost
 * penalty and the mass of MassMatrixOperator(location) follow the sign).
 * flags GDM_CUT_ADV_COMPOSITE: the inflow value u+ of the cut-surface term (II)
 * is the partner field evaluated at the surface point (stiffness.h:448-453),
 * so the surface points are no stage boundary points (collect_boundary_points
 * :115) and gdm_cut_advection_couple adds that part: rhs += P u_partner
 * (u_partner: the other field's DoF vector, same numbering).  compute_rhs(u,
 * bc, rhs) + couple(u_partner, rhs) = the field's block of compute_rhs
 * (stiffness.h:196-214); the box-face inflow (III) still reads bc.
 * gdm_cut_advection_create = create2(..., GDM_CUT_INSIDE, 0, ...). */
#define GDM_CUT_ADV_COMPOSITE 1
int gdm_cut_advection_create2(int fe_degree, int n_subdivisions, double left, double right, const double *level_set,
                              const double *advection /* [2] */, double ghost_parameter_A, double ghost_parameter_M,
                              int location, int flags, int device, gdm_cut_advection **out);
int gdm_cut_advection_couple(gdm_cut_advection *c, const double *u_partner, double *rhs);

/* ------------------------------------------------------------------------
 * Cut-cell wave / heat / poisson (applications/wave, dim 1 and
 * 2: the "wave", "heat-rk", "heat-impl", "heat-composite", "wave-composite"
 * and "step85" presets of wave-app.cc): the device operators of
 * the reference's wave application on a GDM line / square cut by the FE_Q(k)
 * interpolant of a level set (WaveProblem<dim>, wave/problem.h).
 *
 *   compute_rhs   rhs = [u != NULL] (Z S u + C u) + Ff fq + Fg gs
 *                 (wave/stiffness.h:42-407): S = the uncut wave stencil
 *                 -(grad v, grad u) of the box (gdm_op kind wave), Z zeroes
 *                 the rows of the DoFs in the box of a cell that is not fully
 *                 inside, C = those rows of -(grad v, grad u)_inside in full
 *                 + the surface Nitsche terms (:205-259, gamma_D = nitsche) +
 *                 the ghost penalty -0.5 gamma_A h [d_n v][d_n u] on the faces
 *                 (:330-395); Ff fq = (v, f) with fq = f at the inside
 *                 quadrature points, Fg gs = the Nitsche data
 *                 (gamma_D / h v - d_n v, g) with gs = g at the surface points
 *                 (either may be NULL: zero data).  Host assembly
 *                 csrc/gdm_cut_wave.cpp, device CSR products.
 *   mass_apply    out = M u, M = (v, u)_inside + 0.5 gamma_M h^3 [d_n v][d_n u],
 *                 zero diagonals -> 1 (wave/mass.h:47-249); gamma_M < 0 (the
 *                 reference's "not set", e.g. step85): no mass matrix
 *   mass_solve    x = M^-1 rhs (banded Cholesky: host factor, device
 *                 triangular solves; wave/problem.h:457-502)
 *   system_solve  x = (M + dt K)^-1 rhs, K the assembled stiffness matrix
 *                 (stiffness.h:602-800: (grad v, grad u)_inside + surface
 *                 Nitsche + 0.5 gamma_A h^3 [d_n v][d_n u], zero diagonals ->
 *                 1; heat-impl); refactored when dt changes
 *   stiffness_solve  x = K^-1 rhs (the "poisson" simulation type, problem.h:46-71)
 *   eval          vals = u_h at the inside quadrature points (the
 *                 postprocess of problem.h:504-615 reduces them with the
 *                 exact solution and the weights from gdm_cut_wave_points)
 * ls_values: per cell (lexicographic, x fastest) the level set at its
 * (k + 1)^dim Gauss-Lobatto support points (x fastest): the FE_Q(k)
 * interpolant.  Cells are classified by the signs of its Bernstein
 * coefficients (NonMatching::MeshClassifier); intersected cells get deal.II's
 * QuadratureGenerator (Saye) on the cell polynomial.  DoFs: vertices,
 * lexicographic (x fastest).  Vectors: device pointers (n_dofs, n_quad,
 * n_surface doubles).
 *
 * Composite presets (heat-composite, wave-composite; dim 1 and 2): one handle per
 * field, location GDM_CUT_INSIDE (phi < 0) or GDM_CUT_OUTSIDE (phi > 0), each
 * with its region's quadrature, mass and ghost-penalty faces (an intersected
 * cell and a neighbour not of the other location); flags select the Nitsche
 * data: GDM_CUT_WAVE_INTERFACE_DATA (II, the surface points; the presets
 * without composite), GDM_CUT_WAVE_DOMAIN_DATA (IV, the domain boundary faces
 * in the region, stiffness.h:262-330) and GDM_CUT_WAVE_COUPLED (the interface
 * terms of compute_rhs(BlockVector), stiffness.h:420-575: the own field's
 * part in compute_rhs, the partner's added by gdm_cut_wave_couple(c,
 * u_partner, rhs)).  The data points of gdm_cut_wave_points (sx, sn) are, cell
 * by cell, the interface points followed by the Gauss points of the cell's
 * domain faces (QGauss(p + 1) per face in 2D, outward normal), as selected.
 * A domain boundary face the level set crosses is refused (2D).
 * ------------------------------------------------------------------------ */
typedef struct gdm_cut_wave gdm_cut_wave;
#define GDM_CUT_INSIDE (-1)
#define GDM_CUT_OUTSIDE 1
#define GDM_CUT_WAVE_INTERFACE_DATA 1
#define GDM_CUT_WAVE_DOMAIN_DATA 2
#define GDM_CUT_WAVE_COUPLED 4
int gdm_cut_wave_create(int dim, int fe_degree, int n_subdivisions, double left, double right, int ls_degree,
                        const double *ls_values, int location, int flags, double gamma_M, double gamma_A,
                        double nitsche, int device, gdm_cut_wave **out);
/* cells[3] = inside, intersected, outside */
int gdm_cut_wave_info(const gdm_cut_wave *c, int64_t *n_dofs, int64_t *n_quad, int64_t *n_surface, int64_t *cells);
/* host arrays: quadrature points [n_quad][dim] and JxW [n_quad], surface points and unit normals [n_surface][dim] */
int gdm_cut_wave_points(const gdm_cut_wave *c, double *qx, double *qw, double *sx, double *sn);
int gdm_cut_wave_op(gdm_cut_wave *c, gdm_op **op);
int gdm_cut_wave_compute_rhs(gdm_cut_wave *c, const double *u, const double *fq, const double *gs, double *rhs);
int gdm_cut_wave_couple(gdm_cut_wave *c, const double *u_other, double *rhs);
int gdm_cut_wave_mass_apply(gdm_cut_wave *c, const double *u, double *out);
int gdm_cut_wave_mass_solve(gdm_cut_wave *c, const double *rhs, double *x);
int gdm_cut_wave_system_solve(gdm_cut_wave *c, double dt, const double *rhs, double *x);
int gdm_cut_wave_stiffness_solve(gdm_cut_wave *c, const double *rhs, double *x);
int gdm_cut_wave_eval(gdm_cut_wave *c, const double *u, double *vals);
int gdm_cut_wave_destroy(gdm_cut_wave *c);

#ifdef __cplusplus
}
#endif

#endif /* GDM_HIP_H */
