"""Device-resident time integration: the RK drivers of the reference's
problems over the C ABI, every vector in HBM.

  AdvectionProblem   applications/advection/include/gdm/advection/problem.h:31-102
                     (non-composite branch): y = (block(0) boundary values,
                     block(1) u); f(t, y) = (dg/dt, M^-1 (K u + inflow data))
  WaveProblem        applications/wave/include/gdm/wave/problem.h:280-346
                     (wave-rk): y = (u, v); f(t, y) = (v, M^-1 K u)

Both use TimeStepping::ExplicitRungeKutta with RK_CLASSIC_FOURTH_ORDER and
DiscreteTime, restated in low-storage form: the b-weighted sum of the stages
is accumulated as each stage is produced (gdm_vec_rk_update: one pass writes
the accumulator and the next stage vector), in the same order as deal.II's
final y.sadd loop, so no per-stage BlockVector is allocated (problem.h:64-65)
and nothing crosses PCIe inside the loop.  Block(0) of the advection problem
is g(t_n) at the start of every step (initialize_time_step,
advection/stiffness.h:181-194) and dg/dt at the stage times
(stiffness.h:286-289), both evaluated on the device for the built-in
boundary functions.  By default block(0) is not stored at all: stage s reads
y0 + h a_{s,s-1} k_{s-1} = g(t_n) + h a dg/dt(t_n + c_{s-1} h), which the
engine computes per stage itself (gdm_apply_bc_fn, the same bits as
gdm_eval_boundary + gdm_vec_rk_update); block(0) after a step is never read
by the reference (initialize_time_step overwrites it, problem.h:88-90).
carry_bc=True keeps the explicit block(0) vectors (gdm_eval_boundary).
"""
from ._capi import GdmError

# RK_CLASSIC_FOURTH_ORDER (deal.II TimeStepping): c, a_{i,i-1}, b
RK4_C = (0.0, 0.5, 0.5, 1.0)
RK4_A = (0.5, 0.5, 1.0)
RK4_B = (1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0)


class DiscreteTime:
    """deal.II DiscreteTime (base/discrete_time.cc): the next time is the
    current one plus the last step, the step recomputed as the difference of
    the two times (round-off accumulates as in the reference), snapped to the
    end time when within 5 % of a step of it."""

    def __init__(self, start, end, dt):
        self.t, self.end, self.step = float(start), float(end), 0
        self._next = self._next_time(self.t, float(dt))

    def _next_time(self, current, step):
        n = current + step
        if step > 0.0 and n > self.end - 0.05 * step:
            n = self.end
        return n

    def is_at_end(self):
        return self.t == self.end

    def next_step_size(self):
        return self._next - self.t

    def advance(self):
        step = self._next - self.t
        self.t = self._next
        self._next = self._next_time(self.t, step)
        self.step += 1

class WaveProblem:
    """wave-rk on one rank: du/dt = v, dv/dt = M^-1 (K u) with K the wave
    operator of `op` (kind "wave": -(grad v, grad u) [+ box Nitsche])."""

    def __init__(self, op):
        if op.mesh.n_ranks != 1:
            raise GdmError("WaveProblem: single-rank driver (multi-rank: gdm_amd.distributed)")
        self.op = op
        n = op.n_owned
        self.u, self.v = op.new_vector(False), op.new_vector(False)
        self._acc = [op.new_vector(False) for _ in range(2)]
        self._Y = [op.new_vector(False) for _ in range(2)]
        self._kv = op.new_vector(False)
        self.n = n

    def rhs(self, t, U, out):
        """dv/dt = M^-1 compute_rhs(U) (wave/problem.h:313-317)"""
        self.op.apply(U, out)
        self.op.mass_solve(out, out)
        return out

    def step(self, t, h):
        op, y = self.op, (self.u, self.v)
        acc, Y, kv = self._acc, self._Y, self._kv
        stage = y
        for s in range(4):
            # k = (stage_v, M^-1 K stage_u)
            op.apply(stage[0], kv)
            ku = stage[1]
            last = s == 3
            acc_in = y if s == 0 else acc
            acc_out = y if last else acc
            a_next = 0.0 if last else h * RK4_A[s]
            # u block first (stage_u is consumed): it reads ku = stage_v before
            # the v block overwrites Y_v
            op.rk_update(h * RK4_B[s], ku, acc_in[0], acc_out[0], a_next, None if last else y[0],
                         None if last else Y[0])
            # v block: the mass solve with the update fused into its last pass
            op.mass_solve_rk(kv, h * RK4_B[s], acc_in[1], acc_out[1], a_next, None if last else y[1],
                             None if last else Y[1])
            stage = Y

    def run(self, start_t, end_t, dt, max_steps=None, callback=None):
        time = DiscreteTime(start_t, end_t, dt)
        n = 0
        while not time.is_at_end() and (max_steps is None or n < max_steps):
            h = time.next_step_size()
            self.step(time.t, h)
            n += 1
            if callback is not None:
                callback(time.t + h, self)
            time.advance()
        return n


class AdvectionProblem:
    """advection problem.h:31-102 on one rank with a built-in boundary
    function (gdm_fn_kind) for g and dg/dt."""

    def __init__(self, op, fn_kind, fn_params, carry_bc=False):
        if op.mesh.n_ranks != 1:
            raise GdmError("AdvectionProblem: single-rank driver")
        self.op, self.fn, self.prm = op, int(fn_kind), list(fn_params)
        self.carry_bc = bool(carry_bc)
        import torch

        dev = "cuda:%d" % op.device
        # block(0) (the boundary points, ~28 M at C3) exists only on the explicit
        # path: with carry_bc=False the engine computes the stage values itself
        nb = max(op.n_bc_points, 1) if self.carry_bc else 0
        z = lambda m: torch.zeros(m, dtype=torch.float64, device=dev) if m else None  # noqa: E731
        self.u = op.new_vector(False)
        self._bc = z(nb)
        self._acc = [z(nb), op.new_vector(False)]
        self._Y = [z(nb), op.new_vector(False)]
        self._k = [z(nb), op.new_vector(False)]

    @property
    def bc(self):
        """block(0) = g at the boundary points; kept only with carry_bc=True"""
        if not self.carry_bc:
            raise GdmError("AdvectionProblem.bc: block(0) is not kept (carry_bc=False computes the stage "
                           "boundary values on the device)")
        return self._bc

    def initialize_time_step(self, t):
        """block(0) = g(t_n) at the boundary points (stiffness.h:181-194).
        With carry_bc=False there is no block(0) to fill: step() has the
        engine evaluate g(t_n) (+ the stage terms) right before each stencil,
        so this is a no-op and returns False; True when block(0)
        was written."""
        if not self.carry_bc:
            return False
        if self.op.n_bc_points:
            self.op.eval_boundary(self.fn, self.prm, t, 0, self.bc)
        return True

    def rhs(self, t, BC, U, kbc, ku):
        op = self.op
        if op.n_bc_points:
            op.eval_boundary(self.fn, self.prm, t, 1, kbc)  # block(0) = dg/dt (stiffness.h:286-289)
        op.apply(U, ku, BC if op.n_bc_points else None)
        op.mass_solve(ku, ku)

    def step(self, t, h):
        op = self.op
        if not self.carry_bc:
            # block(0) computed by the engine: stage s reads g(t) + alpha dg/dt(t_k)
            y, acc, Y, k = self.u, self._acc[1], self._Y[1], self._k[1]
            stage = y
            for s in range(4):
                alpha, t_k = (0.0, t) if s == 0 else (h * RK4_A[s - 1], t + RK4_C[s - 1] * h)
                op.apply_bc_fn(stage, k, self.fn, self.prm, t, alpha, t_k)
                last = s == 3
                op.mass_solve_rk(k, h * RK4_B[s], y if s == 0 else acc, y if last else acc,
                                 0.0 if last else h * RK4_A[s], None if last else y, None if last else Y)
                stage = Y
            return
        self.initialize_time_step(t)
        y = (self.bc, self.u)
        acc, Y, k = self._acc, self._Y, self._k
        stage = y
        blocks = (0, 1) if op.n_bc_points else (1,)
        for s in range(4):
            self.rhs(t + RK4_C[s] * h, stage[0], stage[1], k[0], k[1])
            last = s == 3
            a_next = 0.0 if last else h * RK4_A[s]
            for b in blocks:
                op.rk_update(h * RK4_B[s], k[b], (y if s == 0 else acc)[b], (y if last else acc)[b], a_next,
                             None if last else y[b], None if last else Y[b])
            stage = Y

    def run(self, start_t, end_t, dt, max_steps=None):
        time = DiscreteTime(start_t, end_t, dt)
        n = 0
        while not time.is_at_end() and (max_steps is None or n < max_steps):
            self.step(time.t, time.next_step_size())
            n += 1
            time.advance()
        return n


class Advection01:
    """prototypes/advection_01_gdm.cc:62-282 (use_mass_lumping = false) on the
    device: periodicity constraints in every direction (:107-110), the
    convective form cell_i -= (a . grad u_q) phi_i JxW (:164-206) on the
    distributed stage vector, SolverCG + PreconditionJacobi with
    ReductionControl(100, 1e-10, 1e-8) from a zero initial guess (:208-217),
    RK_CLASSIC_FOURTH_ORDER + DiscreteTime, constraints.distribute after
    every step (:268).  `op` is a "convective" operator with periodic = all
    directions."""

    def __init__(self, op):
        if op.mesh.n_ranks != 1:
            raise GdmError("Advection01: single rank")
        self.op = op
        self.u = op.new_vector(False)
        self._acc, self._Y, self._k = (op.new_vector(False) for _ in range(3))
        self.cg_iterations = []

    def rhs(self, U, out):
        op = self.op
        op.apply(U, self._r_tmp())  # distributes a copy of U, condenses the result
        out.zero_()
        its, _ = op.mass_solve_cg(self._r, out, rel_tol=1e-8, abs_tol=1e-10, max_it=100, precond=1)
        self.cg_iterations.append(its)
        return out

    def _r_tmp(self):
        if not hasattr(self, "_r"):
            self._r = self.op.new_vector(False)
        return self._r

    def step(self, t, h):
        op, y = self.op, self.u
        acc, Y, k = self._acc, self._Y, self._k
        stage = y
        for s in range(4):
            self.rhs(stage, k)
            last = s == 3
            op.rk_update(h * RK4_B[s], k, y if s == 0 else acc, y if last else acc,
                         0.0 if last else h * RK4_A[s], None if last else y, None if last else Y)
            stage = Y
        op.distribute(y)

    def run(self, start_t, end_t, dt, max_steps=None):
        time = DiscreteTime(start_t, end_t, dt)
        n = 0
        while not time.is_at_end() and (max_steps is None or n < max_steps):
            self.step(time.t, time.next_step_size())
            n += 1
            time.advance()
        return n
