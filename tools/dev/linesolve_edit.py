R = '/root/repo/'
h = open(R + 'include/gdm_hip.h').read()
old = "/* y = a x + b y ; *result_host = x . y */"
new = """/* In-place banded-Cholesky solve with the 1D mass matrix of reference
 * direction `axis` (0 = x, 1 = y, 2 = z) along n_lines lines of full length
 * N[axis]: line l starts at v + (l / A) * B + (l % A) * C and its entries are
 * `stride` apart.  The building block of the distributed mass inverse (the
 * slab-local directions are solved in place, the partitioned one after a
 * transpose; gdm_amd/distributed.py), replacing the CG of
 * advection/problem.h:236-267 on a multi-rank mesh. */
int gdm_mass_solve_lines(gdm_op *op, int axis, double *v, int64_t n_lines, int64_t stride, int64_t A, int64_t B,
                         int64_t C);

/* y = a x + b y ; *result_host = x . y */"""
assert old in h
h = h.replace(old, new)
open(R + 'include/gdm_hip.h', 'w').write(h)

s = open(R + 'dealii-galerkin-difference-methods_amd/csrc/gdm_capi.cpp').read()
old = "int gdm_vec_axpby(gdm_op *op, int64_t n, double a, const double *x, double b, double *y) {"
new = """int gdm_mass_solve_lines(gdm_op *op, int axis, double *v, int64_t n_lines, int64_t stride, int64_t A, int64_t B,
                         int64_t C) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (axis < 0 || axis >= op->dim) return fail(GDM_ERR_ARG, "axis out of range");
  if (n_lines < 0 || stride <= 0 || A <= 0) return fail(GDM_ERR_ARG, "bad line geometry");
  if (n_lines > 0 && !v) return fail(GDM_ERR_ARG, "NULL vector");
  int kax = -1;
  for (int ax = 0; ax < 3; ++ax)
    if (op->kdir[ax] == axis) kax = ax;
  if (kax < 0 || !op->lrow[kax]) return n_lines == 0 || op->N[axis] <= 1 ? GDM_OK : fail(GDM_ERR_STATE, "no factor");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(gdmk_launch_chol_lines(op->p, v, op->N[axis], stride, n_lines, A, B, C, op->lrow[kax], op->invd[kax],
                                   op->stream),
            "chol lines");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_vec_axpby(gdm_op *op, int64_t n, double a, const double *x, double b, double *y) {"""
assert old in s
s = s.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/csrc/gdm_capi.cpp', 'w').write(s)

c = open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/_capi.py').read()
old = '        "gdm_mass_solve": [P, P, P],'
new = '        "gdm_mass_solve": [P, P, P],\n        "gdm_mass_solve_lines": [P, i32, P, i64, i64, i64, i64, i64],'
assert old in c
c = c.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/_capi.py', 'w').write(c)

o = open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/operator.py').read()
old = """    def axpby(self, a, x, b, y):"""
new = """    def mass_solve_lines(self, axis, v, n_lines, stride, A, B, C):
        \"\"\"In-place 1D mass solves along `axis` (gdm_mass_solve_lines).\"\"\"
        check(self.lib.gdm_mass_solve_lines(self.h, int(axis), _ptr(v), int(n_lines), int(stride), int(A), int(B),
                                            int(C)), "gdm_mass_solve_lines")
        return v

    def axpby(self, a, x, b, y):"""
assert old in o
o = o.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/operator.py', 'w').write(o)
print("ok")
