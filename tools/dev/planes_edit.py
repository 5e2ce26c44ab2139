R = '/root/repo/'
s = open(R + 'dealii-galerkin-difference-methods_amd/csrc/gdm_capi.cpp').read()
s = s.replace("hipError_t launch_stencil(gdm_op *op, bool mass, const double *src, double *dst) {",
"""// Output planes [zb, ze) of the owned range (3D: z planes; the full owned
// range otherwise).  dst is the owned vector; only those planes are written.
hipError_t launch_stencil(gdm_op *op, bool mass, const double *src, double *dst, int zb = -1, int ze = -1) {""")
old = """  a.zchunk = std::max(1, std::min(op->zchunk, a.out_z1 - a.out_z0));
  a.x_toep = op->x_toep;"""
new = """  if (zb < 0) zb = a.out_z0;
  if (ze < 0) ze = a.out_z1;
  zb = std::max(zb, a.out_z0);
  ze = std::min(ze, a.out_z1);
  if (ze <= zb) return hipSuccess;
  a.zchunk = std::max(1, std::min(op->zchunk, ze - zb));
  a.x_toep = op->x_toep;"""
assert old in s; s = s.replace(old, new)
old = "  if (!v8) return gdmk_launch_stencil(op->p, bk, a, op->stream);"
new = """  if (!v8) {
    // v7 indexes dst relative to out_z0: shift both to the sub-range
    a.dst = dst + (int64_t)(zb - a.out_z0) * L.plane_size;
    a.out_z0 = zb;
    a.out_z1 = ze;
    return gdmk_launch_stencil(op->p, bk, a, op->stream);
  }"""
assert old in s; s = s.replace(old, new)
s = s.replace("  const int i0 = std::max(a.out_z0, zlo), i1 = std::min(a.out_z1, zhi);",
              "  const int i0 = std::max(zb, zlo), i1 = std::min(ze, zhi);")
s = s.replace("""    a.cz0[0] = a.out_z0; a.cz1[0] = a.out_z1; a.cz0[1] = a.cz1[1] = 0;
    a.zchunk = zchunk_for(a.out_z1 - a.out_z0);""", """    a.cz0[0] = zb; a.cz1[0] = ze; a.cz0[1] = a.cz1[1] = 0;
    a.zchunk = zchunk_for(ze - zb);""")
s = s.replace("""  a.cz0[0] = a.out_z0; a.cz1[0] = i0;
  a.cz0[1] = i1; a.cz1[1] = a.out_z1;
  a.zchunk = std::max(1, std::max(i0 - a.out_z0, a.out_z1 - i1));
  a.nchunk0 = i0 > a.out_z0 ? 1 : 0;
  if (i0 <= a.out_z0 && i1 >= a.out_z1) return hipSuccess;""", """  a.cz0[0] = zb; a.cz1[0] = i0;
  a.cz0[1] = i1; a.cz1[1] = ze;
  a.zchunk = std::max(1, std::max(i0 - zb, ze - i1));
  a.nchunk0 = i0 > zb ? 1 : 0;
  if (i0 <= zb && i1 >= ze) return hipSuccess;""")
old = "int gdm_add_boundary_data(gdm_op *op, const double *bc_values, double *dst_owned) {"
new = """int gdm_apply_planes(gdm_op *op, const double *src_local, double *dst_owned, int plane_begin, int plane_end) {
  if (!op) return fail(GDM_ERR_ARG, "op is NULL");
  if (op->layout.n_owned > 0 && (!src_local || !dst_owned)) return fail(GDM_ERR_ARG, "NULL vector");
  if (op->part_axis != 2 && (plane_begin > op->layout.owned_plane_begin || plane_end < op->layout.owned_plane_end))
    return fail(GDM_ERR_UNSUPPORTED, "gdm_apply_planes: plane sub-ranges need a 3D mesh");
  GDM_GUARD_BEGIN
  hip_check(hipSetDevice(op->device), "hipSetDevice");
  hip_check(launch_stencil(op, op->kind == GDM_OP_MASS, src_local, dst_owned, plane_begin, plane_end),
            "stencil launch");
  return GDM_OK;
  GDM_GUARD_END
}

int gdm_add_boundary_data(gdm_op *op, const double *bc_values, double *dst_owned) {"""
assert old in s; s = s.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/csrc/gdm_capi.cpp', 'w').write(s)

h = open(R + 'include/gdm_hip.h').read()
old = """/* dst_owned += inflow boundary-data term only"""
new = """/* The volume part of gdm_apply for the owned output planes [plane_begin,
 * plane_end) of the last coordinate only (global plane indices; 3D).  Lets a
 * multi-rank caller compute the planes that need no ghost data while the
 * ghost-plane exchange is in flight, then the p planes next to each slab edge
 * (the overlap of update_ghost_values, advection/stiffness.h:343, with the cell
 * loop).  Boundary data: gdm_add_boundary_data afterwards. */
int gdm_apply_planes(gdm_op *op, const double *src_local, double *dst_owned, int plane_begin, int plane_end);
/* dst_owned += inflow boundary-data term only"""
assert old in h; h = h.replace(old, new)
open(R + 'include/gdm_hip.h', 'w').write(h)

c = open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/_capi.py').read()
old = '        "gdm_add_boundary_data": [P, P, P],'
assert old in c
c = c.replace(old, old + '\n        "gdm_apply_planes": [P, P, P, i32, i32],')
open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/_capi.py', 'w').write(c)

o = open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/operator.py').read()
old = """    def add_boundary_data(self, bc_values, dst_owned):"""
new = """    def apply_planes(self, src_local, dst_owned, plane_begin, plane_end):
        \"\"\"Volume term for the owned output planes [plane_begin, plane_end) only.\"\"\"
        self._check_sizes(src_local, dst_owned)
        check(self.lib.gdm_apply_planes(self.h, _ptr(src_local), _ptr(dst_owned), int(plane_begin), int(plane_end)),
              "gdm_apply_planes")
        return dst_owned

    def add_boundary_data(self, bc_values, dst_owned):"""
assert old in o; o = o.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/operator.py', 'w').write(o)
print("ok")
