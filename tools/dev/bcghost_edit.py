import re
R = '/root/repo/'
# --- header: ABI v2, new layout field
h = open(R + 'include/gdm_hip.h').read()
h = h.replace("#define GDM_HIP_ABI_VERSION 1", "#define GDM_HIP_ABI_VERSION 2")
old = "  int64_t n_bc_points;            /* block(0) size (boundary points of owned cells) */\n} gdm_layout;"
new = """  int64_t n_bc_points;            /* device block(0) size: boundary points of the owned
                                     cells plus, on a multi-rank mesh, those of the
                                     neighbour cells whose DoF boxes reach owned DoFs
                                     (owner-computes replaces compress(add)) */
  int64_t n_bc_points_ref;        /* the reference's block(0) size: points of the owned
                                     cells only (stiffness.h:40-160)                  */
} gdm_layout;"""
assert old in h
h = h.replace(old, new)
old = """/* boundary points of the owned cells: coordinates (n_bc_points x 3, device
 * order) and ref_to_dev[i] = device index of the i-th point in the
 * reference's block(0) order (cells lexicographic, faces 0..2dim-1, q). */"""
new = """/* boundary points: coordinates of all n_bc_points device points (device
 * order; the caller evaluates its boundary data there, ghost-cell points
 * included) and ref_to_dev[i] = device index of the i-th point in the
 * reference's block(0) order (owned cells lexicographic, faces 0..2dim-1, q;
 * n_bc_points_ref entries). */"""
assert old in h
h = h.replace(old, new)
open(R + 'include/gdm_hip.h', 'w').write(h)

# --- ctypes layout
c = open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/_capi.py').read()
old = '        ("n_bc_points", ctypes.c_int64),\n    ]'
assert old in c
c = c.replace(old, '        ("n_bc_points", ctypes.c_int64),\n        ("n_bc_points_ref", ctypes.c_int64),\n    ]')
open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/_capi.py', 'w').write(c)

o = open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/operator.py').read()
old = """    def bc_reference_order(self):
        n = self.n_bc_points"""
new = """    @property
    def n_bc_points_ref(self):
        return self.layout["n_bc_points_ref"]

    def bc_reference_order(self):
        n = self.n_bc_points_ref"""
assert old in o
o = o.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/gdm_amd/operator.py', 'w').write(o)

# --- capi: extended cell range in the partition direction, counts
s = open(R + 'dealii-galerkin-difference-methods_amd/csrc/gdm_capi.cpp').read()
old = """      if (e == q) {
        cb = (unsigned)L.cell_plane_begin;
        ce = (unsigned)L.cell_plane_end;
        nb = L.owned_plane_begin;
        ne = L.owned_plane_end;
      }"""
new = """      if (e == q) {
        // owner-computes: every cell whose DoF box reaches an owned node, the
        // neighbour ranks' cells included (their points are ghost points)
        nb = L.owned_plane_begin;
        ne = L.owned_plane_end;
        cb = nce;
        ce = 0;
        for (unsigned c = 0; c < nce; ++c) {
          const int off = (int)gdm::box_offset(c, p, nce);
          if (off + p >= nb && off <= ne - 1) {
            cb = std::min(cb, c);
            ce = std::max(ce, c + 1);
          }
        }
        if (ce <= cb) cb = ce = (unsigned)L.cell_plane_begin;
      }"""
assert old in s
s = s.replace(old, new)
old = """  op->layout.n_bc_points = offset;"""
new = """  op->layout.n_bc_points = offset;
  // the reference's block(0): points of the owned cells only
  {
    int64_t nref = 0;
    const int n1q = p + 1;
    const int nfq = dim == 1 ? 1 : (dim == 2 ? n1q : n1q * n1q);
    int ncell[3] = {1, 1, 1};
    for (int d = 0; d < dim; ++d) ncell[d] = op->mesh.n_subdivisions[d];
    for (const Face &F : op->faces) {
      // owned cells adjacent to face F: product of the tangential owned cell counts
      int64_t cells = 1;
      for (int e = 0; e < dim; ++e) {
        if (e == F.d) continue;
        cells *= e == q ? (L.cell_plane_end - L.cell_plane_begin) : ncell[e];
      }
      nref += cells * nfq;
    }
    op->layout.n_bc_points_ref = nref;
  }"""
assert old in s
s = s.replace(old, new)
old = """  if (k != L.n_bc_points) return fail(GDM_ERR_STATE, "boundary point count mismatch");"""
new = """  if (k != L.n_bc_points_ref) return fail(GDM_ERR_STATE, "boundary point count mismatch");"""
assert old in s
s = s.replace(old, new)
open(R + 'dealii-galerkin-difference-methods_amd/csrc/gdm_capi.cpp', 'w').write(s)
print("ok")
