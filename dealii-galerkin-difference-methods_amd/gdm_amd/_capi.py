"""ctypes binding of libgdm_hip.so (include/gdm_hip.h).

The product path: every device computation goes through these entry points.
There is no CPU fallback -- if the library or a GPU is missing, operator
construction raises GdmError.
"""
import ctypes
import importlib.util
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("GDM_HIP_LIB") or os.path.join(PKG_ROOT, "lib", "libgdm_hip.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "gdm_hip.h")

GDM_OK = 0
GDM_OP_MASS, GDM_OP_ADVECTION, GDM_OP_WAVE, GDM_OP_CONVECTIVE = 0, 1, 2, 3


class GdmError(RuntimeError):
    pass


class MeshDesc(ctypes.Structure):
    _fields_ = [
        ("dim", ctypes.c_int32),
        ("fe_degree", ctypes.c_int32),
        ("n_subdivisions", ctypes.c_int32 * 3),
        ("lo", ctypes.c_double * 3),
        ("hi", ctypes.c_double * 3),
        ("n_ranks", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("periodic", ctypes.c_int32),
    ]


class Halo(ctypes.Structure):
    _fields_ = [
        ("rank_below", ctypes.c_int32),
        ("rank_above", ctypes.c_int32),
        ("owned_offset", ctypes.c_int64),
        ("send_below_offset", ctypes.c_int64),
        ("send_below_count", ctypes.c_int64),
        ("recv_below_offset", ctypes.c_int64),
        ("recv_below_count", ctypes.c_int64),
        ("send_above_offset", ctypes.c_int64),
        ("send_above_count", ctypes.c_int64),
        ("recv_above_offset", ctypes.c_int64),
        ("recv_above_count", ctypes.c_int64),
        ("dealii_ghost_planes_below", ctypes.c_int32),
        ("dealii_ghost_planes_above", ctypes.c_int32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Layout(ctypes.Structure):
    _fields_ = [
        ("n_dofs_global", ctypes.c_int64),
        ("plane_size", ctypes.c_int64),
        ("n_planes_global", ctypes.c_int32),
        ("owned_plane_begin", ctypes.c_int32),
        ("owned_plane_end", ctypes.c_int32),
        ("ghost_planes_below", ctypes.c_int32),
        ("ghost_planes_above", ctypes.c_int32),
        ("cell_plane_begin", ctypes.c_int32),
        ("cell_plane_end", ctypes.c_int32),
        ("halo_depth", ctypes.c_int32),
        ("n_owned", ctypes.c_int64),
        ("n_local", ctypes.c_int64),
        ("n_bc_points", ctypes.c_int64),
        ("n_bc_points_ref", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def torch_hip_runtime():
    """Path of the HIP runtime torch ships (None when torch is absent).

    libgdm_hip.so NEEDs `libamdhip64.so.7` (RUNPATH /opt/rocm/lib) while
    libtorch_hip NEEDs torch's own copy, whose soname is the same
    `libamdhip64.so.7`.  Loaded first, the engine would map /opt/rocm's
    runtime and a later `import torch` a second one (plus a second
    libhsa-runtime64): two HIP runtimes in one process.  Preloading torch's
    copy makes the dynamic linker satisfy the engine's NEEDED entry by soname
    and torch's by file identity, so every Python process maps exactly one.
    """
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return None
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    return path if os.path.exists(path) else None


def load():
    """Load libgdm_hip.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GdmError("libgdm_hip.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    rt = torch_hip_runtime()
    if rt is not None:
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    sig = {
        "gdm_last_error": [ctypes.c_char_p, ctypes.c_size_t],
        "gdm_abi_version": [],
        "gdm_get_device_count": [ctypes.POINTER(ctypes.c_int)],
        "gdm_op_create": [ctypes.POINTER(MeshDesc), i32, P, i32, i32, ctypes.POINTER(P)],
        "gdm_op_destroy": [P],
        "gdm_op_layout": [P, ctypes.POINTER(Layout)],
        "gdm_halo_plan": [ctypes.POINTER(MeshDesc), ctypes.POINTER(Halo)],
        "gdm_mass_diagonal": [P, P],
        "gdm_memcpy_d2d": [P, P, P, ctypes.c_size_t],
        "gdm_vec_pointwise_mult": [P, i64, P, P, P],
        "gdm_op_set_stream": [P, P],
        "gdm_op_use_own_stream": [P],
        "gdm_op_get_stream": [P, P],
        "gdm_apply": [P, P, P, P],
        "gdm_add_boundary_data": [P, P, P],
        "gdm_apply_planes": [P, P, P, i32, i32],
        "gdm_apply_planes2": [P, P, P, i32, i32, i32, i32],
        "gdm_mass_apply": [P, P, P],
        "gdm_mass_solve": [P, P, P],
        "gdm_mass_solve_rk": [P, P, d, P, P, d, P, P],
        "gdm_constraints_distribute": [P, P],
        "gdm_mass_solve_cg": [P, P, P, d, d, i32, i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(d)],
        "gdm_mass_solve_lines": [P, i32, P, i64, i64, i64, i64, i64],
        "gdm_vec_axpby": [P, i64, d, P, d, P],
        "gdm_vec_dot": [P, i64, P, P, ctypes.POINTER(d)],
        "gdm_vec_rk_update": [P, i64, d, P, P, P, d, P, P],
        "gdm_eval_boundary": [P, i32, P, i32, d, i32, P],
        "gdm_apply_bc_fn": [P, P, P, i32, P, i32, d, d, d],
        "gdm_add_boundary_fn": [P, P, i32, P, i32, d, d, d],
        "gdm_error_norms": [P, P, i32, P, i32, d, P, P],
        "gdm_mass_spike_eps": [P, P],
        "gdm_mass_solve_slab": [P, P, P],
        "gdm_mass_solve_interface": [P, P],
        "gdm_mass_solve_interface_ghosts": [P, P],
        "gdm_mass_solve_interface_rk": [P, P, d, P, P, d, P, P],
        "gdm_mass_solve_interface_round": [P, P, i32],
        "gdm_mass_spike_rounds": [P, ctypes.POINTER(ctypes.c_int)],
        "gdm_synchronize": [P],
        "gdm_malloc": [P, ctypes.c_size_t, ctypes.POINTER(P)],
        "gdm_free": [P, P],
        "gdm_memcpy_h2d": [P, P, P, ctypes.c_size_t],
        "gdm_memcpy_d2h": [P, P, P, ctypes.c_size_t],
        "gdm_bc_points": [P, P],
        "gdm_bc_reference_order": [P, P],
        "gdm_time_op": [P, i32, P, P, P, i32, ctypes.POINTER(d)],
        "gdm_csr_create": [i32, i64, i64, i64, P, P, P, i32, ctypes.POINTER(P)],
        "gdm_csr_destroy": [P],
        "gdm_csr_info": [P, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64)],
        "gdm_csr_set_stream": [P, P],
        "gdm_csr_download": [P, P, P, P],
        "gdm_csr_vmult": [P, P, P],
        "gdm_csr_cg": [P, P, P, i32, i32, d, d, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(d)],
        "gdm_csr_read_triplets": [i32, ctypes.c_char_p, i32, ctypes.POINTER(P)],
        "gdm_csr_write_triplets": [P, ctypes.c_char_p, i32],
        "gdm_csr_time_vmult": [P, P, P, i32, ctypes.POINTER(d)],
        "gdm_cut_poisson_create": [i32, i32, d, d, P, d, i32, d, d, ctypes.POINTER(P)],
        "gdm_cut_poisson_info": [P, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64),
                                 ctypes.POINTER(i64)],
        "gdm_cut_poisson_matrix": [P, i32, ctypes.POINTER(P)],
        "gdm_cut_poisson_csr": [P, P, P, P],
        "gdm_cut_poisson_rhs": [P, P],
        "gdm_cut_poisson_solve": [P, P, d, d, i32, P, ctypes.POINTER(i32), ctypes.POINTER(d)],
        "gdm_cut_poisson_l2_error": [P, P, ctypes.POINTER(d)],
        "gdm_cut_poisson_destroy": [P],
        "gdm_cut_advection_create": [i32, i32, d, d, P, P, d, d, i32, ctypes.POINTER(P)],
        "gdm_cut_advection_info": [P, ctypes.POINTER(i64), ctypes.POINTER(i64), P, ctypes.POINTER(i64)],
        "gdm_cut_advection_bc_points": [P, P],
        "gdm_cut_advection_op": [P, ctypes.POINTER(P)],
        "gdm_cut_advection_compute_rhs": [P, P, P, P],
        "gdm_cut_advection_mass_solve": [P, P, P],
        "gdm_cut_advection_create2": [i32, i32, d, d, P, P, d, d, i32, i32, i32, ctypes.POINTER(P)],
        "gdm_cut_advection_couple": [P, P, P],
        "gdm_cut_advection_destroy": [P],
        "gdm_cut_wave_create": [i32, i32, i32, d, d, i32, P, i32, i32, d, d, d, i32, ctypes.POINTER(P)],
        "gdm_cut_wave_info": [P, ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64), P],
        "gdm_cut_wave_points": [P, P, P, P, P],
        "gdm_cut_wave_op": [P, ctypes.POINTER(P)],
        "gdm_cut_wave_compute_rhs": [P, P, P, P, P],
        "gdm_cut_wave_couple": [P, P, P],
        "gdm_cut_wave_mass_apply": [P, P, P],
        "gdm_cut_wave_mass_solve": [P, P, P],
        "gdm_cut_wave_system_solve": [P, d, P, P],
        "gdm_cut_wave_stiffness_solve": [P, P, P],
        "gdm_cut_wave_eval": [P, P, P],
        "gdm_cut_wave_destroy": [P],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    _lib = L
    return L


def last_error():
    buf = ctypes.create_string_buffer(1024)
    load().gdm_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(rc, what=""):
    if rc != GDM_OK:
        raise GdmError("%s failed (%d): %s" % (what, rc, last_error()))
    return rc


def declared_symbols():
    """Every function the public header declares (for the export test)."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^int\s+(gdm_\w+)\s*\(", txt, flags=re.M)))


def device_count():
    n = ctypes.c_int(0)
    rc = load().gdm_get_device_count(ctypes.byref(n))
    return n.value if rc == GDM_OK else 0


def mesh_desc(dim, fe_degree, n_subdivisions, lo=0.0, hi=1.0, n_ranks=1, rank=0, periodic=0):
    m = MeshDesc()
    m.dim, m.fe_degree = dim, fe_degree
    ns = list(n_subdivisions) if hasattr(n_subdivisions, "__len__") else [n_subdivisions] * dim
    for d in range(3):
        m.n_subdivisions[d] = int(ns[d]) if d < dim else 1
        m.lo[d] = float(lo) if d < dim else 0.0
        m.hi[d] = float(hi) if d < dim else 1.0
    m.n_ranks, m.rank, m.periodic = n_ranks, rank, periodic
    return m


def mass_spike_rounds(dim, fe_degree, n_subdivisions, n_ranks, lo=0.0, hi=1.0):
    """Refinement rounds (extra p-plane exchanges) the distributed mass
    inverse needs for this partition; -1: refused (pure host, no GPU)."""
    r = ctypes.c_int(0)
    m = mesh_desc(dim, fe_degree, n_subdivisions, lo, hi, n_ranks)
    check(load().gdm_mass_spike_rounds(ctypes.byref(m), ctypes.byref(r)), "gdm_mass_spike_rounds")
    return r.value


def mesh_spike_rounds(m):
    """mass_spike_rounds for an existing gdm_mesh_desc (an operator's .mesh)."""
    r = ctypes.c_int(0)
    check(load().gdm_mass_spike_rounds(ctypes.byref(m), ctypes.byref(r)), "gdm_mass_spike_rounds")
    return r.value


def mass_spike_eps(dim, fe_degree, n_subdivisions, n_ranks, lo=0.0, hi=1.0):
    """Largest coupling the distributed mass inverse's truncated interface
    systems drop (pure host, no GPU); the solve needs <= 1e-15."""
    e = ctypes.c_double(0.0)
    m = mesh_desc(dim, fe_degree, n_subdivisions, lo, hi, n_ranks)
    check(load().gdm_mass_spike_eps(ctypes.byref(m), ctypes.byref(e)), "gdm_mass_spike_eps")
    return e.value
