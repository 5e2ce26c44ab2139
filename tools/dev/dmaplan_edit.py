s = open('gdm_kernels.hip').read()
anchor = "template <int P, int R, int NC, int NP, int BK, int CH>\n__device__ __forceinline__ void producer8("
new_fn = '''// Per-lane DMA offsets of this producer wave's row groups: they depend on the
// row group, the lane and the input box only, not on the plane, so they are
// computed once per workgroup (the plane loop only moves the buffer base).
template <int P, int R, int NC, int NP, int BK, int CH>
struct DmaPlan8 {
  using G = Geom8<P, R, NC, NP, BK>;
  using S = Dma7<P, R, NC, NP, BK, CH>;
  uint32_t voff[G::NPASS][S::NI_FULL];  // 0x80000000: outside the box (reads 0)
  uint32_t on;                          // bit ps * NI_FULL + i: lane takes part
};

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void dma_plan8(const StencilArgs &a, const Tile7 &t, DmaPlan8<P, R, NC, NP, BK, CH> &pl) {
  using G = Geom8<P, R, NC, NP, BK>;
  using S = Dma7<P, R, NC, NP, BK, CH>;
  pl.on = 0;
#pragma unroll
  for (int ps = 0; ps < G::NPASS; ++ps) {
    const int g = t.wv + ps * NP;
    const bool last = g == G::NG - 1;
    const int nch = (last ? S::ROWS_LAST : 4) * S::CPR;
#pragma unroll
    for (int i = 0; i < S::NI_FULL; ++i) {
      const int e = i * 64 + t.lane;
      const int rr = e / S::CPR, c = e - rr * S::CPR;
      const int gy = t.y0 - P + 4 * g + rr;
      const int gx2 = (t.x0 - G::XH) * 2 + c * S::DPC;  // dword column
      uint32_t voff = 0x80000000u;
      if (gy >= a.in_y0 && gy < a.in_y1 && gx2 >= 0 && gx2 < 2 * a.Nx)
        voff = (uint32_t)(((int64_t)(gy - a.in_y0) * a.Nx * 2 + gx2) * 4);
      pl.voff[ps][i] = voff;
      if (g < G::NG && e < nch) pl.on |= 1u << (ps * S::NI_FULL + i);
    }
  }
}

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void stage_plane8(const StencilArgs &a, const Tile7 &t, int zz, ldouble *ubuf,
                                             const DmaPlan8<P, R, NC, NP, BK, CH> &pl) {
  using G = Geom8<P, R, NC, NP, BK>;
  using S = Dma7<P, R, NC, NP, BK, CH>;
  const int ny_in = a.in_y1 - a.in_y0;
  const double *plane = a.src + (int64_t)(zz - a.in_z0) * ny_in * a.Nx;
  const int nbytes = (int)((int64_t)ny_in * a.Nx * 8);
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)plane, 0, nbytes, 0x00020000);
#pragma unroll
  for (int ps = 0; ps < G::NPASS; ++ps) {
    const int g = t.wv + ps * NP;
    if (g >= G::NG) break;
    auto *gbase = (__attribute__((address_space(3))) char *)(ubuf + g * 4 * G::RL);
    const int ni = g == G::NG - 1 ? S::NI_LAST : S::NI_FULL;
#pragma unroll
    for (int i = 0; i < S::NI_FULL; ++i) {
      if (i < ni && ((pl.on >> (ps * S::NI_FULL + i)) & 1u)) {
        auto *dst = (__attribute__((address_space(3))) void *)(gbase + i * 64 * CH);
        if constexpr (CH == 16)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 16, pl.voff[ps][i], 0, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 4, pl.voff[ps][i], 0, 0, 0);
      }
    }
  }
}

'''
assert anchor in s
s = s.replace(anchor, new_fn + anchor)
old = """  const int n = t.ze - t.zs;
#pragma unroll
  for (int k = 0; k < NS; ++k)
    if (k < n) stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + k, u[k]);"""
new = """  const int n = t.ze - t.zs;
  DmaPlan8<P, R, NC, NP, BK, CH> plan;
  dma_plan8<P, R, NC, NP, BK, CH>(a, t, plan);
#pragma unroll
  for (int k = 0; k < NS; ++k)
    if (k < n) stage_plane8<P, R, NC, NP, BK, CH>(a, t, t.zs + k, u[k], plan);"""
assert old in s
s = s.replace(old, new)
old = """    if (i + NS < n && !GDM_DBG(a, 8)) stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + i + NS, u[slot]);"""
new = """    if (i + NS < n && !GDM_DBG(a, 8)) stage_plane8<P, R, NC, NP, BK, CH>(a, t, t.zs + i + NS, u[slot], plan);"""
assert old in s
s = s.replace(old, new)
open('gdm_kernels.hip', 'w').write(s)
print("ok")
