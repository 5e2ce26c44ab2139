s = open('gdm_kernels.hip').read()
# 1. xwall8 -> compute (before F) + add (after the AB write)
i = s.index("// Wall columns of row group g (first / last x tiles only)")
j = s.index("// store row group g's (A, B) into the interleaved plane buffer")
s = s[:i] + '''// Wall columns of row group g (first / last x tiles only): the
// (wall row - Toeplitz row) corrections of M_x and B_x, one (row, column,
// component) item per lane so the work is spread over the wave instead of
// serialised per lane.  xwall8_calc runs before F (overlapping the consumers'
// y-sweep); xwall8_add adds the values into AB after write_ab8 of the group
// (same wave: LDS operations stay in program order).
template <int P, int BK>
struct XWall {
  static constexpr int NCOMP = BK == 0 ? 1 : 2;
  static constexpr int NI = (4 * (P + 1) * NCOMP + 63) / 64;  // items per lane (one x wall per tile)
  double v[NI];
  int o[NI];  // AB offset, -1: none
};

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xwall8_calc(const StencilArgs &a, const Tile7 &t, lcdouble *us, int g,
                                            XWall<P, BK> &xw) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int W = G::W, RL = G::RL, TX = G::TX, NCOMP = XWall<P, BK>::NCOMP;
  const int nitems = 4 * t.ncw * NCOMP;
#pragma unroll
  for (int it = 0; it < XWall<P, BK>::NI; ++it) {
    const int e = t.lane + 64 * it;
    xw.o[it] = -1;
    xw.v[it] = 0.0;
    const int comp = e % NCOMP, rest = e / NCOMP;
    const int idx = rest % max(t.ncw, 1), rr = rest / max(t.ncw, 1);
    const int r = 4 * g + rr;
    if (e < nitems && r < G::UR) {
      const int x = idx < t.nl ? t.x0 + idx : t.rs + (idx - t.nl);
      const int cs = x < a.x_corr_left ? x : (P + 1) + (x - (a.Nx - a.x_corr_right));
      const int lx = x - t.x0;
      lcdouble *ur = us + r * RL + lx + 1;  // tap k of column x
      lcdouble *cm = t.corr + cs * 2 * W + comp * W;
      double d = 0.0;
#pragma unroll
      for (int k = 0; k < W; ++k) d = fma(cm[k], ur[k], d);
      xw.v[it] = d;
      xw.o[it] = BK != 0 ? (r * TX + lx) * 2 + comp : r * TX + lx;
    }
  }
}

template <int P, int BK>
__device__ __forceinline__ void xwall8_add(const Tile7 &t, const XWall<P, BK> &xw) {
#pragma unroll
  for (int it = 0; it < XWall<P, BK>::NI; ++it)
    if (xw.o[it] >= 0) t.ab0[xw.o[it]] += xw.v[it];
}

''' + s[j:]
# 2. producer loop
i = s.index("    // the first two row groups into registers before F (overlapping the")
j = s.index("  GDM_LDS_BARRIER();  // F_n\n}")
new_loop = '''    // the first two row groups into registers before F (overlapping the
    // consumers' y-sweep of plane i - 1), any further ones straight into AB
    double AR2[4], BR2[4];
    if (!GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], t.wv, AR, BR);
    const bool two = G::NPASS > 1 && t.wv + NP < G::NG;
    if (two && !GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], t.wv + NP, AR2, BR2);
    XWall<P, BK> xw0, xw1;
    if (t.ncw > 0) {
      xwall8_calc<P, R, NC, NP, BK>(a, t, u[slot], t.wv, xw0);
      if (two) xwall8_calc<P, R, NC, NP, BK>(a, t, u[slot], t.wv + NP, xw1);
    }
    if (t.yedge && i > 0) {
      ywall8<P, R, NC, NP, BK>(a, t);  // corrections of plane i - 1 (AB still holds it)
      GDM_LDS_BARRIER();               // M_i-1
    }
    GDM_LDS_BARRIER();  // F_i
    write_ab8<P, R, NC, NP, BK>(t, t.wv, AR, BR);
    if (two) write_ab8<P, R, NC, NP, BK>(t, t.wv + NP, AR2, BR2);
    if (t.ncw > 0) {
      xwall8_add<P, BK>(t, xw0);
      if (two) xwall8_add<P, BK>(t, xw1);
    }
#pragma unroll
    for (int ps = 2; ps < G::NPASS; ++ps) {
      const int g = t.wv + ps * NP;
      if (g < G::NG) {
        if (!GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], g, AR, BR);
        write_ab8<P, R, NC, NP, BK>(t, g, AR, BR);
        if (t.ncw > 0) {
          xwall8_calc<P, R, NC, NP, BK>(a, t, u[slot], g, xw0);
          xwall8_add<P, BK>(t, xw0);
        }
      }
    }
    GDM_LDS_BARRIER();  // L_i: AB(i) loaded
    if (i + NS < n && !GDM_DBG(a, 8)) stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + i + NS, u[slot]);
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  if (t.yedge && n > 0) {
    ywall8<P, R, NC, NP, BK>(a, t);
    GDM_LDS_BARRIER();  // M_n-1
  }
'''
s = s[:i] + new_loop + s[j:]
open('gdm_kernels.hip', 'w').write(s)
print("ok")
