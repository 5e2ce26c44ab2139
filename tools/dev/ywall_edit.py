s = open('gdm_kernels.hip').read()
old = """  static constexpr int OFF_AB = NSLOT * USZ;
  static constexpr int OFF_ZT = OFF_AB + ABSZ;
  static constexpr int OFF_YC = OFF_ZT + ZTSZ;
  static constexpr int OFF_CORR = OFF_YC + YCSZ;
  static constexpr size_t lds_bytes() { return sizeof(double) * (size_t)(OFF_CORR + CORRSZ); }
};"""
new = """  static constexpr int YWSZ = (P + 1) * TX * NAB;  // y-wall corrections of one plane
  static constexpr int OFF_AB = NSLOT * USZ;
  static constexpr int OFF_ZT = OFF_AB + ABSZ;
  static constexpr int OFF_YC = OFF_ZT + ZTSZ;
  static constexpr int OFF_CORR = OFF_YC + YCSZ;
  static constexpr int OFF_YW = OFF_CORR + CORRSZ;
  static constexpr size_t lds_bytes() { return sizeof(double) * (size_t)(OFF_YW + YWSZ); }
};"""
assert old in s
s = s.replace(old, new)
old = """  static constexpr int NSLOT = sizeof(double) * (size_t)(3 * USZ + ABSZ + ZTSZ + YCSZ + CORRSZ) <= LDS_CAP ? 3 : 2;"""
assert old in s
s = s.replace(old, """  static constexpr int NSLOT =
      sizeof(double) * (size_t)(3 * USZ + ABSZ + ZTSZ + YCSZ + CORRSZ + (P + 1) * TX * NAB) <= LDS_CAP ? 3 : 2;""")
old = """template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void producer8(const StencilArgs &a, const Tile7 &t) {"""
new = """// first / end wall row of this tile's y-wall block (tile rows [y0, y0 + TY));
// begin = -1: no wall row in the tile
template <int P, int TY>
__device__ __forceinline__ int ywall_begin(const StencilArgs &a, int y0) {
  if (y0 <= P) return y0;                                          // bottom wall rows [0, p]
  if (y0 + TY - 1 >= a.Ny - P - 1) return max(y0, a.Ny - P - 1);  // top wall rows
  return -1;
}
template <int P, int TY>
__device__ __forceinline__ int ywall_end(const StencilArgs &a, int y0) {
  if (y0 <= P) return min(y0 + TY, P + 1);
  return min(y0 + TY, a.Ny);
}

// y-wall corrections of plane AB (edge tiles only, between L_i and M_i): for
// the wall rows y of this tile dD(y) = sum_s c1(y, s) A(s) and
// dE(y) = sum_s c1 B(s) + c3 A(s) with the (wall - Toeplitz) column tables;
// one row per producer wave, lane = x
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void ywall8(const StencilArgs &a, const Tile7 &t) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int W = G::W, TX = G::TX;
  const int yb = ywall_begin<P, G::TY>(a, t.y0), ye = ywall_end<P, G::TY>(a, t.y0);
  for (int y = yb + t.wv; y < ye; y += NP) {
    const int wi = y - yb;
    double dD = 0.0, dE = 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int rs = y + 2 * P - k - t.y0;  // tile row of input s = y + p - k
      const dpair c = ((lcdouble2 *)t.yc)[rs * W + k];
      if constexpr (BK != 0) {
        const dpair v = ((lcdouble2 *)t.ab0)[rs * TX + t.lane];
        dD = fma(c.x, v.x, dD);
        dE = fma(c.x, v.y, fma(c.y, v.x, dE));
      } else {
        dD = fma(c.x, t.ab0[rs * TX + t.lane], dD);
      }
    }
    if constexpr (BK != 0)
      ((ldouble2 *)t.yw)[wi * TX + t.lane] = dpair{dD, dE};
    else
      t.yw[wi * TX + t.lane] = dD;
  }
}

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void producer8(const StencilArgs &a, const Tile7 &t) {"""
assert old in s
s = s.replace(old, new)
old = """    GDM_LDS_BARRIER();  // L_i: AB(i) loaded
    if (i + NS < n && !GDM_DBG(a, 8)) stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + i + NS, u[slot]);"""
new = """    GDM_LDS_BARRIER();  // L_i: AB(i) loaded
    if (t.yedge) {
      ywall8<P, R, NC, NP, BK>(a, t);
      GDM_LDS_BARRIER();  // M_i: y-wall corrections of plane i ready
    }
    if (i + NS < n && !GDM_DBG(a, 8)) stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + i + NS, u[slot]);"""
assert old in s
s = s.replace(old, new)
i = s.index("template <int P, int R, int NC, int NP, int BK, int PF, bool YW>\n__device__ __forceinline__ void ysweep8(")
j = s.index("template <int JP, int P, int R, int NC, int NP, int BK, int PF, bool WALL, bool YW>")
seg = s[i:j]
out = []
pos = 0
while True:
    k = seg.find("    if constexpr (YW) {", pos)
    if k < 0:
        out.append(seg[pos:])
        break
    st = seg.index("{", k)
    d = 0
    m = st
    while True:
        if seg[m] == '{':
            d += 1
        elif seg[m] == '}':
            d -= 1
            if d == 0:
                break
        m += 1
    out.append(seg[pos:k])
    pos = m + 2
seg = "".join(out)
seg = seg.replace("template <int P, int R, int NC, int NP, int BK, int PF, bool YW>\n__device__ __forceinline__ void ysweep8(",
                  "template <int P, int R, int NC, int NP, int BK, int PF>\n__device__ __forceinline__ void ysweep8(")
s = s[:i] + seg + s[j:]
old = """      ysweep8<P, R, NC, NP, BK, PF, YW>(a, t, D, E);
    }"""
new = """      ysweep8<P, R, NC, NP, BK, PF>(a, t, D, E);
    }
    if constexpr (YW) {
      GDM_LDS_BARRIER();  // M_i
      const int yb = ywall_begin<P, G::TY>(a, t.y0), ye = ywall_end<P, G::TY>(a, t.y0);
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int y = ybase + j;
        if (y >= yb && y < ye) {
          if constexpr (BK != 0) {
            const dpair c = ((lcdouble2 *)t.yw)[(y - yb) * G::TX + t.lane];
            D[j] += c.x;
            E[j] += c.y;
          } else {
            D[j] += t.yw[(y - yb) * G::TX + t.lane];
          }
        }
      }
    }"""
assert old in s
s = s.replace(old, new)
old = """#ifdef GDM_EXP_NOYFIX
  if (false)
#else
  if (ybase < P + 1 || ybase + R - 1 + P + 2 > a.Ny)
#endif
    consumer8_loop<P, R, NC, NP, BK, PF, ZI, true>(a, t, ybase, full);"""
new = """  // edge tiles (rows next to a y wall) wait for the producers' y-wall
  // corrections every plane: their own copy of the loop keeps that out of the
  // hot block of the other tiles
  if (t.yedge)
    consumer8_loop<P, R, NC, NP, BK, PF, ZI, true>(a, t, ybase, full);"""
assert old in s
s = s.replace(old, new)
s = s.replace("""  // waves with a row next to a y wall (non-Toeplitz row of M_y, B_y) run their
  // own copy of the plane loop with the rolled wall corrections: a branch
  // inside the hot unrolled block costs the other waves their schedule
""", "")
old = """struct Tile7 {
  ldouble *u0, *ab0, *zt, *yc, *corr;"""
new = """struct Tile7 {
  ldouble *u0, *ab0, *zt, *yc, *corr, *yw;
  bool yedge;  // v8: the tile has rows next to a y wall"""
assert old in s
s = s.replace(old, new)
old = """  t.corr = lds + G::OFF_CORR;
  t.lane = threadIdx.x & 63;
  t.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.x0 = blockIdx.x * G::TX;
  t.y0 = a.out_y0 + blockIdx.y * G::TY;
  {
    const int r = (int)blockIdx.z < a.nchunk0 ? 0 : 1;"""
new = """  t.corr = lds + G::OFF_CORR;
  t.yw = lds + G::OFF_YW;
  t.lane = threadIdx.x & 63;
  t.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.x0 = blockIdx.x * G::TX;
  t.y0 = a.out_y0 + blockIdx.y * G::TY;
  t.yedge = ywall_begin<P, G::TY>(a, t.y0) >= 0;
  {
    const int r = (int)blockIdx.z < a.nchunk0 ? 0 : 1;"""
assert old in s
s = s.replace(old, new)
old = """  // tiles with rows next to a y wall: (wall - Toeplitz) column corrections
  if (t.y0 < P + 1 || t.y0 + G::TY - 1 + P + 2 > a.Ny)"""
new = """  // tiles with rows next to a y wall: (wall - Toeplitz) column corrections
  if (t.yedge)"""
assert old in s
s = s.replace(old, new)
s = s.replace('''// y-sweep of the consumer's R rows from the (A, B) plane: D' and E with the
// compile-time interior bands, rows read PF ahead of their use.  Waves with a
// row next to a y wall then add (wall row - Toeplitz) corrections from the
// tile's LDS column table in a rolled loop (compact code: the hot unrolled
// block stays small).''', '''// y-sweep of the consumer's R rows from the (A, B) plane: D' and E with the
// compile-time interior bands, rows read PF ahead of their use (wall rows get
// their corrections from the producers' ywall8, see cplane8).''')
open('gdm_kernels.hip', 'w').write(s)
print("ok")
