s = open('gdm_kernels.hip').read()
i = s.index("template <int P, int R, int NC, int NP, int BK>\n__device__ __forceinline__ void xsweep8(")
j = s.index("// Wall columns of row group g (first / last x tiles only)")
s = s[:i] + '''template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xsweep8(const StencilArgs &a, const Tile7 &t, lcdouble *us, int g, dpair (&V)[4]) {
  // V[j] = (A_j, B_j) for x = 4 q + j (the pair the AB plane stores, so no
  // register moves before the b128 stores); mass: V[0] = (A_0, A_1), V[1] = (A_2, A_3)
  using G = Geom8<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W, RL = G::RL;
  const int rr = t.lane >> 4, q = t.lane & 15;
  const int r = 4 * g + rr;
  lcdouble2 *wp = (lcdouble2 *)(us + r * RL + 4 * q);
  double w[G::NWIN];
#pragma unroll
  for (int i = 0; i < G::NWIN / 2; ++i) {
    const dpair v = wp[i];
    w[2 * i] = v.x;
    w[2 * i + 1] = v.y;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) V[j] = dpair{0.0, 0.0};
  if (a.x_toep) {
#pragma unroll
    for (int k = 0; k < W; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (BK == 0) {
          if (j % 2 == 0)
            V[j / 2].x = fma(IR::m[k], w[j + k + 1], V[j / 2].x);
          else
            V[j / 2].y = fma(IR::m[k], w[j + k + 1], V[j / 2].y);
        } else {
          V[j].x = fma(IR::m[k], w[j + k + 1], V[j].x);
          if constexpr (BK == 1) V[j].y = fma(IR::c[k], w[j + k + 1], V[j].y);
          if constexpr (BK == 2) V[j].y = fma(IR::l[k], w[j + k + 1], V[j].y);
        }
      }
  }
  if constexpr (BK != 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) V[j].y *= a.sx;
  }
}

''' + s[j:]
i = s.index("template <int P, int R, int NC, int NP, int BK>\n__device__ __forceinline__ void write_ab8(")
j = s.index("// first / end wall row of this tile's y-wall block")
s = s[:i] + '''template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void write_ab8(const Tile7 &t, int g, const dpair (&V)[4]) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int TX = G::TX;
  const int rr = t.lane >> 4, q = t.lane & 15;
  const int r = 4 * g + rr;
  if (r < G::UR) {
    if constexpr (BK != 0) {
      ldouble2 *p = (ldouble2 *)(t.ab0 + G::ab(r, 4 * q));  // 4 q .. 4 q + 3 share one 8-x block
#pragma unroll
      for (int j = 0; j < 4; ++j) p[j] = V[j];
    } else {
      ldouble2 *p = (ldouble2 *)(t.ab0 + r * TX + 4 * q);
      p[0] = V[0];
      p[1] = V[1];
    }
  }
}

''' + s[j:]
old_calls = [
 ("    double AR2[4], BR2[4];\n    if (!GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], t.wv, AR, BR);",
  "    dpair V2[4];\n    if (!GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], t.wv, V1);"),
 ("    if (two && !GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], t.wv + NP, AR2, BR2);",
  "    if (two && !GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], t.wv + NP, V2);"),
 ("    write_ab8<P, R, NC, NP, BK>(t, t.wv, AR, BR);\n    if (two) write_ab8<P, R, NC, NP, BK>(t, t.wv + NP, AR2, BR2);",
  "    write_ab8<P, R, NC, NP, BK>(t, t.wv, V1);\n    if (two) write_ab8<P, R, NC, NP, BK>(t, t.wv + NP, V2);"),
 ("        if (!GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], g, AR, BR);\n        write_ab8<P, R, NC, NP, BK>(t, g, AR, BR);",
  "        if (!GDM_DBG(a, 4)) xsweep8<P, R, NC, NP, BK>(a, t, u[slot], g, V1);\n        write_ab8<P, R, NC, NP, BK>(t, g, V1);"),
 ("  double AR[4], BR[4];\n  int slot = 0;", "  dpair V1[4];\n  int slot = 0;"),
]
for o, n in old_calls:
    assert o in s, o
    s = s.replace(o, n)
open('gdm_kernels.hip', 'w').write(s)
print("ok")
