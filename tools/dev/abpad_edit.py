s = open('gdm_kernels.hip').read()
old = "  static constexpr int ABSZ = UR * TX * NAB;"
new = """  // (A, B) pairs: row stride 2 TX + 2 TX / 8 doubles with one pair of padding
  // after every 8 x -- the producers' 4-pairs-per-lane ds_write_b128 stores
  // then hit distinct banks; consumers read one pair per lane as before
  static constexpr int ABRS = NAB == 2 ? 2 * TX + 2 * (TX / 8) : TX;
  static constexpr int ABSZ = UR * ABRS;
  static __device__ __forceinline__ int ab(int r, int x) { return NAB == 2 ? r * ABRS + 2 * x + 2 * (x >> 3) : r * TX + x; }"""
assert old in s; s = s.replace(old, new)
old = "    xw.o[it] = BK != 0 ? (r * TX + lx) * 2 + comp : r * TX + lx;"
if old not in s:
    old = "      xw.o[it] = BK != 0 ? (r * TX + lx) * 2 + comp : r * TX + lx;"
assert old in s
s = s.replace(old, old.replace("BK != 0 ? (r * TX + lx) * 2 + comp : r * TX + lx", "G::ab(r, lx) + (BK != 0 ? comp : 0)"))
old = "      ldouble2 *p = (ldouble2 *)(t.ab0 + (r * TX + 4 * q) * 2);"
assert old in s; s = s.replace(old, "      ldouble2 *p = (ldouble2 *)(t.ab0 + G::ab(r, 4 * q));  // 4 q .. 4 q + 3 share one 8-x block")
old = "        const dpair v = ((lcdouble2 *)t.ab0)[rs * TX + t.lane];"
assert old in s; s = s.replace(old, "        const dpair v = *(lcdouble2 *)(t.ab0 + G::ab(rs, t.lane));")
old = "    lcdouble2 *vp = (lcdouble2 *)t.ab0 + row0 * TX + t.lane;"
assert old in s; s = s.replace(old, "    lcdouble2 *vp = (lcdouble2 *)(t.ab0 + G::ab(row0, t.lane));")
# ysweep8 BK != 0 reads use vp[s * TX] -> vp[s * (ABRS / 2)]
i = s.index("__device__ __forceinline__ void ysweep8(")
j = s.index("template <int JP, int P, int R, int NC, int NP, int BK, int PF, bool WALL, bool YW>")
seg = s[i:j]
k = seg.index("  if constexpr (BK != 0) {")
k2 = seg.index("  } else {\n    const volatile lcdouble *vp")
part = seg[k:k2]
part = part.replace("vp[s * TX]", "vp[s * (G::ABRS / 2)]").replace("vp[(s + PF) * TX]", "vp[(s + PF) * (G::ABRS / 2)]")
seg = seg[:k] + part + seg[k2:]
s = s[:i] + seg + s[j:]
open('gdm_kernels.hip', 'w').write(s)
print("ok")
