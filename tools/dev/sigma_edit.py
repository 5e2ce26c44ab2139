R = '/root/repo/dealii-galerkin-difference-methods_amd/csrc/'
s = open(R + 'gdm_kernels.hip').read()
old = """    lcdouble2 *vp = (lcdouble2 *)(t.ab0 + G::ab(row0, t.lane));
    dpair v[NR];"""
new = """    lcdouble2 *vp = (lcdouble2 *)(t.ab0 + G::ab(row0, t.lane));
    dpair v[NR];
#ifdef GDM_SIGMA
    // E = m * B + sy (b * A): compile-time b, one runtime scalar (frees the
    // SGPRs of the runtime band cy)
    double Gs[R];
#pragma unroll
    for (int j = 0; j < R; ++j) Gs[j] = 0.0;
#endif"""
assert old in s; s = s.replace(old, new)
old = """          D[j] = fma(IR::m[k], v[s].x, D[j]);
          E[j] = fma(IR::m[k], v[s].y, fma(a.cy[k], v[s].x, E[j]));
        }
      }
    }
  } else {"""
new = """          D[j] = fma(IR::m[k], v[s].x, D[j]);
#ifdef GDM_SIGMA
          E[j] = fma(IR::m[k], v[s].y, E[j]);
          if constexpr (BK == 1) {
            if (k != P) Gs[j] = fma(IR::c[k], v[s].x, Gs[j]);
          } else {
            Gs[j] = fma(IR::l[k], v[s].x, Gs[j]);
          }
#else
          E[j] = fma(IR::m[k], v[s].y, fma(a.cy[k], v[s].x, E[j]));
#endif
        }
      }
    }
#ifdef GDM_SIGMA
#pragma unroll
    for (int j = 0; j < R; ++j) E[j] = fma(a.sy, Gs[j], E[j]);
#endif
  } else {"""
assert old in s; s = s.replace(old, new)
open(R + 'gdm_kernels.hip', 'w').write(s)
h = open(R + 'gdm_kernels.h').read()
old = "  double dint;\n"
assert old in h
h = h.replace(old, "  double dint;\n  double sy;  // v8: h_x beta_y h_z (cy = sy * bhat), used with -DGDM_SIGMA\n")
open(R + 'gdm_kernels.h', 'w').write(h)
c = open(R + 'gdm_capi.cpp').read()
old = "  double dint = 0, m_dint = 0;  // interior z scales of D (operator, mass)"
assert old in c
c = c.replace(old, old + "\n  double sy8 = 0;               // v8: cy8 = sy8 * bhat")
old = "    op->dint = beta[2] * h[0] * h[1];"
assert old in c
c = c.replace(old, old + "\n    op->sy8 = h[0] * beta[1] * h[2];")
old = "    a.dint = op->dint;\n    a.sx = op->sx8;"
assert old in c
c = c.replace(old, "    a.dint = op->dint;\n    a.sy = op->sy8;\n    a.sx = op->sx8;")
open(R + 'gdm_capi.cpp', 'w').write(c)
print("ok")
