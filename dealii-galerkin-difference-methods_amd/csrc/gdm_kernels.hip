// gdm_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the GDM operator
// engine.  See DESIGN.md for the derivation; in short, on an uncut uniform
// Cartesian mesh every hot-path operator of the reference is a sum of
// Kronecker products of 1D band matrices of half-bandwidth p:
//
//   advection (advection/stiffness.h:345-532, alpha = 0, outflow traces folded
//              into B_d):            K = B_x M_y M_z + M_x B_y M_z + M_x M_y B_z
//   wave      (wave/stiffness.h:171-181):                  same with B_d = -L_d
//   mass      (advection/mass.h:144-156):                  M = M_x M_y M_z
//
// The fused kernel marches each (x, y) tile along z.  Per input plane:
//   1. the (TY + 2p) x (64 + 2p) plane tile is staged in LDS,
//   2. x-sweep  A = M_x u, Bv = B_x u          (LDS -> LDS, lane = x),
//   3. y-sweep  D = M_y A, E = M_y Bv + B_y A  (LDS -> registers, R rows/lane),
//   4. z-scatter: out[z'] += M_z(z', z) E + B_z(z', z) D for the 2p + 1 planes
//      z' around z, kept in a register ring that retires one finished output
//      plane per input plane (coalesced 512-B row stores).
// y- and z-coefficients are wave-uniform (scalar loads); x-coefficients are
// per-lane registers (they differ only near the x faces).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <cstdlib>

#include "gdm_coeffs.h"
#include "gdm_kernels.h"

#ifndef GDM_R5
#define GDM_R5 4
#define GDM_NC5 8
#define GDM_NP5 8
#endif
#ifndef GDM_PF5
#define GDM_PF5 3
#endif
#ifndef GDM_R7
#define GDM_R7 2
#define GDM_NC7 8
#define GDM_NP7 8
#endif
#ifndef GDM_PF7
#define GDM_PF7 3
#endif
// cache policy of the v8 stencil's plane DMA (buffer aux bits on gfx950: 2 =
// nt) and its output stores (1 = non-temporal).  A/B at C3 on the MI355X
// (profiles/r3x, 3 repetitions each): cached 0.840-0.849 ms, non-temporal
// stores 0.822-0.837 ms (the default), non-temporal stores and DMA 0.835-0.845
#ifndef GDM_STENCIL_LD_CPOL
#define GDM_STENCIL_LD_CPOL 0
#endif
#ifndef GDM_STENCIL_ST_NT
#define GDM_STENCIL_ST_NT 1
#endif
#if GDM_STENCIL_ST_NT
#define GDM_STENCIL_STORE(p, v) __builtin_nontemporal_store((v), (p))
#else
#define GDM_STENCIL_STORE(p, v) (*(p) = (v))
#endif

namespace gdmk {



#define GDM_WAIT_VMCNT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")
#define GDM_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Coefficient tables are read-only for the whole launch and indexed by
// wave-uniform positions: read them through the constant address space so
// they become scalar (s_load) loads instead of vector loads.
typedef __attribute__((address_space(4))) const double cdouble;
__device__ __forceinline__ cdouble *cptr(const double *p) { return (cdouble *)(p); }

// ===========================================================================
// Fused Kronecker stencil, v7: producer / consumer waves.
//
// A workgroup owns a 64 x TY column of (x, y) and marches it along z.
//   * NP producer waves stage the (TY + 2p) x (64 + 2p) input plane tile into
//     LDS by LDS-DMA (buffer_load ... lds, out-of-box rows/columns read as 0)
//     and run the x-sweep, 4 consecutive x per lane from a 16-B aligned
//     register window (ds_read_b128).  Each producer wave DMAs exactly the
//     row groups it sweeps, so the u ring needs no workgroup barrier: a
//     counted vmcnt per wave keeps one plane of DMA in flight.
//   * NC consumer waves (lane = x, R rows each) run the y-sweep from the A/B
//     planes and scatter into a register ring of 2p+1 output planes, retiring
//     one finished plane per input plane with coalesced row stores.
// The two roles hand over one A/B plane per barrier (double-buffered), so a
// wave holds either the x-sweep temporaries or the ring, never both.
// ===========================================================================
template <int P, int R, int NC, int NP, int BK>
struct Geom7 {
  static constexpr int W = 2 * P + 1;
  static constexpr int TX = 64;
  static constexpr int TY = R * NC;
  static constexpr int UR = TY + 2 * P;
  static constexpr int XH = P + 1;  // even: keeps the x windows 16-B aligned
  static constexpr int RL0 = TX + 2 * XH;
  // row pitch = 2 mod 4 doubles: the two rows a ds_read_b128 lane group spans
  // land on disjoint bank halves
  static constexpr int RL = (RL0 % 4 == 2) ? RL0 : RL0 + 2;
  static constexpr int NW = NP + NC;
  static constexpr int NT = 64 * NW;
  static constexpr int NG = (UR + 3) / 4;  // producer row groups (4 rows = one wave pass)
  static constexpr int NPASS = (NG + NP - 1) / NP;
  static constexpr int USZ = NG * 4 * RL;
  static constexpr int NAB = BK == 0 ? 1 : 2;
  static constexpr int ABSZ = NAB * UR * TX;
  static constexpr int NZR = 2 * W + 1;
  static constexpr int ZTSZ = NZR * W * 2;
  static constexpr int NCORR = 2 * (P + 1);
  static constexpr int CORRSZ = NCORR * 2 * W;
  static constexpr int YCSZ = UR * W * 2;  // y-wall columns of the tile rows, (M_y/h_y, h_x B_y) pairs
  static constexpr int NWIN = 2 * P + 6;
  static constexpr int OFF_AB = 2 * USZ;
  static constexpr int OFF_ZT = OFF_AB + 2 * ABSZ;
  static constexpr int OFF_YC = OFF_ZT + ZTSZ;
  static constexpr int OFF_CORR = OFF_YC + YCSZ;
  static constexpr size_t lds_bytes() { return sizeof(double) * (size_t)(OFF_CORR + CORRSZ); }
};

template <int P, int R, int NC, int NP, int BK, int CH>
struct Dma7 {
  using G = Geom7<P, R, NC, NP, BK>;
  static constexpr int DPC = CH / 4;             // dwords per lane
  static constexpr int CPR = G::RL * 2 / DPC;    // lane chunks per LDS row
  static constexpr int ROWS_LAST = G::UR - 4 * (G::NG - 1);
  static constexpr int NI_FULL = (4 * CPR + 63) / 64;
  static constexpr int NI_LAST = (ROWS_LAST * CPR + 63) / 64;
  static constexpr int ni(int g) { return g == G::NG - 1 ? NI_LAST : NI_FULL; }
  // DMA instructions producer wave w issues per plane
  static constexpr int nd(int w) {
    int s = 0;
    for (int ps = 0; ps < G::NPASS; ++ps)
      if (w + ps * NP < G::NG) s += ni(w + ps * NP);
    return s;
  }
};

typedef __attribute__((address_space(3))) double ldouble;
typedef __attribute__((address_space(3))) unsigned int lu32;
typedef double dpair __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) dpair ldouble2;
typedef __attribute__((address_space(3))) const double lcdouble;
typedef __attribute__((address_space(3))) const dpair lcdouble2;
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
// compiler-only fence: no memory access and no instruction crosses it, so the
// scheduler cannot hoist all LDS reads of a sweep to its top (their registers
// would overlap the accumulator ring)
#define GDM_FENCE()                      \
  do {                                   \
    asm volatile("" ::: "memory");       \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)

struct Tile7 {
  ldouble *u0, *ab0, *zt, *yc, *corr, *yw;
  lu32 *sync;  // v8: hand-off counters
  int cw;      // v8: this wave's output row block (rows cw R .. cw R + R - 1 of the tile)
  bool yedge;  // v8: the tile has rows next to a y wall
  int ry0;     // v8 y-wall tiles: first tile row of the column table (yb - y0)
  int lane, wv, x0, y0, zc0, zc1, zs, ze, zend;
  unsigned ooff;  // v8 consumers: byte offset of the lane's first output row in an output plane
  int nyw;        // v8 y-wall tiles: producer waves that compute wall-row corrections
  // x wall columns inside this tile: nl from the left wall, nr from column rs on
  int nl, rs, ncw;
};

// wait until at most nd(wv) DMA instructions of this producer wave are in flight
template <int I, int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void wait_dma_plane(int wv) {
  if constexpr (I < NP) {
    if (wv == I) {
      GDM_WAIT_VMCNT((Dma7<P, R, NC, NP, BK, CH>::nd(I)));
      return;
    }
    wait_dma_plane<I + 1, P, R, NC, NP, BK, CH>(wv);
  }
}

// LDS-DMA of row group g of plane zz into u slot ubuf
template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void stage_group7(const StencilArgs &a, const Tile7 &t, int zz, int g, ldouble *ubuf) {
  using G = Geom7<P, R, NC, NP, BK>;
  using S = Dma7<P, R, NC, NP, BK, CH>;
  const int ny_in = a.in_y1 - a.in_y0;
  const double *plane = a.src + (int64_t)(zz - a.in_z0) * ny_in * a.Nx;
  const int nbytes = (int)((int64_t)ny_in * a.Nx * 8);
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)plane, 0, nbytes, 0x00020000);
  const bool last = g == G::NG - 1;
  const int nch = (last ? S::ROWS_LAST : 4) * S::CPR;
  const int ni = last ? S::NI_LAST : S::NI_FULL;
  auto *gbase = (__attribute__((address_space(3))) char *)(ubuf + g * 4 * G::RL);
#pragma unroll
  for (int i = 0; i < S::NI_FULL; ++i) {
    if (i < ni) {
      const int e = i * 64 + t.lane;
      const int rr = e / S::CPR, c = e - rr * S::CPR;
      const int gy = t.y0 - P + 4 * g + rr;
      const int gx2 = (t.x0 - G::XH) * 2 + c * S::DPC;  // dword column
      uint32_t voff = 0x80000000u;                      // out of range -> zeros
      if (e < nch && gy >= a.in_y0 && gy < a.in_y1 && gx2 >= 0 && gx2 < 2 * a.Nx)
        voff = (uint32_t)(((int64_t)(gy - a.in_y0) * a.Nx * 2 + gx2) * 4);
      if (e < nch) {
        auto *dst = (__attribute__((address_space(3))) void *)(gbase + i * 64 * CH);
        if constexpr (CH == 16)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 16, voff, 0, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 4, voff, 0, 0, 0);
      }
    }
  }
}

// plane-invariant per-lane DMA byte offsets of this producer wave's row groups
// (the plane is selected by the buffer resource alone): computed once per
// tile instead of ~15 VALU + ~15 SALU per DMA instruction and plane;
// 0xffffffff = the lane issues nothing for that instruction
template <int P, int R, int NC, int NP, int BK, int CH>
struct DmaPre7 {
  uint32_t vo[Geom7<P, R, NC, NP, BK>::NPASS][Dma7<P, R, NC, NP, BK, CH>::NI_FULL];
};

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void stage_pre7(const StencilArgs &a, const Tile7 &t, DmaPre7<P, R, NC, NP, BK, CH> &d) {
  using G = Geom7<P, R, NC, NP, BK>;
  using S = Dma7<P, R, NC, NP, BK, CH>;
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
      const int gx2 = (t.x0 - G::XH) * 2 + c * S::DPC;
      uint32_t voff = 0x80000000u;  // out of range -> zeros
      if (gy >= a.in_y0 && gy < a.in_y1 && gx2 >= 0 && gx2 < 2 * a.Nx)
        voff = (uint32_t)(((int64_t)(gy - a.in_y0) * a.Nx * 2 + gx2) * 4);
      d.vo[ps][i] = (g < G::NG && e < nch) ? voff : 0xffffffffu;
    }
  }
}

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void stage_plane_pre7(const StencilArgs &a, const Tile7 &t, int zz, ldouble *ubuf,
                                                 const DmaPre7<P, R, NC, NP, BK, CH> &d) {
  using G = Geom7<P, R, NC, NP, BK>;
  using S = Dma7<P, R, NC, NP, BK, CH>;
  const int ny_in = a.in_y1 - a.in_y0;
  const double *plane = a.src + (int64_t)(zz - a.in_z0) * ny_in * a.Nx;
  const int nbytes = (int)((int64_t)ny_in * a.Nx * 8);
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)plane, 0, nbytes, 0x00020000);
#pragma unroll
  for (int ps = 0; ps < G::NPASS; ++ps) {
    const int g = t.wv + ps * NP;
    if (g < G::NG) {
      const int ni = g == G::NG - 1 ? S::NI_LAST : S::NI_FULL;  // wave-uniform: the count wait_dma_planes expects
      auto *gbase = (__attribute__((address_space(3))) char *)(ubuf + g * 4 * G::RL);
#pragma unroll
      for (int i = 0; i < S::NI_FULL; ++i) {
        if (i < ni && d.vo[ps][i] != 0xffffffffu) {
          auto *dst = (__attribute__((address_space(3))) void *)(gbase + i * 64 * CH);
          if constexpr (CH == 16)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 16, d.vo[ps][i], 0, 0, GDM_STENCIL_LD_CPOL);
          else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, dst, 4, d.vo[ps][i], 0, 0, GDM_STENCIL_LD_CPOL);
        }
      }
    }
  }
}

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void stage_plane7(const StencilArgs &a, const Tile7 &t, int zz, ldouble *ubuf) {
  using G = Geom7<P, R, NC, NP, BK>;
#pragma unroll
  for (int ps = 0; ps < G::NPASS; ++ps) {
    const int g = t.wv + ps * NP;
    if (g < G::NG) stage_group7<P, R, NC, NP, BK, CH>(a, t, zz, g, ubuf);
  }
}

// x-sweep of the row groups of this producer wave: A' = mhat*u, B* = sx bhat*u
// (+ wall-column corrections), 4 consecutive x per lane.
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xsweep7(const StencilArgs &a, const Tile7 &t, lcdouble *us, ldouble *ab) {
  using G = Geom7<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W, TX = G::TX, RL = G::RL;
  ldouble *as = ab, *bs = ab + G::UR * TX;
  const int rr = t.lane >> 4, q = t.lane & 15;
#pragma unroll
  for (int ps = 0; ps < G::NPASS; ++ps) {
    const int g = t.wv + ps * NP;
    if (g >= G::NG) break;
    const int r = 4 * g + rr;
    if (r < G::UR) {
      double A[4], B[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) A[j] = B[j] = 0.0;
      if (a.x_toep) {
        lcdouble2 *wp = (lcdouble2 *)(us + r * RL + 4 * q);
        double w[G::NWIN];
#pragma unroll
        for (int i = 0; i < G::NWIN / 2; ++i) {
          const dpair v = wp[i];
          w[2 * i] = v.x;
          w[2 * i + 1] = v.y;
        }
#pragma unroll
        for (int k = 0; k < W; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            A[j] = fma(IR::m[k], w[j + k + 1], A[j]);
            if constexpr (BK == 1) B[j] = fma(IR::c[k], w[j + k + 1], B[j]);
            if constexpr (BK == 2) B[j] = fma(IR::l[k], w[j + k + 1], B[j]);
          }
      }
      ldouble2 *ap = (ldouble2 *)(as + r * TX + 4 * q);
      ap[0] = dpair{A[0], A[1]};
      ap[1] = dpair{A[2], A[3]};
      if constexpr (BK != 0) {
        ldouble2 *bp = (ldouble2 *)(bs + r * TX + 4 * q);
        bp[0] = dpair{a.sx * B[0], a.sx * B[1]};
        bp[1] = dpair{a.sx * B[2], a.sx * B[3]};
      }
    }
    // wall columns of this tile: add the (row - Toeplitz) corrections
    if (t.ncw > 0) {
      const int nrow = min(4, G::UR - 4 * g);
      for (int e = t.lane; e < nrow * t.ncw; e += 64) {
        const int r2 = 4 * g + e / t.ncw, idx = e % t.ncw;
        const int x = idx < t.nl ? t.x0 + idx : t.rs + (idx - t.nl);
        const int cs = x < a.x_corr_left ? x : (P + 1) + (x - (a.Nx - a.x_corr_right));
        const int lx = x - t.x0;
        lcdouble *ur = us + r2 * RL + lx + 1;  // tap k of column x
        lcdouble *cm = t.corr + cs * 2 * W;
        double dA = 0.0, dB = 0.0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const double uv = ur[k];
          dA = fma(cm[k], uv, dA);
          if constexpr (BK != 0) dB = fma(cm[W + k], uv, dB);
        }
        as[r2 * TX + lx] += dA;
        if constexpr (BK != 0) bs[r2 * TX + lx] += dB;
      }
    }
  }
}

// y-sweep of the consumer's R rows: D' (and E) from A/B set `ab`
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void ysweep7(const StencilArgs &a, const Tile7 &t, bool ytoep, int ybase,
                                        lcdouble *ab, double (&D)[R], double (&E)[R]) {
  using G = Geom7<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W, TX = G::TX;
  // volatile: one ds_read_b64 per row (the compiler would pair rows into
  // ds_read2st64_b64, which runs at half the LDS rate)
  const volatile lcdouble *as = ab + ((t.wv - NP) * R) * TX + t.lane;
  const volatile lcdouble *bs = as + G::UR * TX;
#pragma unroll
  for (int j = 0; j < R; ++j) D[j] = E[j] = 0.0;
  if (ytoep) {
    // rows are read one pair ahead of their use
    constexpr int NR = R + 2 * P;
    double av[NR], bv[NR];
    av[0] = as[0];
    if constexpr (BK != 0) bv[0] = bs[0];
    if constexpr (NR > 1) {
      av[1] = as[TX];
      if constexpr (BK != 0) bv[1] = bs[TX];
    }
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      if (s % 2 == 0) {
        GDM_FENCE();
#pragma unroll
        for (int u = s + 2; u < s + 4 && u < NR; ++u) {
          av[u] = as[u * TX];
          if constexpr (BK != 0) bv[u] = bs[u * TX];
        }
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int k = s - j;  // row form: M(y_j, y_j - p + k)
        if (k >= 0 && k < W) {
          D[j] = fma(IR::m[k], av[s], D[j]);
          if constexpr (BK != 0) E[j] = fma(IR::m[k], bv[s], fma(a.cy[k], av[s], E[j]));
        }
      }
    }
  } else {
    // rows next to a y wall: column coefficients from the tile's LDS table
    // (broadcast reads), rows and pairs read one step ahead of their use
    constexpr int NR = R + 2 * P;
    lcdouble2 *yc = (lcdouble2 *)t.yc + ((t.wv - NP) * R) * W;
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      GDM_FENCE();
      const double av = as[s * TX];
      const double bv = BK ? bs[s * TX] : 0.0;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int k = j + 2 * P - s;  // column form: M(s - p + k, s)
        if (k >= 0 && k < W) {
          const dpair c = yc[s * W + k];
          D[j] = fma(c.x, av, D[j]);
          if constexpr (BK != 0) E[j] = fma(c.x, bv, fma(c.y, av, E[j]));
        }
      }
    }
  }
}

// One consumer plane: input plane zz, JP = (zz - zs) mod W (compile-time ring
// phase).  The z column comes from the LDS column table (wall columns, or the
// shared interior column), read one (e, d) pair ahead of its use.
template <int JP, int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void cplane7(const StencilArgs &a, const Tile7 &t, bool ytoep, int ybase, bool full,
                                        double (&acc)[2 * P + 1][R], int zz) {
  using G = Geom7<P, R, NC, NP, BK>;
  constexpr int W = G::W;
  double D[R], E[R];
  if (zz < t.ze) {
    ysweep7<P, R, NC, NP, BK>(a, t, ytoep, ybase, t.ab0 + ((zz - t.zs) & 1) * G::ABSZ, D, E);
    GDM_LDS_BARRIER();
  } else {
#pragma unroll
    for (int j = 0; j < R; ++j) D[j] = E[j] = 0.0;
  }
  const int row = zz < W ? zz : (zz >= a.Nz - W && zz < a.Nz ? W + zz - (a.Nz - W) : 2 * W);
  lcdouble2 *zc = (lcdouble2 *)t.zt + row * W;
  dpair cur = zc[0];
#pragma unroll
  for (int k = 0; k < W; ++k) {
    GDM_FENCE();
    const dpair nxt = zc[k + 1 < W ? k + 1 : k];
    const int slot = (JP - P + k + 2 * W) % W;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if constexpr (BK == 0)
        acc[slot][j] = fma(cur.y, D[j], acc[slot][j]);
      else
        acc[slot][j] = fma(cur.x, E[j], fma(cur.y, D[j], acc[slot][j]));
    }
    cur = nxt;
  }
  // The ring values only feed the conditional retire stores; without this
  // opaque use LLVM sinks each slot's whole FMA chain into its store branch
  // and keeps every plane's D/E and coefficients alive until then.
#pragma unroll
  for (int s = 0; s < W; ++s)
#pragma unroll
    for (int j = 0; j < R; ++j) asm volatile("" : "+v"(acc[s][j]));
  // retire output plane zz - p
  constexpr int rslot = (JP - P + 2 * W) % W;
  const int zo = zz - P;
  if (zo >= t.zc0 && zo < t.zc1) {
    const int Nx = a.Nx, x = t.x0 + t.lane;
    double *orow = a.dst + ((int64_t)(zo - a.out_z0) * (a.out_y1 - a.out_y0) + (ybase - a.out_y0)) * Nx + x;
    if (full) {
#pragma unroll
      for (int j = 0; j < R; ++j) orow[(int64_t)j * Nx] = acc[rslot][j];
    } else {
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (x < Nx && ybase + j < a.out_y1) orow[(int64_t)j * Nx] = acc[rslot][j];
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc[rslot][j] = 0.0;
}

template <int JP, int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void cblock7(const StencilArgs &a, const Tile7 &t, bool ytoep, int ybase, bool full,
                                        double (&acc)[2 * P + 1][R], int zb) {
  if constexpr (JP < 2 * P + 1) {
    cplane7<JP, P, R, NC, NP, BK>(a, t, ytoep, ybase, full, acc, zb + JP);
    cblock7<JP + 1, P, R, NC, NP, BK>(a, t, ytoep, ybase, full, acc, zb);
  }
}

template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void producer7(const StencilArgs &a, const Tile7 &t) {
  using G = Geom7<P, R, NC, NP, BK>;
  ldouble *u[2] = {t.u0, t.u0 + G::USZ};
  // prologue: planes zs, zs+1 in flight; x-sweep zs; plane zs+2 into the freed slot
  if (t.zs < t.ze) stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs, u[0]);
  if (t.zs + 1 < t.ze) {
    stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + 1, u[1]);
    wait_dma_plane<0, P, R, NC, NP, BK, CH>(t.wv);
  } else {
    GDM_WAIT_VMCNT(0);
  }
  if (t.zs < t.ze) {
    xsweep7<P, R, NC, NP, BK>(a, t, u[0], t.ab0);
    if (t.zs + 2 < t.ze) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stage_plane7<P, R, NC, NP, BK, CH>(a, t, t.zs + 2, u[0]);
    }
  }
  GDM_LDS_BARRIER();
  for (int zz = t.zs; zz < t.ze; ++zz) {
    const int q = zz + 1;  // plane swept in this iteration
    if (q < t.ze) {
      if (q + 1 < t.ze)
        wait_dma_plane<0, P, R, NC, NP, BK, CH>(t.wv);
      else
        GDM_WAIT_VMCNT(0);
      const int s = (q - t.zs) & 1;
      xsweep7<P, R, NC, NP, BK>(a, t, u[s], t.ab0 + s * G::ABSZ);
      if (q + 2 < t.ze) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage_plane7<P, R, NC, NP, BK, CH>(a, t, q + 2, u[s]);
      }
    }
    GDM_LDS_BARRIER();
  }
}

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void consumer7(const StencilArgs &a, const Tile7 &t) {
  using G = Geom7<P, R, NC, NP, BK>;
  constexpr int W = G::W;
  const int ybase = t.y0 + (t.wv - NP) * R;
  const bool ytoep = a.y_toep && (ybase >= P + 1) && (ybase + R - 1 + P + 2 <= a.Ny);
  const bool full = (t.x0 + G::TX <= a.Nx) && (ybase + R <= a.out_y1);
  double acc[W][R];
#pragma unroll
  for (int s = 0; s < W; ++s)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[s][j] = 0.0;
  GDM_LDS_BARRIER();
  for (int zb = t.zs; zb < t.zend; zb += W) cblock7<0, P, R, NC, NP, BK>(a, t, ytoep, ybase, full, acc, zb);
}

template <int P, int R, int NC, int NP, int BK, int CH>
__global__ void __launch_bounds__(64 * (NP + NC), (64 * (NP + NC)) / 256) stencil7_kernel(StencilArgs a) {
  using G = Geom7<P, R, NC, NP, BK>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  ldouble *lds = (ldouble *)smem;
  Tile7 t;
  t.u0 = lds;
  t.ab0 = lds + G::OFF_AB;
  t.zt = lds + G::OFF_ZT;
  t.yc = lds + G::OFF_YC;
  t.corr = lds + G::OFF_CORR;
  t.lane = threadIdx.x & 63;
  t.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.x0 = blockIdx.x * G::TX;
  t.y0 = a.out_y0 + blockIdx.y * G::TY;
  t.zc0 = a.out_z0 + blockIdx.z * a.zchunk;
  t.zc1 = min(t.zc0 + a.zchunk, a.out_z1);
  t.zs = max(t.zc0 - P, a.in_z0);
  t.ze = min(t.zc1 + P, a.in_z1);
  t.zend = t.zc1 + P;
  {
    const int L = a.x_corr_left, rb = a.Nx - a.x_corr_right;
    t.nl = max(0, min(L, t.x0 + G::TX) - t.x0);
    t.rs = max(rb, t.x0);
    const int nr = max(0, min(a.Nx, t.x0 + G::TX) - t.rs);
    t.ncw = t.nl + nr;
  }
  // tables into LDS (ordered before the first use by the prologue barrier)
  for (int e = threadIdx.x; e < G::ZTSZ; e += G::NT) t.zt[e] = a.zt[e];
  if (t.ncw > 0)
    for (int e = threadIdx.x; e < G::CORRSZ; e += G::NT) t.corr[e] = a.corrX[e];
  // tiles with rows next to a y wall: their column coefficients, pair (t1, t3)
  // per (tile row r, tap k); global table row = y0 + r (tables are padded by p)
  if (!(a.y_toep && t.y0 >= P + 1 && t.y0 + G::TY - 1 + P + 2 <= a.Ny))
    for (int e = threadIdx.x; e < G::UR * G::W; e += G::NT) {
      const int r = e / G::W, k = e - r * G::W;
      t.yc[2 * e] = a.yT1[(size_t)(t.y0 + r) * G::W + k];
      t.yc[2 * e + 1] = a.yT3[(size_t)(t.y0 + r) * G::W + k];
    }
  if (t.wv < NP)
    producer7<P, R, NC, NP, BK, CH>(a, t);
  else
    consumer7<P, R, NC, NP, BK>(a, t);
}

// ---------------------------------------------------------------------------
// Inflow boundary-data term (advection/stiffness.h:473-532 with a.n < 0):
//   rhs(node) += |a.n| sum_{q on face} u+_q phi_node(x_q) JxW_q
// factorised over the two tangential directions of the face:
//   step 1: T[q1][i0] = sum_m U[q1][qs0(i0) + m] w0[i0][m]
//   step 2: dst(i0, i1) += scale * sum_m w1[i1][m] T[qs1(i1) + m][i0]
// Step 1 stages ROWS rows of U (the q-range of FACE_CHUNK consecutive nodes)
// in LDS with coalesced loads; each lane then owns one node and reads its
// weights node-minor (w0T), so every global access is a contiguous wave row.
// ---------------------------------------------------------------------------
// boundary values U(i0, i1) of the face ([Q1][Q0] array).  (Evaluating the
// stage values of a built-in function here instead, per point, measured 2-3x
// slower than reading them: each lane's six consecutive points make every
// table read touch 64 cache lines; gdm_apply_bc_fn fills the array first.)
struct BcArr {
  const double *__restrict__ U;
  int Q0;
  __device__ __forceinline__ double operator()(int i0, int i1) const { return U[(int64_t)i1 * Q0 + i0]; }
};


template <int ROWS, class Src>
__global__ void __launch_bounds__(FACE_CHUNK) face_step1_kernel(const Src U, int Q0, int Q1,
                                                                 int i0_begin, int n0,
                                                                 const int *__restrict__ qs0,
                                                                 const double *__restrict__ w0T, int wmax0,
                                                                 int ldw0, int qmax, double *__restrict__ T) {
  extern __shared__ double sh[];  // [ROWS][qmax]
  const int c0 = blockIdx.x * FACE_CHUNK;
  const int q1b = blockIdx.y * ROWS;
  const int nc = min(FACE_CHUNK, n0 - c0);
  const int ia = i0_begin + c0;
  const int qa = qs0[ia];
  const int nq = min(Q0, qs0[ia + nc - 1] + wmax0) - qa;  // <= qmax (host-checked)
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    if (q1b + r < Q1) {
      for (int e = threadIdx.x; e < nq; e += FACE_CHUNK) sh[r * qmax + e] = U(qa + e, q1b + r);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x >= nc) return;
  const int i0 = ia + threadIdx.x;
  const int b = qs0[i0] - qa;
  const int mend = min(wmax0, nq - b);  // weights past the node's own count are 0
  double s[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) s[r] = 0.0;
  for (int m = 0; m < mend; ++m) {
    const double w = w0T[(int64_t)m * ldw0 + i0];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) s[r] = fma(w, sh[r * qmax + b + m], s[r]);
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r)
    if (q1b + r < Q1) T[(int64_t)(q1b + r) * n0 + c0 + threadIdx.x] = s[r];
}

// Step 1 in cell form: for one row q1 of the face, every local cell c reduces
// its p + 1 contiguous boundary values with its category's (p+1) x (p+1) table
// (S_c[l] = sum_q Phi[cat(c)][l][q] U[q1][c (p+1) + q], one contiguous read per
// cell, no per-node weight rows), then every owned node gathers the S_c of the
// cells whose DoF boxes contain it (system.h:195-246 box offsets).
__device__ __forceinline__ int face_category(int c, int p, int n) {
  const int half = p / 2;
  return c < half ? c : (c < n - half ? half : p + c - n);
}
__device__ __forceinline__ int face_box_offset(int c, int p, int n) {
  const int half = p / 2;
  return c < half ? 0 : min(n, c + half + 1) - p;
}

template <int P, class Src>
__device__ __forceinline__ void face_cell_step1_body(const Src &U, int Q0, int Q1, int rpb, int i0_begin, int n0,
                                                     const int *__restrict__ crange, const double *__restrict__ phi,
                                                     int ncell_total, int cell_begin, double *__restrict__ T,
                                                     int block) {
  constexpr int N1 = P + 1;
  extern __shared__ double sh[];  // [P][N1][N1] Phi, then [ncells][N1] S
  double *sphi = sh, *S = sh + P * N1 * N1;
  const int ncells = Q0 / N1;
  for (int e = threadIdx.x; e < P * N1 * N1; e += blockDim.x) sphi[e] = phi[e];
  const int r0 = block * rpb, r1 = min(Q1, r0 + rpb);
  for (int row = r0; row < r1; ++row) {
    __syncthreads();  // Phi ready / previous row's gather done
    for (int c = threadIdx.x; c < ncells; c += blockDim.x) {
      const int cat = face_category(cell_begin + c, P, ncell_total);
      double v[N1];
#pragma unroll
      for (int q = 0; q < N1; ++q) v[q] = U(c * N1 + q, row);
      const double *ph = sphi + cat * N1 * N1;
#pragma unroll
      for (int l = 0; l < N1; ++l) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < N1; ++q) s = fma(ph[l * N1 + q], v[q], s);
        S[c * N1 + l] = s;
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n0; t += blockDim.x) {
      const int i0 = i0_begin + t;
      const int cf = crange[2 * i0], cl = crange[2 * i0 + 1];
      double acc = 0.0;
      for (int c = cf; c <= cl; ++c) acc += S[c * N1 + (i0 - face_box_offset(cell_begin + c, P, ncell_total))];
      T[(int64_t)row * n0 + t] = acc;
    }
  }
}

// Step 1 of the rows [block rpb, block rpb + rpb) at once, all threads of the
// workgroup (the stencil's tail): the rows (contiguous in U) are staged in LDS
// with coalesced 16-B loads, all of them in flight together; each (row, cell)
// reduction then reads its N1 values from LDS and writes its N1 results over
// them (the same positions: in place, no barrier); one barrier; every
// (row, node) gather.  The same sums in the same order as
// face_cell_step1_body.  LDS: Phi, then [rpb][Q0] (U rows, then S).
template <int P>
__device__ __forceinline__ void face_cell_step1_rows(const BcArr &U, int Q0, int Q1, int rpb, int i0_begin, int n0,
                                                     const int *__restrict__ crange, const double *__restrict__ phi,
                                                     int ncell_total, int cell_begin, double *__restrict__ T,
                                                     int block) {
  constexpr int N1 = P + 1, MAXLD = 8;
  extern __shared__ double sh[];
  double *sphi = sh, *S = sh + ((P * N1 * N1 + 1) & ~1);  // 16-B aligned rows
  const int ncells = Q0 / N1;
  for (int e = threadIdx.x; e < P * N1 * N1; e += blockDim.x) sphi[e] = phi[e];
  const int r0 = block * rpb, nr = min(Q1, r0 + rpb) - r0;
  // stage rows r0 .. r0 + nr - 1 (nr * Q0 contiguous doubles of U)
  const double *src = U.U + (int64_t)r0 * Q0;
  const int n = nr * Q0;
  if ((((uintptr_t)src) & 15) == 0 && (n & 1) == 0) {
    const dpair *s2 = (const dpair *)src;
    ldouble2 *d2 = (ldouble2 *)S;
    for (int eb = 0; eb < n / 2; eb += MAXLD * (int)blockDim.x) {
      dpair v[MAXLD];
#pragma unroll
      for (int k = 0; k < MAXLD; ++k) {
        const int e = eb + k * (int)blockDim.x + (int)threadIdx.x;
        if (e < n / 2) v[k] = __builtin_nontemporal_load(s2 + e);
      }
#pragma unroll
      for (int k = 0; k < MAXLD; ++k) {
        const int e = eb + k * (int)blockDim.x + (int)threadIdx.x;
        if (e < n / 2) d2[e] = v[k];
      }
    }
  } else {
    for (int e = threadIdx.x; e < n; e += blockDim.x) S[e] = src[e];
  }
  __syncthreads();  // Phi and the rows staged
  for (int e = threadIdx.x; e < nr * ncells; e += blockDim.x) {
    const int r = e / ncells, c = e - r * ncells;
    double *Sc = S + (int64_t)r * Q0 + c * N1;
    double v[N1];
#pragma unroll
    for (int q = 0; q < N1; ++q) v[q] = Sc[q];
    const double *ph = sphi + face_category(cell_begin + c, P, ncell_total) * N1 * N1;
#pragma unroll
    for (int l = 0; l < N1; ++l) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < N1; ++q) acc = fma(ph[l * N1 + q], v[q], acc);
      Sc[l] = acc;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nr * n0; e += blockDim.x) {
    const int r = e / n0, t = e - r * n0;
    const int i0 = i0_begin + t;
    const int cf = crange[2 * i0], cl = crange[2 * i0 + 1];
    const double *Sr = S + (int64_t)r * Q0;
    double acc = 0.0;
    for (int c = cf; c <= cl; ++c) acc += Sr[c * N1 + (i0 - face_box_offset(cell_begin + c, P, ncell_total))];
    T[(int64_t)(r0 + r) * n0 + t] = acc;
  }
}

template <int P, class Src>
__global__ void __launch_bounds__(512) face_cell_step1_kernel(const Src U, int Q0, int Q1, int rpb,
                                                               int i0_begin, int n0, const int *__restrict__ crange,
                                                               const double *__restrict__ phi, int ncell_total,
                                                               int cell_begin, double *__restrict__ T) {
  face_cell_step1_body<P>(U, Q0, Q1, rpb, i0_begin, n0, crange, phi, ncell_total, cell_begin, T, blockIdx.x);
}

// every inflow face's step 1 (cell form) in one launch, face = blockIdx.y:
// the faces are independent (own T), so their rows share the GPU instead of
// running one face after the other (gdmk_launch_faces_step1)
template <class Src>
struct Step1Face {
  Src U;
  int Q0, Q1, i0_begin, n0;
  const int *crange;
  const double *phi;
  int ncell_total, cell_begin;
  double *T;
};
template <class Src>
struct Step1Set {
  Step1Face<Src> f[BcStage::kMaxFaces];
  int rpb;
};
template <int P, class Src>
__global__ void __launch_bounds__(512) face_cell_step1_multi_kernel(const Step1Set<Src> set) {
  const Step1Face<Src> &F = set.f[blockIdx.y];
  if ((int)blockIdx.x * set.rpb >= F.Q1) return;
  face_cell_step1_body<P>(F.U, F.Q0, F.Q1, set.rpb, F.i0_begin, F.n0, F.crange, F.phi, F.ncell_total, F.cell_begin,
                          F.T, blockIdx.x);
}

// ===========================================================================
// Fused Kronecker stencil, v8.  Same roles and tiles as v7:
//   * each producer wave DMAs its own row groups of the (TY + 2p) x (64 + 2p)
//     plane into a 2-slot LDS ring (a counted vmcnt keeps the next plane in
//     flight) and x-sweeps them straight into the (A, B) plane buffer i & 1,
//   * consumers read (A, B) pairs with one ds_read_b128, PF rows ahead, and
//     scatter into a register ring of 2p + 1 output planes,
//   * interior z planes use the compile-time bands (E arrives pre-scaled by
//     the z mass scale, D is scaled by dint): no LDS reads in the z phase;
//     only the 2(2p+1) wall planes read the LDS column table.
// The roles hand over the (A, B) planes through counters in LDS instead of a
// workgroup barrier per plane (the barrier serialised them):
//   FULL[s]  producers, after their rows of the plane in slot s are stored,
//   FREE[s]  consumers, once their reads of slot s have returned,
//   YWF      producers of a y-wall tile, after their y-wall corrections,
//   YWR      consumers, after reading the corrections (single-buffered only).
// Counters only grow; a wave waits for the count the plane needs, so waves
// of one role drift against each other and every SIMD keeps issuing.
// ===========================================================================
template <int P, int R, int NC, int NP, int BK>
struct Geom8 {
  static constexpr int W = 2 * P + 1;
  static constexpr int TX = 64;
  static constexpr int TY = R * NC;
  static constexpr int UR = TY + 2 * P;
  static constexpr int XH = P + 1;
  static constexpr int RL0 = TX + 2 * XH;
  static constexpr int RL = (RL0 % 4 == 2) ? RL0 : RL0 + 2;
  static constexpr int NW = NP + NC;
  static constexpr int NT = 64 * NW;
  static constexpr int NG = (UR + 3) / 4;
  static constexpr int NPASS = (NG + NP - 1) / NP;
  static constexpr int USZ = NG * 4 * RL;
  static constexpr int NAB = BK == 0 ? 1 : 2;
  // (A, B) pairs: row stride 2 TX doubles, pair x stored in slot
  // sw(x) = x ^ ((x >> 3) & 3).  Both access patterns are then bank-conflict
  // free: the consumers' ds_read_b128 (one pair per lane, lane groups
  // {0-3,12-15,20-27}, ... of MI355X_MICROARCH.md section LDS: 16 distinct
  // 16-B slots of the 256-B bank row) and the producers' ds_write_b128 (lane q
  // stores pairs 4q..4q+3; 8 contiguous lanes hit 8 distinct slots of 128 B).
  // (The padded layout of v8 made the reads 2-way: 41 % of LDS cycles.)
  static constexpr int ABRS = NAB == 2 ? 2 * TX : TX;
  static constexpr int ABSZ = UR * ABRS;
  static __device__ __forceinline__ int sw(int x) { return x ^ ((x >> 3) & 3); }
  static __device__ __forceinline__ int ab(int r, int x) { return NAB == 2 ? r * ABRS + 2 * sw(x) : r * TX + x; }
  static constexpr int ZTSZ = (2 * W + 1) * W * 2;  // wall planes + interior row
  // y-wall column tables: the tile rows [yb - y0, yb - y0 + YCR) that feed the
  // (at most p + 1) wall rows of the tile's one y wall
  static constexpr int YCR = 3 * P + 1;
  static constexpr int YCSZ = YCR * W * 2;
  static constexpr int CORRSZ = 2 * (P + 1) * 2 * W;
  static constexpr int NWIN = 2 * P + 6;
  // workgroups per CU the tile is sized for (<= 12 waves: two)
  static constexpr int WGS = NW <= 12 ? 2 : 1;
  static constexpr size_t LDS_CAP = (160 * 1024) / WGS;
  // double-buffered (A, B) planes, 2-slot DMA ring (the single-buffered
  // handoff and a 3-slot ring measured slower: profiles/r2_early, r3g)
  static constexpr int NSLOT = 2;
  static constexpr int NABUF = 2;
  static constexpr int YWSZ = (P + 1) * TX * NAB;  // y-wall corrections of one plane
  static constexpr int NSYNC = 8;                  // 32-bit hand-off counters (SY_*)
  static constexpr int OFF_AB = NSLOT * USZ;
  static constexpr int OFF_ZT = OFF_AB + NABUF * ABSZ;
  static constexpr int OFF_YC = OFF_ZT + ZTSZ;
  static constexpr int OFF_CORR = OFF_YC + YCSZ;
  static constexpr int OFF_SYNC = OFF_CORR + CORRSZ;
  static constexpr int OFF_YW = OFF_SYNC + NSYNC / 2;
  // y-wall corrections double-buffered where the LDS has room (p <= 7), else
  // one buffer and the producers wait for the consumers' reads (YWR)
  static constexpr int NYW = sizeof(double) * (size_t)(OFF_YW + 2 * YWSZ) <= LDS_CAP ? 2 : 1;
  static constexpr size_t lds_bytes() { return sizeof(double) * (size_t)(OFF_YW + NYW * YWSZ); }
};

// LDS hand-off counters of the v8 stencil (indices into Tile7::sync)
enum { SY_FULL = 0, SY_FREE = 2, SY_YWF = 4, SY_YWR = 5, SY_TAIL = 6 };

// wait until counter c has reached target (wave-uniform).  One asm block,
// spin included: a loop the compiler can see splits the live ranges of the
// consumers' register ring around it (158 VGPRs spilled to scratch); the
// spin sleeps between polls so that it takes few issue slots from the
// working waves
__device__ __forceinline__ void sync_wait(lu32 *c, unsigned target) {
  unsigned v, sv;
  asm volatile(
      "1:\n\t"
      "ds_read_b32 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %1, %0\n\t"
      "s_cmp_ge_u32 %1, %3\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n"
      "2:"
      : "=&v"(v), "=&s"(sv)
      : "v"((unsigned)(uintptr_t)c), "s"(target)
      : "memory", "scc");
}

// count this wave (one lane) in counter c once its LDS accesses so far have
// completed (stores landed, reads returned)
__device__ __forceinline__ void sync_signal(lu32 *c) {
  unsigned long long ex;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_u32 %1, %2\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(ex)
      : "v"((unsigned)(uintptr_t)c), "v"(1u)
      : "memory");
}

// the z-direction interior band of operator kind BK (column form index 2p - k)
template <int P, int BK>
__device__ __forceinline__ constexpr double zband(int k) {
  using IR = InteriorRows<P>;
  return BK == 0 ? IR::m[2 * P - k] : (BK == 1 ? IR::c[2 * P - k] : IR::l[2 * P - k]);
}

// run-time interior band coefficient k of kind BK from its first half: the
// bands are symmetric (mass, wave) or antisymmetric (advection, c[p] = 0), and
// the host tables (cy8, zd8, m_zd8: a scale times the band) inherit that
// exactly, so only p + 1 SGPR pairs stay live (the negation is an operand
// modifier of the FMA)
template <int P>
constexpr bool interior_bands_symmetric() {
  using IR = InteriorRows<P>;
  for (int k = 0; k <= 2 * P; ++k)
    if (IR::m[k] != IR::m[2 * P - k] || IR::l[k] != IR::l[2 * P - k] || IR::c[k] != -IR::c[2 * P - k]) return false;
  return IR::c[P] == 0.0;
}
// hcoef's reconstruction is exact only for exactly (anti)symmetric generated
// bands (gdm_coeffs.h); a one-ulp asymmetry would change the stencil silently
static_assert(interior_bands_symmetric<1>() && interior_bands_symmetric<3>() && interior_bands_symmetric<5>() &&
                  interior_bands_symmetric<7>() && interior_bands_symmetric<9>(),
              "interior bands must be exactly symmetric (m, l) / antisymmetric (c, c[p] = 0)");

template <int P, int BK>
__device__ __forceinline__ double hcoef(const double *c, int k) {
  if (k <= P) return c[k];
  return BK == 1 ? -c[2 * P - k] : c[2 * P - k];
}

// wait until at most K planes of DMA of this producer wave are in flight
template <int I, int K, int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void wait_dma_planes(int wv) {
  if constexpr (I < NP) {
    if (wv == I) {
      GDM_WAIT_VMCNT((K * Dma7<P, R, NC, NP, BK, CH>::nd(I)));
      return;
    }
    wait_dma_planes<I + 1, K, P, R, NC, NP, BK, CH>(wv);
  }
}

// x-sweep of row group g (pass of this producer wave) into registers:
// A = mhat*u (+ wall rows), B = sx bhat*u (+ wall rows), 4 consecutive x per lane.
// xload8 reads the lane's 16-B aligned window of the group's plane rows from
// LDS, xcalc8 computes from it (split so that a producer can release the u
// slot -- and issue the next DMA into it -- before the FMAs).
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xload8(const Tile7 &t, lcdouble *us, int g, double (&w)[Geom8<P, R, NC, NP, BK>::NWIN]) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int RL = G::RL;
  const int rr = t.lane >> 4, q = t.lane & 15;
  const int r = 4 * g + rr;
  lcdouble2 *wp = (lcdouble2 *)(us + r * RL + 4 * q);
#pragma unroll
  for (int i = 0; i < G::NWIN / 2; ++i) {
    const dpair v = wp[i];
    w[2 * i] = v.x;
    w[2 * i + 1] = v.y;
  }
}

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xcalc8(const StencilArgs &a, const double (&w)[Geom8<P, R, NC, NP, BK>::NWIN],
                                       dpair (&V)[4]) {
  // V[j] = (A_j, B_j) for x = 4 q + j (the pair the AB plane stores, so no
  // register moves before the b128 stores); mass: V[0] = (A_0, A_1), V[1] = (A_2, A_3)
  using G = Geom8<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W;
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
          // B* = sx bhat * u with the scale folded into the run-time band
          // cxs = sx bhat (first half in SGPRs, hcoef), c[p] == 0 skipped
          if (BK != 1 || k != P) V[j].y = fma(hcoef<P, BK>(a.cxs, k), w[j + k + 1], V[j].y);
        }
      }
  }
}

// The last row group of a tile when it holds at most 2 rows (p = 5: rows
// 40, 41 of 42): 2 rows x 64 x, two consecutive x per lane, so the wave
// issues half the FMAs of a 4-row group (whose rows 42, 43 would be discarded)
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xload8_half(const Tile7 &t, lcdouble *us, int g,
                                            double (&w)[Geom8<P, R, NC, NP, BK>::NWIN]) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int RL = G::RL, NW2 = 2 * P + 4;
  static_assert(NW2 <= G::NWIN, "half window");
  const int rr = t.lane >> 5, q = t.lane & 31;
  const int r = 4 * g + rr;
  lcdouble2 *wp = (lcdouble2 *)(us + r * RL + 2 * q);
#pragma unroll
  for (int i = 0; i < NW2 / 2; ++i) {
    const dpair v = wp[i];
    w[2 * i] = v.x;
    w[2 * i + 1] = v.y;
  }
}

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xcalc8_half(const StencilArgs &a, const Tile7 &t, int g,
                                            const double (&w)[Geom8<P, R, NC, NP, BK>::NWIN]) {
  using G = Geom8<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W;
  const int rr = t.lane >> 5, q = t.lane & 31;
  const int r = 4 * g + rr;
  dpair V[2] = {dpair{0.0, 0.0}, dpair{0.0, 0.0}};
#pragma unroll
  for (int k = 0; k < W; ++k)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (BK == 0) {
        if (j == 0)
          V[0].x = fma(IR::m[k], w[j + k + 1], V[0].x);
        else
          V[0].y = fma(IR::m[k], w[j + k + 1], V[0].y);
      } else {
        V[j].x = fma(IR::m[k], w[j + k + 1], V[j].x);
        if (BK != 1 || k != P) V[j].y = fma(hcoef<P, BK>(a.cxs, k), w[j + k + 1], V[j].y);
      }
    }
  if (r < G::UR) {
    if constexpr (BK != 0) {
      ldouble2 *row = (ldouble2 *)(t.ab0 + r * G::ABRS);
      row[G::sw(2 * q)] = V[0];
      row[G::sw(2 * q + 1)] = V[1];
    } else {
      *(ldouble2 *)(t.ab0 + r * G::TX + 2 * q) = V[0];
    }
  }
}

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xsweep8_half(const StencilArgs &a, const Tile7 &t, lcdouble *us, int g) {
  double w[Geom8<P, R, NC, NP, BK>::NWIN];
  xload8_half<P, R, NC, NP, BK>(t, us, g, w);
  xcalc8_half<P, R, NC, NP, BK>(a, t, g, w);
}

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xsweep8(const StencilArgs &a, const Tile7 &t, lcdouble *us, int g, dpair (&V)[4]) {
  double w[Geom8<P, R, NC, NP, BK>::NWIN];
  xload8<P, R, NC, NP, BK>(t, us, g, w);
  xcalc8<P, R, NC, NP, BK>(a, w, V);
}

// Wall columns of row group g (first / last x tiles only): the
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

// per-lane item geometry of the x-wall corrections, independent of the plane
// and (up to 4 g rows) of the row group: computed once per tile, so the plane
// loop carries no integer division
template <int P, int BK>
struct XWallPre {
  static constexpr int NI = XWall<P, BK>::NI;
  int u[NI], o[NI], c[NI], rr[NI];  // u-row offset, AB offset, table offset at g = 0; rr < 0: no item
};

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xwall8_pre(const StencilArgs &a, const Tile7 &t, XWallPre<P, BK> &pre) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int W = G::W, RL = G::RL, NCOMP = XWall<P, BK>::NCOMP;
  const int nitems = 4 * t.ncw * NCOMP;
#pragma unroll
  for (int it = 0; it < XWall<P, BK>::NI; ++it) {
    const int e = t.lane + 64 * it;
    const int comp = e % NCOMP, rest = e / NCOMP;
    const int idx = rest % max(t.ncw, 1), rr = rest / max(t.ncw, 1);
    const int x = idx < t.nl ? t.x0 + idx : t.rs + (idx - t.nl);
    const int cs = x < a.x_corr_left ? x : (P + 1) + (x - (a.Nx - a.x_corr_right));
    const int lx = x - t.x0;
    pre.rr[it] = e < nitems ? rr : -1;
    pre.u[it] = rr * RL + lx + 1;
    pre.o[it] = G::ab(rr, lx) + (BK != 0 ? comp : 0);
    pre.c[it] = cs * 2 * W + comp * W;
  }
}

template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void xwall8_calc(const Tile7 &t, lcdouble *us, int g, const XWallPre<P, BK> &pre,
                                            XWall<P, BK> &xw) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int W = G::W, RL = G::RL;
#pragma unroll
  for (int it = 0; it < XWall<P, BK>::NI; ++it) {
    xw.o[it] = -1;
    xw.v[it] = 0.0;
    if (pre.rr[it] >= 0 && 4 * g + pre.rr[it] < G::UR) {
      lcdouble *ur = us + 4 * g * RL + pre.u[it];  // tap k of the wall column
      lcdouble *cm = t.corr + pre.c[it];
      double d = 0.0;
#pragma unroll
      for (int k = 0; k < W; ++k) d = fma(cm[k], ur[k], d);
      xw.v[it] = d;
      // rows 4g.. of AB: G::ab is linear in the row
      xw.o[it] = 4 * g * G::ABRS + pre.o[it];
    }
  }
}

template <int P, int BK>
__device__ __forceinline__ void xwall8_add(const Tile7 &t, const XWall<P, BK> &xw) {
#pragma unroll
  for (int it = 0; it < XWall<P, BK>::NI; ++it)
    if (xw.o[it] >= 0) t.ab0[xw.o[it]] += xw.v[it];
}

// store row group g's (A, B) into the interleaved plane buffer
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void write_ab8(const Tile7 &t, int g, const dpair (&V)[4]) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int TX = G::TX;
  const int rr = t.lane >> 4, q = t.lane & 15;
  const int r = 4 * g + rr;
  if (r < G::UR) {
    if constexpr (BK != 0) {
      // sw(4q + j) = 4q + (j ^ t), t = (q >> 1) & 3: the lane's 4 pairs stay in its 4-pair block
      ldouble2 *p = (ldouble2 *)(t.ab0 + r * G::ABRS + 8 * q);
      const int tq = (q >> 1) & 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) p[j ^ tq] = V[j];
    } else {
      ldouble2 *p = (ldouble2 *)(t.ab0 + r * TX + 4 * q);
      p[0] = V[0];
      p[1] = V[1];
    }
  }
}

// first / end wall row of this tile's y-wall block (tile rows [y0, y0 + TY));
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

// y-wall corrections of the (A, B) plane in t.ab0 (y-wall tiles only, once
// every producer's rows of the plane are stored): for the wall rows y of this
// tile dD(y) = sum_s c1(y, s) A(s) and dE(y) = sum_s c1 B(s) + c3 A(s) with the
// (wall - Toeplitz) column tables, into t.yw; one row per producer wave, lane = x
template <int P, int R, int NC, int NP, int BK>
__device__ __forceinline__ void ywall8(const StencilArgs &a, const Tile7 &t) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int W = G::W, TX = G::TX;
  const int yb = ywall_begin<P, G::TY>(a, t.y0), ye = ywall_end<P, G::TY>(a, t.y0);
  // rows go to the producer waves from the last one down: the first waves
  // may own a second row group
  for (int y = yb + (NP - 1 - t.wv); y < ye; y += NP) {
    const int wi = y - yb;
    double dD = 0.0, dE = 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int rs = y + 2 * P - k - t.y0;  // tile row of input s = y + p - k
      const dpair c = ((lcdouble2 *)t.yc)[(rs - t.ry0) * W + k];
      if constexpr (BK != 0) {
        const dpair v = *(lcdouble2 *)(t.ab0 + G::ab(rs, t.lane));
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

// producer wave, plane i:
//   wait DMA(i) | wait FREE[i & 1] (consumers done with plane i - 2) |
//   X(i) -> (A, B) buffer i & 1 | FULL[i & 1] | DMA(i + 2) into the u slot just read |
//   [y-wall tile: wait FULL (all producers) | ywall(i) | YWF]
template <int P, int R, int NC, int NP, int BK, int CH>
__device__ __forceinline__ void producer8(const StencilArgs &a, const Tile7 &t) {
  using G = Geom8<P, R, NC, NP, BK>;
  ldouble *u[2] = {t.u0, t.u0 + G::USZ};
  const int n = t.ze - t.zs;
  DmaPre7<P, R, NC, NP, BK, CH> dpre;
  stage_pre7<P, R, NC, NP, BK, CH>(a, t, dpre);
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (k < n) stage_plane_pre7<P, R, NC, NP, BK, CH>(a, t, t.zs + k, u[k], dpre);
  GDM_LDS_BARRIER();  // tables in LDS, counters zeroed
  dpair V1[4];
  XWallPre<P, BK> xpre;
  if (t.ncw > 0) xwall8_pre<P, R, NC, NP, BK>(a, t, xpre);
  for (int i = 0; i < n; ++i) {
    const int slot = i & 1;
    if (i + 1 < n)
      wait_dma_planes<0, 1, P, R, NC, NP, BK, CH>(t.wv);
    else
      GDM_WAIT_VMCNT(0);
    Tile7 tt = t;
    tt.ab0 = t.ab0 + slot * G::ABSZ;
    tt.yw = t.yw + (G::NYW == 2 ? slot : 0) * G::YWSZ;
    sync_wait(t.sync + SY_FREE + slot, NC * (i >> 1));
    constexpr bool half_last = G::UR - 4 * (G::NG - 1) <= 2;
    // the window reads of all this wave's row groups first: the second
    // group's LDS latency overlaps the first group's FMAs (the compiler cannot
    // hoist them itself past the (A, B) stores, which it cannot prove disjoint)
    double win[G::NPASS][G::NWIN];
#pragma unroll
    for (int ps = 0; ps < G::NPASS; ++ps) {
      const int g = t.wv + ps * NP;
      if (g < G::NG) {
        if (half_last && g == G::NG - 1)
          xload8_half<P, R, NC, NP, BK>(tt, u[slot], g, win[ps]);
        else
          xload8<P, R, NC, NP, BK>(tt, u[slot], g, win[ps]);
      }
    }
#pragma unroll
    for (int ps = 0; ps < G::NPASS; ++ps) {
      const int g = t.wv + ps * NP;
      if (g < G::NG) {
        if (half_last && g == G::NG - 1) {
          xcalc8_half<P, R, NC, NP, BK>(a, tt, g, win[ps]);
        } else {
          xcalc8<P, R, NC, NP, BK>(a, win[ps], V1);
          write_ab8<P, R, NC, NP, BK>(tt, g, V1);
        }
        if (t.ncw > 0) {
          XWall<P, BK> xw0;
          xwall8_calc<P, R, NC, NP, BK>(tt, u[slot], g, xpre, xw0);
          xwall8_add<P, BK>(tt, xw0);
        }
      }
    }
    // (the wait in sync_signal also orders this wave's reads of the u slot
    // before the DMA that overwrites it)
    sync_signal(t.sync + SY_FULL + slot);
    if (i + 2 < n) stage_plane_pre7<P, R, NC, NP, BK, CH>(a, t, t.zs + i + 2, u[slot], dpre);
    // y-wall tiles: only the waves that own a wall row (rows go to the waves
    // from the last one down) wait for the whole plane and count in YWF; the
    // others -- the first waves, which carry the second row groups -- go on
    // to their next plane
    if (t.yedge && NP - 1 - t.wv < t.nyw) {
      sync_wait(t.sync + SY_FULL + slot, NP * ((i >> 1) + 1));
      if constexpr (G::NYW == 1) sync_wait(t.sync + SY_YWR, NC * i);
      ywall8<P, R, NC, NP, BK>(a, tt);
      sync_signal(t.sync + SY_YWF);
    }
  }
}

// y-sweep of the consumer's R rows from the (A, B) plane: D' and E with the
// compile-time interior bands, rows read PF ahead of their use (wall rows get
// their corrections from the producers' ywall8, see cplane8).
template <int P, int R, int NC, int NP, int BK, int PF>
__device__ __forceinline__ void ysweep8(const StencilArgs &a, const Tile7 &t, double (&D)[R], double (&E)[R]) {
  using G = Geom8<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W, TX = G::TX, NR = R + 2 * P;
  const int row0 = t.cw * R;
#pragma unroll
  for (int j = 0; j < R; ++j) D[j] = E[j] = 0.0;
  if constexpr (BK != 0) {
    lcdouble2 *vp = (lcdouble2 *)(t.ab0 + G::ab(row0, t.lane));
    dpair v[NR];
#pragma unroll
    for (int s = 0; s < PF && s < NR; ++s) v[s] = vp[s * (G::ABRS / 2)];
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      GDM_FENCE();
      if (s + PF < NR) v[s + PF] = vp[(s + PF) * (G::ABRS / 2)];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int k = s - j;  // row form: M(y_j, y_j - p + k)
        if (k >= 0 && k < W) {
          D[j] = fma(IR::m[k], v[s].x, D[j]);
          if (BK == 1 && k == P)  // cy[p] = h_x a_y chat[p] = 0
            E[j] = fma(IR::m[k], v[s].y, E[j]);
          else
            E[j] = fma(IR::m[k], v[s].y, fma(hcoef<P, BK>(a.cy, k), v[s].x, E[j]));
        }
      }
    }
  } else {
    const volatile lcdouble *vp = t.ab0 + row0 * TX + t.lane;
    double v[NR];
#pragma unroll
    for (int s = 0; s < PF && s < NR; ++s) v[s] = vp[s * TX];
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      GDM_FENCE();
      if (s + PF < NR) v[s + PF] = vp[(s + PF) * TX];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int k = s - j;
        if (k >= 0 && k < W) D[j] = fma(IR::m[k], v[s], D[j]);
      }
    }
  }
}

// consumer wave, input plane zz (index i = zz - zs):
//   wait FULL[i & 1] | Y(i) [+ y-wall corrections after YWF] | FREE[i & 1] |
//   Z(i) | retire output plane zz - p
template <int JP, int P, int R, int NC, int NP, int BK, int PF, bool WALL, bool YW>
__device__ __forceinline__ void cplane8(const StencilArgs &a, const Tile7 &t, int ybase, bool full, bool ywave,
                                        double (&acc)[2 * P + 1][R], int zz) {
  using G = Geom8<P, R, NC, NP, BK>;
  using IR = InteriorRows<P>;
  constexpr int W = G::W;
  if (zz < t.ze) {
    const int i = zz - t.zs, bs = i & 1;  // (A, B) buffer of the plane
    double D[R], E[R];
    sync_wait(t.sync + SY_FULL + bs, NP * ((i >> 1) + 1));
    Tile7 tt = t;
    tt.ab0 = t.ab0 + bs * G::ABSZ;
    ysweep8<P, R, NC, NP, BK, PF>(a, tt, D, E);
    if constexpr (YW) {
      if (ywave) {
        sync_wait(t.sync + SY_YWF, t.nyw * (i + 1));
        const ldouble *yw = t.yw + (G::NYW == 2 ? bs : 0) * G::YWSZ;
        const int yb = ywall_begin<P, G::TY>(a, t.y0), ye = ywall_end<P, G::TY>(a, t.y0);
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const int y = ybase + j;
          if (y >= yb && y < ye) {
            if constexpr (BK != 0) {
              const dpair c = ((lcdouble2 *)yw)[(y - yb) * G::TX + t.lane];
              D[j] += c.x;
              E[j] += c.y;
            } else {
              D[j] += yw[(y - yb) * G::TX + t.lane];
            }
          }
        }
      }
      if constexpr (G::NYW == 1) sync_signal(t.sync + SY_YWR);
    }
    sync_signal(t.sync + SY_FREE + bs);
    // MF: the slot of output zz + p (k = 2p) was retired by the previous
    // plane; its first term overwrites it (a multiply instead of a zeroing
    // move + FMA).  Outputs whose first plane zz + p - 2p precedes the chunk
    // start keep the ring's initial zeros and only ever see FMAs.
    constexpr bool MF = true;
    if constexpr (!WALL) {
      // interior z column: out += mhat[k] E + zd[k] D with zd = dint dhat[2p - k]
      // (the scale folded into the coefficients; zd[p] = 0 for advection)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        GDM_FENCE();
        const int slot = (JP - P + k + 2 * W) % W;
        const bool first = MF && k == W - 1;
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const double c0 = first ? 0.0 : acc[slot][j];
          if constexpr (BK == 0)
            acc[slot][j] = first ? hcoef<P, BK>(a.zd, k) * D[j] : fma(hcoef<P, BK>(a.zd, k), D[j], c0);
          else if (zband<P, BK>(k) == 0.0)
            acc[slot][j] = first ? IR::m[k] * E[j] : fma(IR::m[k], E[j], c0);
          else
            acc[slot][j] =
                fma(IR::m[k], E[j], first ? hcoef<P, BK>(a.zd, k) * D[j] : fma(hcoef<P, BK>(a.zd, k), D[j], c0));
        }
      }
    } else {
      // wall blocks: every plane from the column table (row 2W = interior)
      const int row = zz < W ? zz : (zz >= a.Nz - W ? W + zz - (a.Nz - W) : 2 * W);
      lcdouble2 *zc = (lcdouble2 *)t.zt + row * W;
      dpair cur = zc[0];
#pragma unroll
      for (int k = 0; k < W; ++k) {
        GDM_FENCE();
        const dpair nxt = zc[k + 1 < W ? k + 1 : k];
        const int slot = (JP - P + k + 2 * W) % W;
        const bool first = MF && k == W - 1;
#pragma unroll
        for (int j = 0; j < R; ++j) {
          if constexpr (BK == 0)
            acc[slot][j] = first ? cur.y * D[j] : fma(cur.y, D[j], acc[slot][j]);
          else
            acc[slot][j] = fma(cur.x, E[j], first ? cur.y * D[j] : fma(cur.y, D[j], acc[slot][j]));
        }
        cur = nxt;
      }
    }
  }
  // The ring values only feed the conditional retire stores; without this
  // opaque use LLVM sinks each slot's whole FMA chain into its store branch
  // and keeps every plane's D/E and coefficients alive until then.
#pragma unroll
  for (int s = 0; s < W; ++s)
#pragma unroll
    for (int j = 0; j < R; ++j) asm volatile("" : "+v"(acc[s][j]));
  // retire output plane zz - p
  constexpr int rslot = (JP - P + 2 * W) % W;
  const int zo = zz - P;
  if (zo >= t.zc0 && zo < t.zc1) {
    const int Nx = a.Nx, x = t.x0 + t.lane;
    // buffer stores: the plane's base in the resource (scalar), the lane's
    // row offset a per-wave constant, row j's offset in soffset -- no 64-bit
    // per-lane address arithmetic per plane (non-temporal, cpol 2 = nt);
    // partial tiles mask rows (wave-uniform) and lanes
    const double *pb = a.dst + (int64_t)(zo - a.out_z0) * (a.out_y1 - a.out_y0) * Nx;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)pb, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (full || (ybase + j < a.out_y1 && x < Nx))
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, acc[rslot][j]), rs, t.ooff, j * Nx * 8, 2);
  }
  }

template <int JP, int P, int R, int NC, int NP, int BK, int PF, bool WALL, bool YW>
__device__ __forceinline__ void cblock8(const StencilArgs &a, const Tile7 &t, int ybase, bool full, bool ywave,
                                        double (&acc)[2 * P + 1][R], int zb) {
  if constexpr (JP < 2 * P + 1) {
    cplane8<JP, P, R, NC, NP, BK, PF, WALL, YW>(a, t, ybase, full, ywave, acc, zb + JP);
    cblock8<JP + 1, P, R, NC, NP, BK, PF, WALL, YW>(a, t, ybase, full, ywave, acc, zb);
  }
}

template <int P, int R, int NC, int NP, int BK, int PF, bool YW>
__device__ __forceinline__ void consumer8_loop(const StencilArgs &a, const Tile7 &t, int ybase, bool full,
                                               bool ywave) {
  using G = Geom8<P, R, NC, NP, BK>;
  constexpr int W = G::W;
  double acc[W][R];
#pragma unroll
  for (int s = 0; s < W; ++s)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[s][j] = 0.0;
  GDM_LDS_BARRIER();  // tables in LDS, counters zeroed
  // Input plane zz scatters with its z column: a wall column for zz < W or
  // zz >= Nz - W (LDS table), else the interior one.  Blocks of W planes that
  // hold a wall column run the table path for all their planes, the others
  // the compile-time bands; the table's interior row holds exactly the
  // compile-time coefficients, so a plane gives the same bits in either path,
  // whatever the launched plane range (gdm_apply_planes, the overlapped
  // exchange).  The z-wall planes are part of the chunks of this launch: no
  // second launch with 2p-plane halos of its own.  Three loops, not a branch
  // per block (a loop carrying both paths measured 1.25 vs 0.86 ms at C3 in
  // round 3, profiles/r3j/ab_zmix.txt).
  int zb = t.zs;
  for (; zb < t.zend && zb < W; zb += W) cblock8<0, P, R, NC, NP, BK, PF, true, YW>(a, t, ybase, full, ywave, acc, zb);
  const int zhi = a.Nz - 2 * W + 1;  // zb < zhi: no wall column in [zb, zb + W)
  for (; zb < t.zend && zb < zhi; zb += W)
    cblock8<0, P, R, NC, NP, BK, PF, false, YW>(a, t, ybase, full, ywave, acc, zb);
  for (; zb < t.zend; zb += W) cblock8<0, P, R, NC, NP, BK, PF, true, YW>(a, t, ybase, full, ywave, acc, zb);
}

template <int P, int R, int NC, int NP, int BK, int PF>
__device__ __forceinline__ void consumer8(const StencilArgs &a, Tile7 t) {
  using G = Geom8<P, R, NC, NP, BK>;
  const int ybase = t.y0 + t.cw * R;
  const bool full = (t.x0 + G::TX <= a.Nx) && (ybase + R <= a.out_y1);
  t.ooff = (unsigned)(((ybase - a.out_y0) * a.Nx + t.x0 + t.lane) * 8);
  // edge tiles (rows next to a y wall) wait for the producers' y-wall
  // corrections every plane: their own copy of the loop keeps that out of the
  // hot block of the other tiles
  if (t.yedge) {
    const int yb = ywall_begin<P, G::TY>(a, t.y0), ye = ywall_end<P, G::TY>(a, t.y0);
    const bool ywave = ybase < ye && ybase + R > yb;
    consumer8_loop<P, R, NC, NP, BK, PF, true>(a, t, ybase, full, ywave);
  } else {
    consumer8_loop<P, R, NC, NP, BK, PF, false>(a, t, ybase, full, false);
  }
}

// Work the stencil's workgroups take on once their chunk is done: the inflow
// faces' step 1 (face_cell_step1_body), row blocks handed out by a device
// counter.  One workgroup per CU and one round: the wall tiles finish last,
// and this fills their tail.  A separate side-stream launch of the same work
// starved the stencil instead: its small workgroups took the CUs that the
// stencil's whole-CU workgroups were waiting for.  Each launch is
// self-contained: the counter is 0 when it starts, every workgroup ends with
// one claim past the items, and the workgroup that makes the launch's last
// claim (items + workgroups - 1) sets it back to 0 -- all other claims have
// been made by then -- so stream-ordered launches and graph replays need no
// host-side state.
struct StencilTail {
  Step1Set<BcArr> s1;
  int nfaces, items;
  int first[BcStage::kMaxFaces + 1];  // item range of face f: [first[f], first[f + 1])
  unsigned long long *counter;
};

template <int P>
__device__ __forceinline__ void stencil_tail(const StencilTail &tl, lu32 *slot) {
  __syncthreads();  // every role is done with the LDS
  while (true) {
    if (threadIdx.x == 0) {
      const unsigned long long v = atomicAdd(tl.counter, 1ull);
      const unsigned long long last =
          (unsigned long long)tl.items + (unsigned long long)gridDim.x * gridDim.y * gridDim.z - 1ull;
      if (v == last) atomicExch(tl.counter, 0ull);  // the launch's last claim: reset for the next launch
      *slot = (unsigned)(v < (unsigned long long)tl.items ? v : (unsigned long long)tl.items);
    }
    __syncthreads();
    const int it = (int)*slot;
    __syncthreads();
    if (it >= tl.items) break;
    int f = 0;
    while (f + 1 < tl.nfaces && it >= tl.first[f + 1]) ++f;
    const Step1Face<BcArr> &F = tl.s1.f[f];
    face_cell_step1_rows<P>(F.U, F.Q0, F.Q1, tl.s1.rpb, F.i0_begin, F.n0, F.crange, F.phi, F.ncell_total,
                            F.cell_begin, F.T, it - tl.first[f]);
    __syncthreads();  // the rows' gathers are done with S before the next item's reductions
  }
}

template <int P, int R, int NC, int NP, int BK, int CH, int PF>
__global__ void __launch_bounds__(64 * (NP + NC), ((NP + NC) * Geom8<P, R, NC, NP, BK>::WGS) / 4)
    stencil8_kernel(StencilArgs a, StencilTail tail) {
  using G = Geom8<P, R, NC, NP, BK>;
  static_assert(G::lds_bytes() <= G::LDS_CAP, "LDS budget");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  ldouble *lds = (ldouble *)smem;
  Tile7 t;
  t.u0 = lds;
  t.ab0 = lds + G::OFF_AB;
  t.zt = lds + G::OFF_ZT;
  t.yc = lds + G::OFF_YC;
  t.corr = lds + G::OFF_CORR;
  t.sync = (lu32 *)(lds + G::OFF_SYNC);
  t.yw = lds + G::OFF_YW;
  t.lane = threadIdx.x & 63;
  t.wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  t.cw = t.wv - NP;
  // XCD-aware tile order: the hardware deals workgroup b to XCD b % 8; XCD k
  // gets the contiguous logical range [k q, (k + 1) q) of tiles (x fastest),
  // so the tiles sharing x- and y-halo lines run on one XCD at the same time
  // and those lines are fetched from HBM once into that XCD's L2.
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (a.xcd_map) {
    const int64_t gx = gridDim.x, gy = gridDim.y;
    const int64_t nb = gx * gy * gridDim.z, q = nb / 8;
    const int64_t b = blockIdx.x + gx * (blockIdx.y + gy * (int64_t)blockIdx.z);
    const int64_t L = b >= 8 * q ? b : (b % 8) * q + b / 8;
    bx = (int)(L % gx);
    by = (int)((L / gx) % gy);
    bz = (int)(L / (gx * gy));
  }
  t.x0 = bx * G::TX;
  t.y0 = a.out_y0 + by * G::TY;
  const int yb = ywall_begin<P, G::TY>(a, t.y0);
  t.yedge = yb >= 0;
  t.ry0 = yb - t.y0;
  t.nyw = t.yedge ? min(NP, ywall_end<P, G::TY>(a, t.y0) - yb) : 0;
  {
    const int r = bz < a.nchunk0 ? 0 : 1;
    const int c = bz - (r ? a.nchunk0 : 0);
    t.zc0 = a.cz0[r] + c * a.zchunk;
    t.zc1 = min(t.zc0 + a.zchunk, a.cz1[r]);
  }
  t.zs = max(t.zc0 - P, a.in_z0);
  t.ze = min(t.zc1 + P, a.in_z1);
  t.zend = t.zc1 + P;
  {
    const int L = a.x_corr_left, rb = a.Nx - a.x_corr_right;
    t.nl = max(0, min(L, t.x0 + G::TX) - t.x0);
    t.rs = max(rb, t.x0);
    const int nr = max(0, min(a.Nx, t.x0 + G::TX) - t.rs);
    t.ncw = t.nl + nr;
  }
  if (threadIdx.x < G::NSYNC) t.sync[threadIdx.x] = 0u;
  for (int e = threadIdx.x; e < G::ZTSZ; e += G::NT) t.zt[e] = a.zt[e];
  if (t.ncw > 0)
    for (int e = threadIdx.x; e < G::CORRSZ; e += G::NT) t.corr[e] = a.corrX[e];
  // y-wall tiles: (wall - Toeplitz) column corrections of the tile rows
  // [ry0, ry0 + YCR) (global table row = y0 + tile row; tables are padded by p)
  if (t.yedge) {
    const int nr = min(G::YCR, G::UR - t.ry0);
    for (int e = threadIdx.x; e < nr * G::W; e += G::NT) {
      const int r = e / G::W, k = e - r * G::W;
      t.yc[2 * e] = a.yT1[(size_t)(t.y0 + t.ry0 + r) * G::W + k];
      t.yc[2 * e + 1] = a.yT3[(size_t)(t.y0 + t.ry0 + r) * G::W + k];
    }
  }
  if (t.wv < NP)
    producer8<P, R, NC, NP, BK, CH>(a, t);
  else
    consumer8<P, R, NC, NP, BK, PF>(a, t);
  if (tail.items > 0) stencil_tail<P>(tail, t.sync + SY_TAIL);
}

// ---------------------------------------------------------------------------
// Exact Kronecker mass inverse: banded Cholesky solves along one direction.
// One thread per line; the position along the line is wave-uniform, so the
// factor entries are scalar loads.  line l -> base = (l / A) * B + (l % A) * C.
// lrow: (len + P) x (P + 1), rows >= len zero-padded.
// ---------------------------------------------------------------------------
template <int P>
__global__ void __launch_bounds__(256) chol_lines_kernel(double *__restrict__ v, int len, int64_t stride,
                                                          int64_t n_lines, int64_t A, int64_t B, int64_t C,
                                                          const double *__restrict__ lrow,
                                                          const double *__restrict__ inv_diag) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_lines) return;
  double *line = v + (l / A) * B + (l % A) * C;
  double win[P];
#pragma unroll
  for (int k = 0; k < P; ++k) win[k] = 0.0;
  // forward: w_i = (r_i - sum_k L(i, i-P+k) w_{i-P+k}) / L(i,i)
  for (int i = 0; i < len; ++i) {
    const double *L = lrow + (size_t)i * (P + 1);
    double s = line[(int64_t)i * stride];
#pragma unroll
    for (int k = 0; k < P; ++k) s = fma(-L[k], win[k], s);
    s *= inv_diag[i];
    line[(int64_t)i * stride] = s;
#pragma unroll
    for (int k = 0; k < P - 1; ++k) win[k] = win[k + 1];
    win[P - 1] = s;
  }
#pragma unroll
  for (int k = 0; k < P; ++k) win[k] = 0.0;
  // backward: x_i = (w_i - sum_m L(i+m, i) x_{i+m}) / L(i,i)
  for (int i = len - 1; i >= 0; --i) {
    double s = line[(int64_t)i * stride];
#pragma unroll
    for (int m = 1; m <= P; ++m) s = fma(-lrow[(size_t)(i + m) * (P + 1) + (P - m)], win[m - 1], s);
    s *= inv_diag[i];
    line[(int64_t)i * stride] = s;
#pragma unroll
    for (int m = P - 1; m > 0; --m) win[m] = win[m - 1];
    win[0] = s;
  }
}

// scale sum_m w1[i1][m] T[q + m][t], the product rounded on its own: the
// compiler may not fuse it into the later add (one FMA would round
// differently from the face-by-face path's dst + G)
__device__ __forceinline__ double face_step2_value(const double *__restrict__ T, int n0, int t, int i1,
                                                   const int *__restrict__ qs1, const int *__restrict__ qc1,
                                                   const double *__restrict__ w1, int wmax1, double scale) {
  const double *w = w1 + (int64_t)i1 * wmax1;
  const int n = qc1[i1], q = qs1[i1];
  const double *Tc = T + (int64_t)q * n0 + t;
  double s = 0.0;
  int m = 0;
  // groups of 6 loads in flight, the FMAs in increasing m (the order of the
  // one-at-a-time loop: same bits)
  for (; m + 6 <= n; m += 6) {
    double tv[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) tv[u] = Tc[(int64_t)(m + u) * n0];
#pragma unroll
    for (int u = 0; u < 6; ++u) s = fma(w[m + u], tv[u], s);
  }
  for (; m < n; ++m) s = fma(w[m], Tc[(int64_t)m * n0], s);
  double v;
  {
#pragma clang fp contract(off)
    v = scale * s;
  }
  asm volatile("" : "+v"(v));
  return v;
}

// dst node (t, i1) += scale sum_m w1[i1][m] T[q + m][t]: one face (face by face, in face order)
__global__ void __launch_bounds__(256) face_step2_kernel(const double *__restrict__ T, int n0, int i1_begin,
                                                          int i1_end, const int *__restrict__ qs1,
                                                          const int *__restrict__ qc1,
                                                          const double *__restrict__ w1, int wmax1,
                                                          double *__restrict__ dst, int64_t base,
                                                          int64_t stride0, int64_t stride1, double scale) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i1 = i1_begin + (int)blockIdx.y;
  if (t >= n0 || i1 >= i1_end) return;
  const double v = face_step2_value(T, n0, t, i1, qs1, qc1, w1, wmax1, scale);
  double *d = dst + base + (int64_t)t * stride0 + (int64_t)(i1 - i1_begin) * stride1;
  *d = *d + v;
}

// step-2 data of one face for face_step2_add_kernel
struct Step2Face {
  const double *T;
  int n0, i1_begin, i1_end;
  const int *qs1, *qc1;
  const double *w1;
  int wmax1;
  double scale;
};
__device__ __forceinline__ bool face_add_member(const FaceAddFace &g, const int c[3]) {
  return c[g.d] == g.plane && (g.a0 < 0 || (c[g.a0] >= g.b0 && c[g.a0] < g.e0)) &&
         (g.a1 < 0 || (c[g.a1] >= g.b1 && c[g.a1] < g.e1));
}
// step 2 of every inflow face fused with the ordered adds (one launch, face =
// blockIdx.z): a node is handled by the thread of the first face containing
// it, which adds its own face's G = scale sum_m w1 T and then every later
// containing face's G, in face order -- the sums (and roundings) of the
// per-face step-2 launches, without the G buffers and the separate add launch
struct Step2AddSet {
  Step2Face f[BcStage::kMaxFaces];
  FaceAddFace g[BcStage::kMaxFaces];
  int n;
  int64_t N0, N1, own_off;
};
// One thread per node column t and R1 consecutive i1 rows: the rows' T
// windows overlap (consecutive nodes shift by one cell), so the thread walks
// the union of their q ranges once and feeds each row's sum in increasing m
// -- the same FMA sequence per node as face_step2_value, with ~R1 / 4 of its
// T loads.  Weights and q ranges are wave-uniform (scalar loads).
template <int R1>
__global__ void __launch_bounds__(64) face_step2_add_kernel(const Step2AddSet set, double *__restrict__ dst) {
  const int f = blockIdx.z;
  const Step2Face &F = set.f[f];
  const FaceAddFace &A = set.g[f];
  const int r0 = blockIdx.y * R1, nr = min(R1, F.i1_end - F.i1_begin - r0);
  if (nr <= 0) return;
  const int t = blockIdx.x * 64 + threadIdx.x;
  const bool on = t < F.n0;
  const int tt = on ? t : F.n0 - 1;  // idle lanes repeat a valid column (no divergence in the q walk)
  const int i1a = F.i1_begin + r0;
  int qlo = F.qs1[i1a], qhi = qlo;
#pragma unroll
  for (int j = 0; j < R1; ++j)
    if (j < nr) {
      qlo = min(qlo, F.qs1[i1a + j]);
      qhi = max(qhi, F.qs1[i1a + j] + F.qc1[i1a + j]);
    }
  double sum[R1];
  int qs[R1], qe[R1];
  const double *wr[R1];
#pragma unroll
  for (int j = 0; j < R1; ++j) {
    sum[j] = 0.0;
    qs[j] = j < nr ? F.qs1[i1a + j] : 0;
    qe[j] = j < nr ? qs[j] + F.qc1[i1a + j] : 0;
    wr[j] = F.w1 + (int64_t)(i1a + j) * F.wmax1 - qs[j];  // wr[j][q] = w1[i1][q - qs]
  }
  const double *Tc = F.T + tt;
  int q = qlo;
  for (; q + 6 <= qhi; q += 6) {
    double tv[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) tv[u] = Tc[(int64_t)(q + u) * F.n0];
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
      for (int j = 0; j < R1; ++j)
        if (q + u >= qs[j] && q + u < qe[j]) sum[j] = fma(wr[j][q + u], tv[u], sum[j]);
  }
  for (; q < qhi; ++q) {
    const double tv = Tc[(int64_t)q * F.n0];
#pragma unroll
    for (int j = 0; j < R1; ++j)
      if (q >= qs[j] && q < qe[j]) sum[j] = fma(wr[j][q], tv, sum[j]);
  }
  if (!on) return;
#pragma unroll
  for (int j = 0; j < R1; ++j) {
    if (j >= nr) break;
    const int r = r0 + j;
    const int64_t o = A.base + (int64_t)t * A.stride0 + (int64_t)r * A.stride1;
    const int64_t gi = o + set.own_off;
    const int c[3] = {(int)(gi % set.N0), (int)((gi / set.N0) % set.N1), (int)(gi / (set.N0 * set.N1))};
    bool mine = true;
    for (int g = 0; g < f; ++g)
      if (face_add_member(set.g[g], c)) mine = false;
    if (!mine) continue;  // the node's first face adds every face's term
    double gv;
    {
#pragma clang fp contract(off)
      gv = F.scale * sum[j];
    }
    asm volatile("" : "+v"(gv));
    double v = dst[o];
    v = v + gv;
    for (int g = f + 1; g < set.n; ++g) {
      const FaceAddFace &H = set.g[g];
      if (!face_add_member(H, c)) continue;
      const Step2Face &S = set.f[g];
      const int u0 = H.a0 < 0 ? 0 : c[H.a0] - H.b0, u1 = H.a1 < 0 ? 0 : c[H.a1] - H.b1;
      v = v + face_step2_value(S.T, S.n0, u0, S.i1_begin + u1, S.qs1, S.qc1, S.w1, S.wmax1, S.scale);
    }
    dst[o] = v;
  }
}

// ---------------------------------------------------------------------------
// BLAS-1
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) axpby_kernel(int64_t n, double a, const double *__restrict__ x, double b,
                                                     double *__restrict__ y) {
  const int64_t n2 = n / 2;
  const double2 *x2 = reinterpret_cast<const double2 *>(x);
  double2 *y2 = reinterpret_cast<double2 *>(y);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 xv = x2[i];
    double2 yv = y2[i];
    yv.x = fma(a, xv.x, b * yv.x);
    yv.y = fma(a, xv.y, b * yv.y);
    y2[i] = yv;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) y[n - 1] = fma(a, x[n - 1], b * y[n - 1]);
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) dot_partial_kernel(int64_t n, const double *__restrict__ x,
                                                           const double *__restrict__ y,
                                                           double *__restrict__ partial) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s = fma(x[i], y[i], s);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) dot_final_kernel(int n, const double *__restrict__ partial,
                                                         double *__restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) zero_kernel(int64_t n, double *__restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = 0.0;
}

// ---------------------------------------------------------------------------
// host-side launchers (called from gdm_capi.cpp)
// ---------------------------------------------------------------------------
template <int P, int R, int NC, int NP, int BK, int CH>
static hipError_t launch7_t(const StencilArgs &a, hipStream_t st) {
  using G = Geom7<P, R, NC, NP, BK>;
  static_assert(G::lds_bytes() <= 160 * 1024, "LDS budget");
  const size_t lds = G::lds_bytes();
  {
    // the LDS attribute is per device; one bit per device, set from any thread
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = gdmk_set_lds_attr((const void *)stencil7_kernel<P, R, NC, NP, BK, CH>, lds, attr_mask);
    if (e != hipSuccess) return e;
  }
  dim3 grid((a.Nx + G::TX - 1) / G::TX, (a.out_y1 - a.out_y0 + G::TY - 1) / G::TY,
            (a.out_z1 - a.out_z0 + a.zchunk - 1) / a.zchunk);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  hipLaunchKernelGGL((stencil7_kernel<P, R, NC, NP, BK, CH>), grid, dim3(G::NT), lds, st, a);
  return hipGetLastError();
}

template <int P, int R, int NC, int NP>
static hipError_t launch7_p(int bk, const StencilArgs &a, hipStream_t st) {
  // 16-B LDS-DMA chunks need every staged row to start 16-B aligned
  const bool vec = (a.Nx % 2 == 0) && ((reinterpret_cast<uintptr_t>(a.src) & 15) == 0);
  switch (bk) {
    case 0: return vec ? launch7_t<P, R, NC, NP, 0, 16>(a, st) : launch7_t<P, R, NC, NP, 0, 4>(a, st);
    case 1: return vec ? launch7_t<P, R, NC, NP, 1, 16>(a, st) : launch7_t<P, R, NC, NP, 1, 4>(a, st);
    case 2: return vec ? launch7_t<P, R, NC, NP, 2, 16>(a, st) : launch7_t<P, R, NC, NP, 2, 4>(a, st);
    default: return hipErrorInvalidValue;
  }
}

// what the caller asks of a launch's tail (gdmk_launch_stencil8)
struct TailReq {
  const FaceArgs *faces;
  int n;
  unsigned long long *counter;
  bool *ran;
};

// the tail work of a launch: step 1 of the faces fa[0, nf) (cell form, each its
// own T); items = 0 when nf = 0 or a face cannot run in the tail
static StencilTail make_tail(const FaceArgs *fa, int nf, int p, unsigned long long *counter, size_t lds_avail) {
  StencilTail tl{};
  if (nf <= 0 || nf > BcStage::kMaxFaces || !counter) return tl;
  // rows per item: as many as the launch's LDS holds (the rows form keeps
  // them all), at most 4
  size_t q0max = 1;
  for (int i = 0; i < nf; ++i) q0max = std::max(q0max, (size_t)std::max(fa[i].Q0, 1));
  const size_t phi = sizeof(double) * (size_t)((p * (p + 1) * (p + 1) + 1) & ~1);
  if (lds_avail <= phi) return tl;
  tl.s1.rpb = (int)std::min<size_t>(4, (lds_avail - phi) / (sizeof(double) * q0max));
  if (tl.s1.rpb < 1) return StencilTail{};
  int items = 0;
  for (int i = 0; i < nf; ++i) {
    const FaceArgs &f = fa[i];
    const size_t need = sizeof(double) * ((size_t)f.p * (f.p + 1) * (f.p + 1) + (size_t)tl.s1.rpb * f.Q0);
    if (!f.phi0 || f.p != p || !f.T || f.Q1 <= 0 || f.i0_end <= f.i0_begin || need > lds_avail) return StencilTail{};
    tl.s1.f[i] = Step1Face<BcArr>{BcArr{f.U, f.Q0}, f.Q0, f.Q1, f.i0_begin, f.i0_end - f.i0_begin, f.crange0, f.phi0,
                                  f.ncell0_total, f.cell0_begin, f.T};
    tl.first[i] = items;
    items += (f.Q1 + tl.s1.rpb - 1) / tl.s1.rpb;
  }
  tl.first[nf] = items;
  tl.nfaces = nf;
  tl.items = items;
  tl.counter = counter;
  return tl;
}

template <int P, int R, int NC, int NP, int BK, int CH, int PF>
static hipError_t launch8_t(const StencilArgs &a, const TailReq &tr, hipStream_t st) {
  using G = Geom8<P, R, NC, NP, BK>;
  static_assert(G::lds_bytes() <= 160 * 1024, "LDS budget");
  const size_t lds = G::lds_bytes();
  {
    // the LDS attribute is per device; one bit per device, set from any thread
    static std::atomic<uint64_t> attr_mask{0};
    hipError_t e = gdmk_set_lds_attr((const void *)stencil8_kernel<P, R, NC, NP, BK, CH, PF>, lds, attr_mask);
    if (e != hipSuccess) return e;
  }
  int nz = 0;
  for (int r = 0; r < 2; ++r)
    if (a.cz1[r] > a.cz0[r]) nz += (a.cz1[r] - a.cz0[r] + a.zchunk - 1) / a.zchunk;
  dim3 grid((a.Nx + G::TX - 1) / G::TX, (a.out_y1 - a.out_y0 + G::TY - 1) / G::TY, nz);
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return hipSuccess;
  const StencilTail tail = make_tail(tr.faces, tr.n, P, tr.counter, lds);
  hipLaunchKernelGGL((stencil8_kernel<P, R, NC, NP, BK, CH, PF>), grid, dim3(G::NT), lds, st, a, tail);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && tail.items > 0) *tr.ran = true;
  return e;
}

template <int P, int R, int NC, int NP, int PF>
static hipError_t launch8_p(int bk, const StencilArgs &a, const TailReq &tail, hipStream_t st) {
  const bool vec = (a.Nx % 2 == 0) && ((reinterpret_cast<uintptr_t>(a.src) & 15) == 0);
  switch (bk) {
    case 0:
      return vec ? launch8_t<P, R, NC, NP, 0, 16, PF>(a, tail, st) : launch8_t<P, R, NC, NP, 0, 4, PF>(a, tail, st);
    case 1:
      return vec ? launch8_t<P, R, NC, NP, 1, 16, PF>(a, tail, st) : launch8_t<P, R, NC, NP, 1, 4, PF>(a, tail, st);
    case 2:
      return vec ? launch8_t<P, R, NC, NP, 2, 16, PF>(a, tail, st) : launch8_t<P, R, NC, NP, 2, 4, PF>(a, tail, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_stencil8(int p, int bk, const gdmk::StencilArgs &a, const gdmk::FaceArgs *tail_faces,
                                           int n_tail, unsigned long long *counter, bool *tail_ran,
                                           hipStream_t st) {
  using namespace gdmk;
  *tail_ran = false;
  const TailReq tail{tail_faces, n_tail, counter, tail_ran};
  hipError_t e = hipErrorInvalidValue;
  switch (p) {
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 1
    case 1: e = launch8_p<1, 4, 8, 8, 3>(bk, a, tail, st); break;
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 3
    case 3: e = launch8_p<3, 4, 8, 8, 3>(bk, a, tail, st); break;
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 5
    case 5: e = launch8_p<5, GDM_R5, GDM_NC5, GDM_NP5, GDM_PF5>(bk, a, tail, st); break;
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 7
    case 7: e = launch8_p<7, GDM_R7, GDM_NC7, GDM_NP7, GDM_PF7>(bk, a, tail, st); break;
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 9
    case 9: e = launch8_p<9, 2, 8, 8, 3>(bk, a, tail, st); break;
#endif
    default: break;
  }
  return e;
}

// <P, R, NC, NP>: R output rows per consumer wave, NC consumer and NP producer
// waves -> tile 64 x (R NC)
extern "C" int gdmk_stencil_tile_rows(int p) {
  using namespace gdmk;
  return p < 5 ? 32 : (p == 5 ? Geom8<5, GDM_R5, GDM_NC5, GDM_NP5, 1>::TY : (p == 7 ? Geom8<7, GDM_R7, GDM_NC7, GDM_NP7, 1>::TY : 16));
}

extern "C" void gdmk_stencil8_geom(int p, int *tile_rows, int *wgs_per_cu) {
  using namespace gdmk;
  switch (p) {
    case 5:
      *tile_rows = Geom8<5, GDM_R5, GDM_NC5, GDM_NP5, 1>::TY;
      *wgs_per_cu = Geom8<5, GDM_R5, GDM_NC5, GDM_NP5, 1>::WGS;
      return;
    case 7:
      *tile_rows = Geom8<7, GDM_R7, GDM_NC7, GDM_NP7, 1>::TY;
      *wgs_per_cu = Geom8<7, GDM_R7, GDM_NC7, GDM_NP7, 1>::WGS;
      return;
    case 9: *tile_rows = 16; *wgs_per_cu = 1; return;
    default: *tile_rows = 32; *wgs_per_cu = 1; return;
  }
}

extern "C" hipError_t gdmk_launch_stencil(int p, int bk, const gdmk::StencilArgs &a, hipStream_t st) {
  using namespace gdmk;
  switch (p) {
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 1
    case 1: return launch7_p<1, 4, 8, 8>(bk, a, st);
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 3
    case 3: return launch7_p<3, 4, 8, 8>(bk, a, st);
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 5
    case 5: return launch7_p<5, 4, 8, 8>(bk, a, st);
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 7
    case 7: return launch7_p<7, 2, 8, 8>(bk, a, st);
#endif
#if !defined(GDM_ONLY_P) || GDM_ONLY_P == 9
    case 9: return launch7_p<9, 2, 8, 8>(bk, a, st);
#endif
    
    default: return hipErrorInvalidValue;
  }
}

extern "C" hipError_t gdmk_launch_chol_lines(int p, double *v, int len, int64_t stride, int64_t n_lines, int64_t A,
                                             int64_t B, int64_t C, const double *lrow, const double *inv_diag,
                                             hipStream_t st) {
  using namespace gdmk;
  if (n_lines <= 0) return hipSuccess;
  dim3 grid((unsigned)((n_lines + 255) / 256)), block(256);
  switch (p) {
    case 1: hipLaunchKernelGGL(chol_lines_kernel<1>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 3: hipLaunchKernelGGL(chol_lines_kernel<3>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 5: hipLaunchKernelGGL(chol_lines_kernel<5>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 7: hipLaunchKernelGGL(chol_lines_kernel<7>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    case 9: hipLaunchKernelGGL(chol_lines_kernel<9>, grid, block, 0, st, v, len, stride, n_lines, A, B, C, lrow, inv_diag); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <class Src, class Step2>
static hipError_t face_launch(const gdmk::FaceArgs &f, const Src &U, hipStream_t st, Step2 &step2) {
  using namespace gdmk;
  const int n0 = f.i0_end - f.i0_begin;
  const size_t cell_lds = sizeof(double) * ((size_t)f.p * (f.p + 1) * (f.p + 1) + (size_t)f.Q0);
  if (f.phi0 && cell_lds <= 48 * 1024) {
    // cell form of step 1, then the usual step 2
    const int rpb = 4;
    dim3 g1c((f.Q1 + rpb - 1) / rpb);
    if (f.phase != 2) switch (f.p) {
#define GDM_FACE_CELL(PP)                                                                                            \
  case PP:                                                                                                         \
    hipLaunchKernelGGL((face_cell_step1_kernel<PP, Src>), g1c, dim3(512), cell_lds, st, U, f.Q0, f.Q1, rpb, f.i0_begin, \
                       n0, f.crange0, f.phi0, f.ncell0_total, f.cell0_begin, f.T);                                 \
    break;
      GDM_FACE_CELL(1) GDM_FACE_CELL(3) GDM_FACE_CELL(5) GDM_FACE_CELL(7) GDM_FACE_CELL(9)
#undef GDM_FACE_CELL
      default: return hipErrorInvalidValue;
    }
    dim3 g2((n0 + 255) / 256, f.i1_end - f.i1_begin);
    if (f.phase != 1) step2(g2);
    return hipGetLastError();
  }
  // rows per workgroup: as many as fit 48 KiB of LDS (up to 4)
  const size_t row_bytes = sizeof(double) * (size_t)f.qmax0;
  const int rows = row_bytes * 4 <= 48 * 1024 ? 4 : (row_bytes * 2 <= 48 * 1024 ? 2 : 1);
  if (row_bytes > 48 * 1024) return hipErrorInvalidValue;  // <= (FACE_CHUNK + 2p) (p + 1) doubles in practice
  dim3 g1((n0 + FACE_CHUNK - 1) / FACE_CHUNK, (f.Q1 + rows - 1) / rows);
  const size_t lds = row_bytes * rows;
  if (f.phase == 2)
    ;
  else if (rows == 4)
    hipLaunchKernelGGL((face_step1_kernel<4, Src>), g1, dim3(FACE_CHUNK), lds, st, U, f.Q0, f.Q1, f.i0_begin, n0, f.qs0,
                       f.w0T, f.wmax0, f.ldw0, f.qmax0, f.T);
  else if (rows == 2)
    hipLaunchKernelGGL((face_step1_kernel<2, Src>), g1, dim3(FACE_CHUNK), lds, st, U, f.Q0, f.Q1, f.i0_begin, n0, f.qs0,
                       f.w0T, f.wmax0, f.ldw0, f.qmax0, f.T);
  else
    hipLaunchKernelGGL((face_step1_kernel<1, Src>), g1, dim3(FACE_CHUNK), lds, st, U, f.Q0, f.Q1, f.i0_begin, n0, f.qs0,
                       f.w0T, f.wmax0, f.ldw0, f.qmax0, f.T);
  dim3 g2((n0 + 255) / 256, f.i1_end - f.i1_begin);
  if (f.phase != 1) step2(g2);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_face(const gdmk::FaceArgs &f, hipStream_t st) {
  using namespace gdmk;
  const int n0 = f.i0_end - f.i0_begin;
  if (n0 <= 0 || f.Q1 <= 0 || f.i1_end <= f.i1_begin) return hipSuccess;
  if (f.phase < 0 || f.phase > 2) return hipErrorInvalidValue;
  auto step2 = [&](dim3 g2) {
    hipLaunchKernelGGL(face_step2_kernel, g2, dim3(256), 0, st, f.T, n0, f.i1_begin, f.i1_end, f.qs1, f.qc1, f.w1,
                       f.wmax1, f.dst, f.base, f.stride0, f.stride1, f.scale);
  };
  return face_launch(f, BcArr{f.U, f.Q0}, st, step2);
}

// step 1 (cell form) of n inflow faces in one launch (each face its own T)
extern "C" hipError_t gdmk_launch_faces_step1(const gdmk::FaceArgs *fa, int n, hipStream_t st) {
  using namespace gdmk;
  if (n <= 0) return hipSuccess;
  if (n > BcStage::kMaxFaces) return hipErrorNotSupported;
  Step1Set<BcArr> s1{};
  s1.rpb = 4;
  size_t lds = 0;
  int g1 = 0;
  for (int i = 0; i < n; ++i) {
    const FaceArgs &f = fa[i];
    const size_t cell_lds = sizeof(double) * ((size_t)f.p * (f.p + 1) * (f.p + 1) + (size_t)f.Q0);
    if (!f.phi0 || cell_lds > 48 * 1024 || !f.T || f.p != fa[0].p || f.Q1 <= 0 || f.i0_end <= f.i0_begin)
      return hipErrorNotSupported;
    for (int j = 0; j < i; ++j)
      if (fa[j].T == f.T) return hipErrorNotSupported;  // faces must not share T
    s1.f[i] = Step1Face<BcArr>{BcArr{f.U, f.Q0}, f.Q0, f.Q1, f.i0_begin, f.i0_end - f.i0_begin, f.crange0, f.phi0,
                               f.ncell0_total, f.cell0_begin, f.T};
    lds = std::max(lds, cell_lds);
    g1 = std::max(g1, (f.Q1 + s1.rpb - 1) / s1.rpb);
  }
  switch (fa[0].p) {
#define GDM_FACES_S1(PP)                                                                                       \
  case PP:                                                                                                   \
    hipLaunchKernelGGL((face_cell_step1_multi_kernel<PP, BcArr>), dim3(g1, n), dim3(512), lds, st, s1); \
    break;
    GDM_FACES_S1(1) GDM_FACES_S1(3) GDM_FACES_S1(5) GDM_FACES_S1(7) GDM_FACES_S1(9)
#undef GDM_FACES_S1
    default: return hipErrorNotSupported;
  }
  return hipGetLastError();
}

// step 2 of n inflow faces (their T from gdmk_launch_faces_step1) with the
// ordered adds into dst, one launch (face_step2_add_kernel)
extern "C" hipError_t gdmk_launch_faces_step2_add(const gdmk::FaceArgs *fa, const gdmk::FaceAddFace *fg, int n,
                                                  int64_t N0, int64_t N1, int64_t own_off, double *dst,
                                                  hipStream_t st) {
  using namespace gdmk;
  // rows per thread: 1 / 2 / 4 / 8 measured 41.5 / 37.0 / 45.6 / 74.9 us at C3
  // (three 512^2 faces, profiles/r5_experiments/face_step2_rows.txt)
  constexpr int kRows = 2;
  if (n <= 0) return hipSuccess;
  if (n > BcStage::kMaxFaces || N0 <= 0 || N1 <= 0) return hipErrorNotSupported;
  Step2AddSet set{};
  set.n = n;
  set.N0 = N0;
  set.N1 = N1;
  set.own_off = own_off;
  int gx = 0, gy = 0;
  for (int i = 0; i < n; ++i) {
    const FaceArgs &f = fa[i];
    const int n0 = f.i0_end - f.i0_begin;
    if (!f.T || fg[i].e0 - fg[i].b0 != n0 || fg[i].e1 - fg[i].b1 != f.i1_end - f.i1_begin) return hipErrorNotSupported;
    set.f[i] = Step2Face{f.T, n0, f.i1_begin, f.i1_end, f.qs1, f.qc1, f.w1, f.wmax1, f.scale};
    set.g[i] = fg[i];
    gx = std::max(gx, (n0 + 63) / 64);
    gy = std::max(gy, (f.i1_end - f.i1_begin + kRows - 1) / kRows);
  }
  if (gx <= 0 || gy <= 0) return hipSuccess;
  hipLaunchKernelGGL(face_step2_add_kernel<kRows>, dim3(gx, gy, n), dim3(64), 0, st, set, dst);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_axpby(int64_t n, double a, const double *x, double b, double *y, hipStream_t st) {
  using namespace gdmk;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n / 2 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, a, x, b, y);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_dot(int64_t n, const double *x, const double *y, double *partial, int n_partial,
                                     double *out, hipStream_t st) {
  using namespace gdmk;
  hipLaunchKernelGGL(dot_partial_kernel, dim3(n_partial), dim3(256), 0, st, n, x, y, partial);
  hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(256), 0, st, n_partial, partial, out);
  return hipGetLastError();
}

extern "C" hipError_t gdmk_launch_zero(int64_t n, double *y, hipStream_t st) {
  using namespace gdmk;
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, y);
  return hipGetLastError();
}
