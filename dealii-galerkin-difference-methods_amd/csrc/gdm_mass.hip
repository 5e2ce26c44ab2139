// gdm_mass.hip -- exact Kronecker mass inverse, v2 (replaces the CG + ILU/AMG
// solve of applications/advection/include/gdm/advection/problem.h:236-267 and
// applications/wave/include/gdm/wave/problem.h:471-502 on the uncut mesh).
//
// M^-1 = M_z^-1 (x) M_y^-1 (x) M_x^-1 is applied as three passes of batched
// banded-Cholesky line solves (M_d = L L^T, half-bandwidth p):
//   forward  w_i = (r_i - sum_k L(i, i-p+k) w_{i-p+k}) / L(i, i)
//   backward x_i = (w_i - sum_m L(i+m, i) x_{i+m}) / L(i, i)
//
// Strided lines (y, z): lane = one line, consecutive lanes = consecutive x, so
// every load / store instruction moves one contiguous 512-B row; the values
// of a line are fetched U positions ahead of the recurrence (register
// double-buffer), so the dependent FMA chain never waits on HBM latency.
//
// Contiguous lines (x): one wave owns 64 lines and walks them in chunks of U
// positions; a chunk (64 lines x U doubles) is loaded row-coalesced into LDS,
// each lane runs the recurrence over its line's U values in LDS, and the
// chunk is written back row-coalesced.  The next chunk's loads are issued
// before the current chunk is processed.
//
// The first pass reads the right-hand side and writes the result vector (no
// separate copy); the forward sweep stores w into the result, the backward
// sweep reads it back right away (mostly from L2 / the memory-side cache).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "gdm_kernels.h"

namespace gdmk {

#define GDM_WAIT_VMCNT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory")
// wave-uniform coefficient reads through the constant address space (scalar loads)
typedef __attribute__((address_space(4))) const double cdouble;
__device__ __forceinline__ cdouble *cptr(const double *p) { return (cdouble *)(p); }
typedef double dpair __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) dpair ldouble2;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

namespace {

// factor rows: lrow[i * (P + 1) + k] = L(i, i - P + k), k = P is the diagonal;
// rows >= len are zero (backward sweep reads P rows past the end)
template <int P>
struct Chol {
  const double *__restrict__ lrow;
  const double *__restrict__ invd;
  __device__ __forceinline__ double fwd(int i, const double (&win)[P > 0 ? P : 1], double r) const {
    const double *L = lrow + (size_t)i * (P + 1);
    double s = r;
#pragma unroll
    for (int k = 0; k < P; ++k) s = fma(-L[k], win[k], s);
    return s * invd[i];
  }
  __device__ __forceinline__ double bwd(int i, const double (&win)[P > 0 ? P : 1], double w) const {
    double s = w;
#pragma unroll
    for (int m = 1; m <= P; ++m) s = fma(-lrow[(size_t)(i + m) * (P + 1) + (P - m)], win[m - 1], s);
    return s * invd[i];
  }
};

template <int P>
__device__ __forceinline__ void push_fwd(double (&win)[P], double s) {
#pragma unroll
  for (int k = 0; k < P - 1; ++k) win[k] = win[k + 1];
  win[P - 1] = s;
}
template <int P>
__device__ __forceinline__ void push_bwd(double (&win)[P], double s) {
#pragma unroll
  for (int m = P - 1; m > 0; --m) win[m] = win[m - 1];
  win[0] = s;
}

}  // namespace

// line l -> base = (l / A) * B + (l % A); consecutive l are consecutive addresses
template <int P, int U>
__global__ void __launch_bounds__(64) chol_strided_kernel(const double *src, double *dst, int len,
                                                          int64_t stride, int64_t n_lines, int64_t A, int64_t B,
                                                          const double *__restrict__ lrow,
                                                          const double *__restrict__ invd) {
  const Chol<P> ch{lrow, invd};
  for (int64_t l = (int64_t)blockIdx.x * 64 + threadIdx.x - threadIdx.x % 64; l < n_lines;
       l += (int64_t)gridDim.x * 64) {
    const int64_t line = l + threadIdx.x % 64;
    const bool on = line < n_lines;
    const int64_t base = on ? (line / A) * B + (line % A) : 0;
    double win[P];
    double cur[U], nxt[U];
    // ---- forward: src -> dst (w) ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = (on && u < len) ? src[base + (int64_t)u * stride] : 0.0;
    for (int i0 = 0; i0 < len; i0 += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + U + u;
        nxt[u] = (on && i < len) ? src[base + (int64_t)i * stride] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u;
        if (i < len) {
          const double s = ch.fwd(i, win, cur[u]);
          push_fwd<P>(win, s);
          if (on) dst[base + (int64_t)i * stride] = s;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
    // ---- backward: dst (w) -> dst (x) ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
    const int last = len - 1;
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = (on && last - u >= 0) ? dst[base + (int64_t)(last - u) * stride] : 0.0;
    for (int i0 = last; i0 >= 0; i0 -= U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 - U - u;
        nxt[u] = (on && i >= 0) ? dst[base + (int64_t)i * stride] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 - u;
        if (i >= 0) {
          const double s = ch.bwd(i, win, cur[u]);
          push_bwd<P>(win, s);
          if (on) dst[base + (int64_t)i * stride] = s;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
  }
}

// contiguous lines of length len: line l starts at l * len.  One wave per
// workgroup; chunk = 64 lines x U positions staged in LDS (row pitch U + 2).
template <int P, int U>
__global__ void __launch_bounds__(64) chol_rows_kernel(const double *src, double *dst, int len, int64_t n_lines,
                                                       int vec_ok, const double *__restrict__ lrow,
                                                       const double *__restrict__ invd) {
  static_assert(U % 2 == 0 && (64 * U / 2) % 64 == 0, "chunk geometry");
  constexpr int PITCH = U + 2;      // doubles; keeps 16-B alignment, spreads banks
  constexpr int NV = 64 * U / 2 / 64;  // 16-B vectors per lane per chunk
  __shared__ __attribute__((aligned(16))) double tile[64 * PITCH];
  const Chol<P> ch{lrow, invd};
  const int lane = threadIdx.x;  // vec_ok: every row start is 16-B aligned (host-checked)
  for (int64_t l0 = (int64_t)blockIdx.x * 64; l0 < n_lines; l0 += (int64_t)gridDim.x * 64) {
    const int nl = (int)min<int64_t>(64, n_lines - l0);
    // element e of a chunk: line e / (U/2), vector (e % (U/2)) -> positions 2v, 2v+1
    auto load_chunk = [&](const double *from, int i0, double2 (&r)[NV]) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int e = q * 64 + lane, ln = e / (U / 2), v = e % (U / 2);
        const int i = i0 + 2 * v;
        double2 val = make_double2(0.0, 0.0);
        if (ln < nl && i >= 0 && i < len) {
          const double *p = from + (l0 + ln) * (int64_t)len + i;
          if (vec_ok && i + 1 < len)
            val = *reinterpret_cast<const double2 *>(p);
          else {
            val.x = p[0];
            val.y = i + 1 < len ? p[1] : 0.0;
          }
        }
        r[q] = val;
      }
    };
    auto put_lds = [&](const double2 (&r)[NV]) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int e = q * 64 + lane, ln = e / (U / 2), v = e % (U / 2);
        *reinterpret_cast<double2 *>(&tile[ln * PITCH + 2 * v]) = r[q];
      }
    };
    auto store_chunk = [&](int i0) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int e = q * 64 + lane, ln = e / (U / 2), v = e % (U / 2);
        const int i = i0 + 2 * v;
        if (ln < nl && i >= 0 && i < len) {
          const double2 val = *reinterpret_cast<const double2 *>(&tile[ln * PITCH + 2 * v]);
          double *p = dst + (l0 + ln) * (int64_t)len + i;
          if (vec_ok && i + 1 < len)
            *reinterpret_cast<double2 *>(p) = val;
          else {
            p[0] = val.x;
            if (i + 1 < len) p[1] = val.y;
          }
        }
      }
    };
    double win[P];
    double2 cur[NV], nxt[NV];
    // ---- forward: chunks [i0, i0 + U) ascending ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
    load_chunk(src, 0, cur);
    for (int i0 = 0; i0 < len; i0 += U) {
      load_chunk(src, i0 + U, nxt);
      __syncthreads();  // previous chunk's stores have read the tile
      put_lds(cur);
      __syncthreads();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u;
        if (i < len) {
          const double s = ch.fwd(i, win, tile[lane * PITCH + u]);
          push_fwd<P>(win, s);
          tile[lane * PITCH + u] = s;
        }
      }
      __syncthreads();
      store_chunk(i0);
#pragma unroll
      for (int q = 0; q < NV; ++q) cur[q] = nxt[q];
    }
    // ---- backward: chunks [i0, i0 + U) descending ----
#pragma unroll
    for (int k = 0; k < P; ++k) win[k] = 0.0;
    const int c_last = ((len - 1) / U) * U;
    __syncthreads();
    load_chunk(dst, c_last, cur);
    for (int i0 = c_last; i0 >= 0; i0 -= U) {
      load_chunk(dst, i0 - U, nxt);
      __syncthreads();
      put_lds(cur);
      __syncthreads();
#pragma unroll
      for (int u = U - 1; u >= 0; --u) {
        const int i = i0 + u;
        if (i < len) {
          const double s = ch.bwd(i, win, tile[lane * PITCH + u]);
          push_bwd<P>(win, s);
          tile[lane * PITCH + u] = s;
        }
      }
      __syncthreads();
      store_chunk(i0);
#pragma unroll
      for (int q = 0; q < NV; ++q) cur[q] = nxt[q];
    }
    __syncthreads();
  }
}

// ===========================================================================
// v3: single-sweep line solves, 16 B/DoF per direction.
//
// The forward factor L^-1 and the backward factor L^-T are stable recurrences
// whose homogeneous solutions decay below 1e-16 (relative) within C positions
// (the impulse response of the p = 5 GDM mass factor drops below 1e-17 after
// 50 positions, p = 7 after 57).  A line is therefore marched
// ONCE: the forward values of two consecutive chunks live in a register ring
// (2 x C doubles, compile-time indices), and as soon as chunk c is
// forward-solved, chunk c-1 is back-solved, the backward recurrence starting
// from a zero state at the end of chunk c (a warm-up over chunk c whose values
// are not kept): its initial-state error has decayed below 1e-16 by the time
// it reaches chunk c-1.  The last chunk of a line is back-solved from the true
// (zero) end state.  Every value is read once and written once.
//
// Coefficient tables (wave-uniform positions -> scalar loads), padded with zero
// rows past the line end so positions >= len produce exact zeros, prescaled by
// the inverse diagonal so each position's dependence on its predecessor is a
// single FMA:
//   lrow[i][k] = L(i, i - P + k) / L(i, i), k < P;  urow[i][m - 1] = L(i + m, i) / L(i, i);
//   invd[i] = 1 / L(i, i)
// The Cholesky rows reach a fixed point a few dozen rows into the line and keep
// it until the last p rows; chunks inside that range take the coefficients
// from kernel arguments (SGPRs) instead.
template <int P>
struct Cst3 {
  double l[P], u[P], d;
  int row_lo, row_hi;  // rows [row_lo, row_hi) of lrow / invd, [row_lo, row_hi - P) of urow equal l, d, u
};

template <int P>
struct Geo3 {
  static constexpr int C = P <= 5 ? 48 : 56;  // chunk = warm-up length
  // strided: loads in flight per lane.  One chunk ahead: with the 2C-double
  // ring this runs one wave per SIMD, so the FIFO alone must cover the HBM
  // latency (Q * 512 B per wave; a 16-deep FIFO measured as latency-bound)
  // with the stores streamed between the loads (Ring3::fwd ST), load j waits
  // for vmcnt <= ~2 Q: Q = C / 2 <= 31 keeps that within the 6-bit counter
  static constexpr int Q = P <= 5 ? C / 2 : C / 4;  // p = 7: C / 2 spills to scratch
  static constexpr int QL = 4;                // rows: LDS pair reads ahead
  static constexpr int UPR = (C + 2) / 2;     // rows: 16-B units per LDS row (pitch C + 2 doubles)
  static constexpr int TILE = 64 * UPR;       // rows: units per tile (= 64 x DMA instructions)
  static constexpr size_t lds_bytes() { return 2 * (size_t)TILE * 16; }
  static_assert(C % Q == 0 && C % 4 == 0, "chunk geometry");
};

// cache policy of the v3 kernels' global accesses (buffer aux bits on gfx950:
// 2 = nt): the line data stream through once per pass, so loads and stores are
// non-temporal.  A/B on the MI355X (profiles/r3v, mass solve): C3 1.515 ->
// 1.425 ms, C4 0.323 -> 0.249 ms, C2 0.0378 -> 0.0356 ms; stores alone gave
// -2 % / -1 % / -7 %, loads alone nothing
#ifndef GDM_MASS_LD_CPOL
#define GDM_MASS_LD_CPOL 2
#endif
#ifndef GDM_MASS_ST_CPOL
#define GDM_MASS_ST_CPOL 2
#endif
// line-end chunks take their table rows for the whole chunk (a per-group
// table / interior-row decision measured slower: SGPR spills, round 2)
#define GDM_MASS_EDGE_MODE 1

// passes with fewer waves of lines than this split their lines into segments:
// one wave per SIMD (1024 on the chip) is these kernels' occupancy.  512 ->
// 1024 moved the C3 rank's (512^2 x 64 planes) y and x passes, 512 waves each,
// to two segments: SPIKE solve 0.335 / 0.340 -> 0.304 / 0.314 ms (same box,
// gpurun_out r6f rank legs)
#ifndef GDM_MASS_SEG_WAVES
#define GDM_MASS_SEG_WAVES 1024
#endif

// compiler-only fence: the scheduler may not move instructions across it
#define GDM_FENCE()                    \
  do {                                 \
    asm volatile("" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

template <int P>
struct Ring3 {
  static constexpr int C = Geo3<P>::C;
  cdouble *L, *U, *D;
  const Cst3<P> &k;

  template <bool TAB>
  __device__ __forceinline__ double lco(int i, int q) const {
    if constexpr (TAB) return L[(size_t)i * P + q]; else return k.l[q];
  }
  template <bool TAB>
  __device__ __forceinline__ double uco(int i, int q) const {
    if constexpr (TAB) return U[(size_t)i * P + q]; else return k.u[q];
  }
  template <bool TAB>
  __device__ __forceinline__ double dco(int i) const {
    if constexpr (TAB) return D[i]; else return k.d;
  }
  // table mode: the row index of every group of 4 positions passes through an
  // opaque SGPR move, so the (invariant, scalar) coefficient loads cannot be
  // hoisted over the whole chunk (that spills hundreds of SGPRs)
  template <bool TAB>
  __device__ __forceinline__ int grp(int i) const {
    if constexpr (TAB) asm volatile("" : "+s"(i));
    return i;
  }
  // MODE 0: every row of the call is an interior (constant) row; 1: every row
  // from the tables; 2: decided per group of 4 positions (wave-uniform
  // branch), so only the groups that touch the ~p/2 + 30 special rows at the
  // line ends pay the table loads (a chunk-level decision ran 5 of 11 chunk
  // steps of a 512-line from the tables)
  __device__ __forceinline__ bool fwd_const(int i_lo, int i_hi) const { return i_lo >= k.row_lo && i_hi <= k.row_hi; }
  __device__ __forceinline__ bool bwd_const(int i_lo, int i_hi) const {
    return i_lo >= k.row_lo && i_hi <= k.row_hi - P;
  }

  // cur <- w of the chunk at base (b values from get(j), j chunk-local and
  // compile-time, increasing); prev = w of the previous chunk (zeros before
  // the line start)
  // ST: cur holds the final values of an earlier chunk that are stored (put,
  // ascending) just before the forward values overwrite them, so the stores
  // stream one per position between the loads instead of in a burst of C
  // (a burst of C stores on top of the load FIFO overflows the 6-bit vmcnt)
  template <int MODE, bool ST = false, class Get, class Put>
  __device__ __forceinline__ void fwd(double (&cur)[C], const double (&prev)[C], int base, Get &&get, Put &&put) const {
    int ib = base;
    bool tabg = MODE == 1;
    auto pos = [&](auto tab, int j) {
      constexpr bool T = decltype(tab)::value;
      const int i = ib + j;
      if constexpr (ST) put(cur[j]);
      double s = get(j) * dco<T>(i);
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const int jj = j - P + q;
        s = fma(-lco<T>(i, q), jj >= 0 ? cur[jj] : prev[C + jj], s);
      }
      cur[j] = s;
    };
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (j % 4 == 0) {
        GDM_FENCE();
        ib = grp<MODE != 0>(base + j) - j;
        if constexpr (MODE == 2) tabg = !fwd_const(base + j, base + j + 4);
      }
      if constexpr (MODE == 2) {
        if (tabg)
          pos(std::true_type{}, j);
        else
          pos(std::false_type{}, j);
      } else {
        pos(std::integral_constant<bool, MODE == 1>{}, j);
      }
    }
    GDM_FENCE();
  }
  // out: w on entry, x on exit (positions base .. base + C - 1).  WARM: start
  // the recurrence from zero at base + 2C - 1 and run it over `next` (the
  // following chunk's w, not modified); otherwise the state after the chunk is
  // zero (line end).
  template <bool WARM, int MODE, int WMODE = MODE>
  __device__ __forceinline__ void bwd(double (&out)[C], const double (&next)[C], int base) const {
    double t[P];  // x at positions base + C + q, slot q % P
#pragma unroll
    for (int q = 0; q < P; ++q) t[q] = 0.0;
    bool tabg = MODE == 1;
    if constexpr (WARM) {
      int ib = base + C;
      auto wpos = [&](auto tab, int q) {
        constexpr bool T = decltype(tab)::value;
        const int i = ib + q;
        double s = next[q] * dco<T>(i);
#pragma unroll
        for (int m = P; m >= 1; --m)
          if (q + m < C) s = fma(-uco<T>(i, m - 1), t[(q + m) % P], s);
        t[q % P] = s;
      };
#pragma unroll
      for (int q = C - 1; q >= 0; --q) {
        if ((C - 1 - q) % 4 == 0) {
          ib = grp<WMODE != 0>(base + C + q) - q;
          if constexpr (WMODE == 2) tabg = !bwd_const(base + C + q - 3, base + C + q + 1);
        }
        if constexpr (WMODE == 2) {
          if (tabg)
            wpos(std::true_type{}, q);
          else
            wpos(std::false_type{}, q);
        } else {
          wpos(std::integral_constant<bool, WMODE == 1>{}, q);
        }
      }
    }
    int ib = base;
    auto bpos = [&](auto tab, int j) {
      constexpr bool T = decltype(tab)::value;
      const int i = ib + j;
      double s = out[j] * dco<T>(i);
#pragma unroll
      for (int m = P; m >= 1; --m) {
        const int jj = j + m;
        s = fma(-uco<T>(i, m - 1), jj < C ? out[jj] : t[(jj - C) % P], s);
      }
      out[j] = s;
    };
#pragma unroll
    for (int j = C - 1; j >= 0; --j) {
      if ((C - 1 - j) % 4 == 0) {
        ib = grp<MODE != 0>(base + j) - j;
        if constexpr (MODE == 2) tabg = !bwd_const(base + j - 3, base + j + 1);
      }
      if constexpr (MODE == 2) {
        if (tabg)
          bpos(std::true_type{}, j);
        else
          bpos(std::false_type{}, j);
      } else {
        bpos(std::integral_constant<bool, MODE == 1>{}, j);
      }
    }
    GDM_FENCE();
  }
  // one march step: forward chunk c into cur, then back-solve chunk c - 1
  // (prev) with the warm-up over cur
  template <bool ST = false, class Get, class Put>
  __device__ __forceinline__ void step(double (&cur)[C], double (&prev)[C], int c, Get &&get, Put &&put) const {
    const int base = c * C;
    // forward rows [base, base + C); warm-up rows [base, base + C) with their
    // u rows; back-solved rows [base - C, base): each part takes the interior
    // row from kernel arguments when all its rows hold it
    if (fwd_const(base, base + C))
      fwd<0, ST>(cur, prev, base, get, put);
    else
      fwd<GDM_MASS_EDGE_MODE, ST>(cur, prev, base, get, put);
    const bool wc = bwd_const(base, base + C), mc = bwd_const(base - C, base);
    if (wc && mc)
      bwd<true, 0, 0>(prev, cur, base - C);
    else if (mc)
      bwd<true, 0, GDM_MASS_EDGE_MODE>(prev, cur, base - C);
    else if (wc)
      bwd<true, GDM_MASS_EDGE_MODE, 0>(prev, cur, base - C);
    else
      bwd<true, GDM_MASS_EDGE_MODE, GDM_MASS_EDGE_MODE>(prev, cur, base - C);
  }
};

// Strided lines: lane = line, line l -> base (l / A) * B + l % A, step stride
// (consecutive lanes = consecutive addresses: every load / store instruction
// moves one contiguous 512-B row segment).  The loads stream Q positions ahead
// of the forward recurrence through a register FIFO, across chunk borders.
// Requires ((len - 1) * stride + 64) * 8 < 2^31 bytes: the buffer resource's
// num_records is 0x7fffffff and the position offsets are 32-bit (checked by
// mass_solve_passes in gdm_capi.cpp, which runs the 64-bit-addressed v2
// kernel for larger spans).  src may equal dst.
template <int P, bool SEG>
__global__ void __launch_bounds__(64) mass3_strided_kernel(const double *src, double *dst, int len, int64_t stride,
                                                           int64_t n_lines, int64_t A, int64_t B,
                                                           const double *__restrict__ lrow,
                                                           const double *__restrict__ urow,
                                                           const double *__restrict__ invd, const Cst3<P> k,
                                                           int seg_chunks) {
  using R = Ring3<P>;
  constexpr int C = R::C, Q = Geo3<P>::Q;
  const R r{cptr(lrow), cptr(urow), cptr(invd), k};
  // lanes past n_lines repeat the last line (same values, same addresses)
  const int64_t line = min((int64_t)blockIdx.x * 64 + threadIdx.x, n_lines - 1);
  // wave-uniform base (lane 0's line) + a 32-bit lane byte offset; the
  // position offset is a running 32-bit SGPR (buffer soffset): one SALU per
  // access instead of a 64-bit multiply-add chain per position
  const int64_t b0 = (line / A) * B + (line % A);
  const int64_t bw = ((int64_t)__builtin_amdgcn_readfirstlane((int)(b0 >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b0);
  const uint32_t lbyte = (uint32_t)(b0 - bw) * 8u;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(src + bw), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void *)(dst + bw), 0, 0x7fffffff, 0x00020000);
  const uint32_t s8 = (uint32_t)(stride * 8), last = (uint32_t)(len - 1) * s8;
  // segment blockIdx.y: chunks [cb, ce) of the line (seg_chunks = 0: the whole
  // line); the march starts one chunk early at c0 = cb - 1 (a forward warm-up
  // from a zero state, forgotten within C positions like the backward one)
  const int n_chunks = (len + C - 1) / C;
  const int cb = SEG ? (int)blockIdx.y * seg_chunks : 0;
  const int ce = SEG ? min(n_chunks, cb + seg_chunks) : n_chunks;
  const int c0 = SEG && cb > 0 ? cb - 1 : 0;
  uint32_t lo = (uint32_t)(c0 * C) * s8, so = (uint32_t)(cb * C) * s8;  // byte offsets of the next load / store
  auto load = [&]() -> double {
    uint32_t o = min(lo, last);
    asm volatile("" : "+s"(o));
    lo += s8;
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, lbyte, o, GDM_MASS_LD_CPOL));
  };
  auto put = [&](double v) {
    uint32_t o = so;
    asm volatile("" : "+s"(o));
    so += s8;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rd, lbyte, o, GDM_MASS_ST_CPOL);
  };
  double fifo[Q];
  auto get = [&](int j) -> double {
    const double b = fifo[j % Q];
    fifo[j % Q] = load();
    return b;
  };
  auto store = [&](const double (&h)[C], int base) {
    if (base + C <= len) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (j % 8 == 0) GDM_FENCE();
        put(h[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < C; ++j)
        if (base + j < len) put(h[j]);
    }
    GDM_FENCE();
  };
  double h0[C], h1[C];
#pragma unroll
  for (int j = 0; j < C; ++j) h1[j] = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q) fifo[q] = load();
  auto none = [](double) {};
  // the final values of chunk c - 2 are stored by the forward sweep of chunk
  // c (fwd<.., true>), the last one or two chunks explicitly; the warm-up
  // chunk's (c0 < cb) are never stored
  if (SEG && r.fwd_const(c0 * C, c0 * C + C))
    r.template fwd<0>(h0, h1, c0 * C, get, none);
  else
    r.template fwd<GDM_MASS_EDGE_MODE>(h0, h1, c0 * C, get, none);
  for (int c = c0 + 1;; c += 2) {
    // ---- chunk c into h1, back-solve chunk c - 1 (h0) ----
    if (c * C >= len) {
      if (c - 2 >= cb) store(h1, (c - 2) * C);
      r.template bwd<false, GDM_MASS_EDGE_MODE>(h0, h1, (c - 1) * C);
      if (c - 1 >= cb) store(h0, (c - 1) * C);
      break;
    }
    if (c == c0 + 1 || c - 2 < cb)
      r.step(h1, h0, c, get, none);
    else
      r.template step<true>(h1, h0, c, get, put);
    if (SEG && c == ce) {  // the segment ends inside the line: chunk ce was the backward warm-up
      store(h0, (c - 1) * C);
      break;
    }
    // ---- chunk c + 1 into h0, back-solve chunk c (h1) ----
    if ((c + 1) * C >= len) {
      if (c - 1 >= cb) store(h0, (c - 1) * C);
      r.template bwd<false, GDM_MASS_EDGE_MODE>(h1, h0, c * C);
      store(h1, c * C);
      break;
    }
    if (c - 1 < cb)
      r.step(h0, h1, c + 1, get, none);
    else
      r.template step<true>(h0, h1, c + 1, get, put);
    if (SEG && c + 1 == ce) {
      store(h1, c * C);
      break;
    }
  }
}

// Contiguous lines (x): one wave owns 64 consecutive lines; chunk c of all 64
// lines (64 rows x C doubles) is staged by LDS-DMA (16 B per lane, the
// row-coalesced image of the rows, pitch C + 2 doubles: conflict-free
// ds_read_b128 of a lane's own row) one chunk ahead into tile c % 2; the
// back-solved chunk is written into the tile just consumed and stored
// row-coalesced.  Every lane issues every store (invalid lanes repeat a valid
// lane's store with the same data), so the counted vmcnt is exact.  (Three
// waves per CU fit the 2 x 25.6 KB of LDS; a one-tile variant with the next
// chunk staged in registers ran all four SIMDs but measured 2-9 % slower on
// the MI355X, profiles/r3i/ab_mass.txt.)
// Requires len even and 16-B aligned src / dst (host-checked).
// RKM (the RK stage update fused into the store, gdmk_launch_mass3_rk): 0 = store
// the solution into dst; 1 = acc_out = acc_in + beta k; 2 = also Y = y + alpha
// k; 3 = 2 with acc_in == y (the first RK stage: one load serves both, 8 B per
// DoF less).  acc_in / y of the chunk to be stored are loaded into registers
// before the chunk's arithmetic (their latency hides behind it); k never
// reaches memory.
template <int P, bool SEG, int RKM = 0>
__global__ void __launch_bounds__(64) mass3_rows_kernel(const double *src, double *dst, int len, int64_t n_lines,
                                                        const double *__restrict__ lrow,
                                                        const double *__restrict__ urow,
                                                        const double *__restrict__ invd, const Cst3<P> k,
                                                        int seg_chunks, const RkOut rk) {
  using R = Ring3<P>;
  using G = Geo3<P>;
  constexpr int C = R::C, UPR = G::UPR, QL = G::QL;
  static_assert(RKM == 0 || !SEG, "the fused RK update runs unsegmented");
  // stores in flight after the last load of an iteration (the loop-top wait)
  constexpr int NST = UPR * (RKM >= 2 ? 2 : 1);
  extern __shared__ __attribute__((aligned(16))) char smem3[];
  ldouble2 *tile0 = (ldouble2 *)smem3;
  ldouble2 *tile1 = tile0 + G::TILE;
  const R r{cptr(lrow), cptr(urow), cptr(invd), k};
  const int lane = threadIdx.x;
  const int64_t l0 = (int64_t)blockIdx.x * 64;
  const int nl = (int)min<int64_t>(64, n_lines - l0);
  __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void *)(src + l0 * len), 0, (int)((int64_t)nl * len * 8), 0x00020000);
  double *dbase = dst + l0 * len;

  // the lane index passes through an opaque VGPR move in the helpers below:
  // otherwise LICM keeps every per-instruction (row, pair) offset of the DMA
  // and the stores live across the march loop (~100 VGPRs)
  // The LDS row's pad pair (pair UPR - 1, positions base + C, base + C + 1) is
  // never read back, and positions past the line end (the last chunk) only
  // meet zero table coefficients: those lanes take an offset past the
  // resource's range (the load returns zeros without a memory request).
  // Fetching the pad pulled a 4th 128-B line into every 384-B chunk row: 1.31x
  // the x pass's algorithmic reads, 1.03x after it, 1.00x with the line end
  // (FETCH_SIZE, profiles/r6p)
  auto dma = [&](ldouble2 *t, int base) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int q = 0; q < UPR; ++q) {
      const int u = q * 64 + ln, row = u / UPR, pair = u - row * UPR;
      const uint32_t voff = (pair == UPR - 1 || base + 2 * pair >= len)
                                ? 0x7ffffff0u
                                : (uint32_t)(((int64_t)row * len + base + 2 * pair) * 8);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(t + q * 64), 16,
                                               voff, 0, 0, GDM_MASS_LD_CPOL);
    }
  };
  // b values of the lane's row, read QL pairs ahead from the tile
  dpair fl[QL];
  const ldouble2 *trow = tile0;
  auto get = [&](int j) -> double {
    const dpair v = fl[(j / 2) % QL];
    if (j % 2 == 1 && j / 2 + QL < C / 2) fl[(j / 2) % QL] = trow[j / 2 + QL];
    return j % 2 ? v.y : v.x;
  };
  auto open_row = [&](const ldouble2 *t) {
    trow = t + lane * UPR;
#pragma unroll
    for (int q = 0; q < QL; ++q) fl[q] = trow[q];
  };
  auto write_row = [&](ldouble2 *t, const double (&h)[C]) {
#pragma unroll
    for (int jp = 0; jp < C / 2; ++jp) {
      dpair v;
      v.x = h[2 * jp];
      v.y = h[2 * jp + 1];
      t[lane * UPR + jp] = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  // the RK operands of the chunk at `base` (RKM > 0), fetched one chunk of
  // arithmetic ahead of their use
  dpair pa[RKM ? UPR : 1], py[RKM >= 2 ? UPR : 1];
  const int64_t obase = l0 * len;
  auto prefetch = [&](int base) {
    if constexpr (RKM > 0) {
      const int last_pair = min(C / 2, (len - base) / 2) - 1;
      int ln = lane;
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int q = 0; q < UPR; ++q) {
        const int u = q * 64 + ln;
        const int row = min(u / UPR, nl - 1), pair = min(u % UPR, last_pair);
        const int64_t e = obase + (int64_t)row * len + base + 2 * pair;
        pa[q] = __builtin_nontemporal_load(reinterpret_cast<const dpair *>(rk.acc_in + e));
        if constexpr (RKM == 2) py[q] = __builtin_nontemporal_load(reinterpret_cast<const dpair *>(rk.y + e));
        if constexpr (RKM == 3) py[q] = pa[q];
      }
    }
  };
  auto store = [&](const ldouble2 *t, int base) {
    const int last_pair = min(C / 2, (len - base) / 2) - 1;  // >= 0: base < len, len even
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int q = 0; q < UPR; ++q) {
      if (q % 6 == 0) GDM_FENCE();
      const int u = q * 64 + ln;
      const int row = min(u / UPR, nl - 1), pair = min(u % UPR, last_pair);
      const dpair v = t[row * UPR + pair];
      if constexpr (RKM > 0) {
        // gdm_vec_rk_update (rk_update2_kernel): acc_in + beta k, y + alpha k, one FMA each
        const int64_t e = obase + (int64_t)row * len + base + 2 * pair;
        const dpair bv = {rk.beta, rk.beta};
        __builtin_nontemporal_store(__builtin_elementwise_fma(bv, v, pa[q]),
                                    reinterpret_cast<dpair *>(rk.acc_out + e));
        if constexpr (RKM >= 2) {
          const dpair av = {rk.alpha, rk.alpha};
          __builtin_nontemporal_store(__builtin_elementwise_fma(av, v, py[q]), reinterpret_cast<dpair *>(rk.Y + e));
        }
      } else {
#if GDM_MASS_ST_CPOL
        __builtin_nontemporal_store(v, reinterpret_cast<dpair *>(dbase + (int64_t)row * len + base + 2 * pair));
#else
        *reinterpret_cast<dpair *>(dbase + (int64_t)row * len + base + 2 * pair) = v;
#endif
      }
    }
    GDM_FENCE();
  };

  // segment blockIdx.y: chunks [cb, ce) (seg_chunks = 0: the whole line), the
  // march from c0 = cb - 1 (forward warm-up chunk, not stored) to ce (the
  // backward warm-up chunk when the segment ends inside the line)
  const int n_chunks = (len + C - 1) / C;
  const int cb = SEG ? (int)blockIdx.y * seg_chunks : 0;
  const int ce = SEG ? min(n_chunks, cb + seg_chunks) : n_chunks;
  const int c0 = SEG && cb > 0 ? cb - 1 : 0;
  double h0[C], h1[C];
#pragma unroll
  for (int j = 0; j < C; ++j) h1[j] = 0.0;
  dma(tile0, c0 * C);
  GDM_WAIT_VMCNT(0);
  if ((c0 + 1) * C < len) dma(tile1, (c0 + 1) * C);
  open_row(tile0);
  auto none = [](double) {};
  if (SEG && r.fwd_const(c0 * C, c0 * C + C))
    r.template fwd<0>(h0, h1, c0 * C, get, none);
  else
    r.template fwd<GDM_MASS_EDGE_MODE>(h0, h1, c0 * C, get, none);
  for (int c = c0 + 1;; c += 2) {
    // ---- chunk c: tile1, ring h1; chunk c - 1 in h0 (its input tile0 is free) ----
    if (c * C >= len) {
      if (c - 1 >= cb) prefetch((c - 1) * C);
      r.template bwd<false, GDM_MASS_EDGE_MODE>(h0, h1, (c - 1) * C);
      if (c - 1 >= cb) {
        write_row(tile0, h0);
        store(tile0, (c - 1) * C);
      }
      break;
    }
    if (c == c0 + 1 || c - 2 < cb)
      GDM_WAIT_VMCNT(0);  // only DMA(c) is in flight (no stores were issued after it)
    else
      GDM_WAIT_VMCNT(NST);  // DMA(c) retired (RKM: so did the loads after it); the stores may be in flight
    if ((c + 1) * C < len && (!SEG || c + 1 <= ce)) dma(tile0, (c + 1) * C);
    if (c - 1 >= cb) prefetch((c - 1) * C);
    open_row(tile1);
    r.step(h1, h0, c, get, none);
    if (c - 1 >= cb) {
      write_row(tile1, h0);
      store(tile1, (c - 1) * C);
    }
    if (SEG && c == ce) break;  // chunk ce was the backward warm-up
    // ---- chunk c + 1: tile0, ring h0; chunk c in h1 ----
    if ((c + 1) * C >= len) {
      prefetch(c * C);
      r.template bwd<false, GDM_MASS_EDGE_MODE>(h1, h0, c * C);
      write_row(tile1, h1);
      store(tile1, c * C);
      break;
    }
    if (c - 1 < cb)
      GDM_WAIT_VMCNT(0);
    else
      GDM_WAIT_VMCNT(NST);
    if ((c + 2) * C < len && (!SEG || c + 2 <= ce)) dma(tile1, (c + 2) * C);
    prefetch(c * C);
    open_row(tile0);
    r.step(h0, h1, c + 1, get, none);
    write_row(tile0, h1);
    store(tile0, c * C);
    if (SEG && c + 1 == ce) break;
  }
  GDM_WAIT_VMCNT(0);
}

namespace {

template <int P>
hipError_t launch_mass_lines_p(int dir_kind, const double *src, double *dst, int len, int64_t stride, int64_t n_lines,
                               int64_t A, int64_t B, const double *lrow, const double *invd, int max_wgs,
                               hipStream_t st) {
  const int64_t groups = (n_lines + 63) / 64;
  const unsigned grid = (unsigned)(max_wgs > 0 ? std::min<int64_t>(groups, max_wgs) : groups);
  const int vec = (len % 2 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(dst) & 15) == 0) ? 1 : 0;
  // x chunk width: 16 positions (one 128-B line per row; measured 1.15 vs 1.30 ms for 8 at 512^3)
  if (dir_kind == 0)
    hipLaunchKernelGGL((chol_rows_kernel<P, 16>), dim3(grid), dim3(64), 0, st, src, dst, len, n_lines, vec, lrow,
                       invd);
  else
    hipLaunchKernelGGL((chol_strided_kernel<P, 8>), dim3(grid), dim3(64), 0, st, src, dst, len, stride, n_lines, A,
                       B, lrow, invd);
  return hipGetLastError();
}

template <int P>
hipError_t launch_mass3_p(int dir_kind, const double *src, double *dst, int len, int64_t stride, int64_t n_lines,
                          int64_t A, int64_t B, const double *lrow, const double *urow, const double *invd,
                          const double *cst, int row_lo, int row_hi, int allow_segments, hipStream_t st) {
  Cst3<P> k;
  for (int q = 0; q < P; ++q) {
    k.l[q] = cst[q];
    k.u[q] = cst[P + q];
  }
  k.d = cst[2 * P];
  k.row_lo = row_lo;
  k.row_hi = row_hi;
  const unsigned grid = (unsigned)((n_lines + 63) / 64);
  // too few lines to give every SIMD a wave (C2: 16 waves of 64 lines): split
  // each line into segments of >= 1 chunk with forward and backward warm-ups
  // (one wave per SIMD is the occupancy of these kernels, 1024 on the chip).
  // Segments read their neighbours' input chunks: only out of place (src != dst)
  constexpr int C = Geo3<P>::C;
  const int n_chunks = (len + C - 1) / C;
  int seg_chunks = 0, n_segs = 1;
  if (allow_segments && src != dst && grid < GDM_MASS_SEG_WAVES && n_chunks >= 4) {
    const int want = (int)std::min<int64_t>(n_chunks, (1024 + grid - 1) / grid);
    seg_chunks = (n_chunks + want - 1) / want;
    n_segs = (n_chunks + seg_chunks - 1) / seg_chunks;
    if (n_segs < 2) seg_chunks = 0, n_segs = 1;
  }
  if (dir_kind == 0) {
    // <= 59 KB (p = 7): within the 64 KB default, no attribute needed
    constexpr size_t lds = Geo3<P>::lds_bytes();
    static_assert(lds <= 64 * 1024, "mass3_rows_kernel LDS above the default limit");
    if (seg_chunks)
      hipLaunchKernelGGL((mass3_rows_kernel<P, true>), dim3(grid, n_segs), dim3(64), lds, st, src, dst, len, n_lines,
                         lrow, urow, invd, k, seg_chunks, RkOut{});
    else
      hipLaunchKernelGGL((mass3_rows_kernel<P, false>), dim3(grid), dim3(64), lds, st, src, dst, len, n_lines, lrow,
                         urow, invd, k, 0, RkOut{});
  } else {
    if (seg_chunks)
      hipLaunchKernelGGL((mass3_strided_kernel<P, true>), dim3(grid, n_segs), dim3(64), 0, st, src, dst, len, stride,
                         n_lines, A, B, lrow, urow, invd, k, seg_chunks);
    else
      hipLaunchKernelGGL((mass3_strided_kernel<P, false>), dim3(grid), dim3(64), 0, st, src, dst, len, stride, n_lines,
                         A, B, lrow, urow, invd, k, 0);
  }
  return hipGetLastError();
}

template <int P>
hipError_t launch_mass3_rk_p(const double *src, int len, int64_t n_lines, const double *lrow, const double *urow,
                             const double *invd, const double *cst, int row_lo, int row_hi, const RkOut &rk,
                             hipStream_t st) {
  Cst3<P> k;
  for (int q = 0; q < P; ++q) {
    k.l[q] = cst[q];
    k.u[q] = cst[P + q];
  }
  k.d = cst[2 * P];
  k.row_lo = row_lo;
  k.row_hi = row_hi;
  const unsigned grid = (unsigned)((n_lines + 63) / 64);
  constexpr size_t lds = Geo3<P>::lds_bytes();
  if (rk.Y && rk.acc_in == rk.y)
    hipLaunchKernelGGL((mass3_rows_kernel<P, false, 3>), dim3(grid), dim3(64), lds, st, src, nullptr, len, n_lines,
                       lrow, urow, invd, k, 0, rk);
  else if (rk.Y)
    hipLaunchKernelGGL((mass3_rows_kernel<P, false, 2>), dim3(grid), dim3(64), lds, st, src, nullptr, len, n_lines,
                       lrow, urow, invd, k, 0, rk);
  else
    hipLaunchKernelGGL((mass3_rows_kernel<P, false, 1>), dim3(grid), dim3(64), lds, st, src, nullptr, len, n_lines,
                       lrow, urow, invd, k, 0, rk);
  return hipGetLastError();
}

}  // namespace

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_mass3_rk(int p, const double *src, int len, int64_t n_lines, const double *lrow,
                                          const double *urow, const double *invd, const double *cst, int row_lo,
                                          int row_hi, const gdmk::RkOut &rk, hipStream_t st) {
  using namespace gdmk;
  if (n_lines <= 0 || len <= 0) return hipSuccess;
  auto al16 = [](const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (len % 2 != 0 || !al16(src) || !al16(rk.acc_in) || !al16(rk.acc_out) || (rk.Y && (!al16(rk.y) || !al16(rk.Y))))
    return hipErrorNotSupported;
  switch (p) {
    case 3: return launch_mass3_rk_p<3>(src, len, n_lines, lrow, urow, invd, cst, row_lo, row_hi, rk, st);
    case 5: return launch_mass3_rk_p<5>(src, len, n_lines, lrow, urow, invd, cst, row_lo, row_hi, rk, st);
    case 7: return launch_mass3_rk_p<7>(src, len, n_lines, lrow, urow, invd, cst, row_lo, row_hi, rk, st);
    default: return hipErrorNotSupported;
  }
}

// v3 single-sweep line solves.  Tables: lrow [rows][p], urow [rows][p], invd
// [rows], rows >= len + 3 C + p with zero rows from len on; cst = the interior
// row (l[p], u[p], d) that rows [row_lo, row_hi) (urow: [row_lo, row_hi - p))
// hold exactly.
// dir_kind 0 (contiguous lines) requires len even and 16-B aligned src / dst.
extern "C" int gdmk_mass3_seg_waves() { return GDM_MASS_SEG_WAVES; }

extern "C" int gdmk_mass3_chunk(int p) {
  switch (p) {
    case 3: return gdmk::Geo3<3>::C;
    case 5: return gdmk::Geo3<5>::C;
    case 7: return gdmk::Geo3<7>::C;
    default: return 0;
  }
}
extern "C" hipError_t gdmk_launch_mass3(int p, int dir_kind, const double *src, double *dst, int len, int64_t stride,
                                       int64_t n_lines, int64_t A, int64_t B, const double *lrow, const double *urow,
                                       const double *invd, const double *cst, int row_lo, int row_hi,
                                       int allow_segments, hipStream_t st) {
  using namespace gdmk;
  if (n_lines <= 0 || len <= 0) return hipSuccess;
  switch (p) {
    case 3: return launch_mass3_p<3>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, urow, invd, cst, row_lo, row_hi, allow_segments, st);
    case 5: return launch_mass3_p<5>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, urow, invd, cst, row_lo, row_hi, allow_segments, st);
    case 7: return launch_mass3_p<7>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, urow, invd, cst, row_lo, row_hi, allow_segments, st);
    default: return hipErrorInvalidValue;
  }
}

// dir_kind 0: contiguous lines (line l at l * len, stride 1);
// dir_kind 1: strided lines, base = (l / A) * B + (l % A), step `stride`.
// src may equal dst.  max_wgs > 0 caps the grid (lines are walked grid-stride).
extern "C" hipError_t gdmk_launch_mass_lines(int p, int dir_kind, const double *src, double *dst, int len,
                                            int64_t stride, int64_t n_lines, int64_t A, int64_t B,
                                            const double *lrow, const double *inv_diag, int max_wgs,
                                            hipStream_t st) {
  using namespace gdmk;
  if (n_lines <= 0 || len <= 0) return hipSuccess;
  switch (p) {
    case 1: return launch_mass_lines_p<1>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 3: return launch_mass_lines_p<3>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 5: return launch_mass_lines_p<5>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 7: return launch_mass_lines_p<7>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    case 9: return launch_mass_lines_p<9>(dir_kind, src, dst, len, stride, n_lines, A, B, lrow, inv_diag, max_wgs, st);
    default: return hipErrorInvalidValue;
  }
}
