// gdm_kernels.h -- device-side argument blocks and launchers of gdm_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "gdm_rk.h"

namespace gdmk {

// Fused Kronecker stencil: out = B_x M_y M_z + M_x B_y M_z + M_x M_y B_z (or
// M_x M_y M_z for the mass operator) applied to the input box, written for
// the output box.  Arrays are [z - z0][y - y0][x] with full x extent.
//
// Interior x and y rows use the compile-time unit bands mhat, bhat of
// gdm_coeffs.h (bhat = chat for advection/convective, lhat for wave):
//   A' = M_x u / h_x = mhat*u,   B* = h_y B_x u = sx bhat*u,
//   D' = M_y A' / h_y,           E  = M_y B* / h_y + h_x B_y A' = mhat*B* + cy*A'
//   out(z') += M_z(z', z) E(z) + h_x h_y B_z(z', z) D'(z)   (mass: h_x h_y M_z D')
// x/y rows next to a wall read runtime tables; z columns come from a small
// column table (wall columns + the interior column).
struct StencilArgs {
  const double *__restrict__ src;
  double *__restrict__ dst;
  int Nx, Ny, Nz;
  int in_y0, in_y1, in_z0, in_z1;      // valid input box (global indices)
  int out_y0, out_y1, out_z0, out_z1;  // output box
  int zchunk;                          // output planes per workgroup
  // Toeplitz interiors exist (N >= 2p + 3) per axis
  int x_toep, y_toep, z_toep;
  double sx;        // h_y beta_x
  double cxs[19];   // v8: sx bhat[k] (the x-sweep's B band with the scale folded in)
  double cy[19];    // h_x beta_y bhat[k]
  // x: wall-column corrections [2(p+1)][2(2p+1)]: ((M_x row - [x_toep] h_x mhat) / h_x,
  //    h_y (B_x row - [x_toep] beta_x bhat)); slot x for x < x_corr_left, slot p+1+j
  //    for column Nx - x_corr_right + j
  const double *__restrict__ corrX;
  int x_corr_left, x_corr_right;
  // y wall rows, column tables [Ny + 2p + pad][2p+1] (row s + p: A(s - p + k, s)):
  const double *__restrict__ yT1;  // M_y / h_y
  const double *__restrict__ yT3;  // h_x B_y
  // z columns [2(2p+1)+1][2p+1][2] = (e, d) pairs, out(zz - p + k) += e E + d D':
  // rows 0..2p: planes 0..2p; rows 2p+1..4p+1: planes Nz-2p-1..Nz-1; row 4p+2: interior
  const double *__restrict__ zt;
  // v8 only: E arrives pre-scaled by the interior z mass scale (sx, cy, corrX's
  // B part and yT3 carry it), interior z planes use the compile-time bands
  // out(zz - p + k) += mhat[k] E + dint dhat[2p - k] D, and zt's wall rows hold
  // (M_z / h_z, B_z) pairs.
  double dint;
  double zd[19];  // v8 interior z column of D: dint * dhat[2p - k]
  int xcd_map;    // v8: XCD-aware tile order (GDM_XCD=0 disables)
  // v8 only: output plane ranges computed by this launch (chunks of zchunk
  // planes; blockIdx.z < nchunk0 -> range 0, else range 1)
  int cz0[2], cz1[2], nchunk0;
};

// Inflow boundary-data projection of one box face (two tangential directions
// t0, t1; trivial directions have one node, one point and weight 1).
struct FaceArgs {
  const double *U;  // [Q1][Q0] stage boundary values of the face
  int Q0, Q1;
  int i0_begin, i0_end, i1_begin, i1_end;  // owned output nodes
  const int *qs0, *qs1, *qc1;
  const double *w0T;  // [wmax0][ldw0]: weights of t0, node-minor (coalesced over nodes)
  const double *w1;   // [n_nodes1][wmax1]: weights of t1, node-major (wave-uniform rows)
  int wmax0, wmax1, ldw0;
  int qmax0;  // largest q-range of FACE_CHUNK consecutive t0 nodes (LDS row length)
  // cell form of step 1 (t0 non-trivial and its local cells fit LDS): Phi0 =
  // [category][l][q] values phi_l(x_q) w_q h of t0, crange0[2 i] / [2 i + 1] =
  // first / last local cell of node i
  const double *phi0;
  const int *crange0;
  int p, ncell0_total, cell0_begin;
  double *T;  // step-1 result Q1 x (i0_end - i0_begin)
  double *dst;
  int64_t base, stride0, stride1;  // dst offset of node (i0_begin, i1_begin)
  double scale;
  int phase;  // 0: both steps, 1: step 1 only (writes T), 2: step 2 only (T -> dst)
};

// The RK stage update fused into the mass inverse's x pass (gdmk_launch_mass3_rk):
// the line solve's result k is not stored; acc_out = acc_in + beta k and, with
// Y, Y = y + alpha k (gdm_vec_rk_update's arithmetic) are.  acc_in may alias
// acc_out; Y may be NULL.  Element offsets relative to each pointer = k's.
struct RkOut {
  const double *acc_in;
  double *acc_out;
  const double *y;
  double *Y;
  double beta, alpha;
};

// node geometry of one inflow face (gdmk_launch_faces_step2_add): normal axis
// d at global node coordinate `plane`, tangential axes a0 / a1 (-1 = trivial)
// with owned node ranges [b0, e0) / [b1, e1)
struct FaceAddFace {
  int64_t base, stride0, stride1;  // owned index of node (b0, b1), index strides along a0 / a1
  int d, plane, a0, b0, e0, a1, b1, e1;
};

constexpr int FACE_CHUNK = 256;  // t0 nodes per workgroup of the face row kernel

// hipFuncAttributeMaxDynamicSharedMemorySize is a per-device property of a
// kernel: `mask` holds one bit per device that has it (a second thread racing
// on the same device sets the same value again, which is harmless)
inline hipError_t gdmk_set_lds_attr(const void *kernel, size_t lds, std::atomic<uint64_t> &mask) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = 1ull << (dev & 63);
  if (mask.load(std::memory_order_acquire) & bit) return hipSuccess;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) mask.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

}  // namespace gdmk

extern "C" {
hipError_t gdmk_launch_stencil(int p, int bk, const gdmk::StencilArgs &a, hipStream_t st);
// v8: output planes [cz0[r], cz1[r]) in chunks of zchunk, z-wall planes included.
// Tail work: the workgroups that finish their chunk run step 1 of the inflow
// faces tail_faces[0, n_tail) (cell form, own T each) in row blocks claimed from
// the device counter (0 between launches: the launch's last claim resets it);
// *tail_ran: the tail was launched.  n_tail = 0: no tail work.  Launches that
// share a counter must be stream-ordered.
hipError_t gdmk_launch_stencil8(int p, int bk, const gdmk::StencilArgs &a, const gdmk::FaceArgs *tail_faces, int n_tail,
                                unsigned long long *counter, bool *tail_ran, hipStream_t st);
int gdmk_stencil_tile_rows(int p);
void gdmk_stencil8_geom(int p, int *tile_rows, int *wgs_per_cu);
hipError_t gdmk_launch_chol_lines(int p, double *v, int len, int64_t stride, int64_t n_lines, int64_t A, int64_t B,
                                  int64_t C, const double *lrow, const double *inv_diag, hipStream_t st);
// mass inverse v2 line solves (gdm_mass.hip): dir_kind 0 = contiguous lines
// (line l at l * len), 1 = strided lines (base (l / A) * B + l % A, step stride)
hipError_t gdmk_launch_mass_lines(int p, int dir_kind, const double *src, double *dst, int len, int64_t stride,
                                  int64_t n_lines, int64_t A, int64_t B, const double *lrow, const double *inv_diag,
                                  int max_wgs, hipStream_t st);
// mass inverse v3 single-sweep line solves (gdm_mass.hip); chunk length C(p)
// (0 = unsupported degree); tables padded with zero rows to len + 3 C + p
int gdmk_mass3_chunk(int p);
// passes with fewer waves of lines than this run segmented (gdm_mass.hip)
int gdmk_mass3_seg_waves();
// allow_segments (src != dst only): lines of a pass with fewer than
// gdmk_mass3_seg_waves() waves are split into segments of >= 1 chunk with
// warm-ups (one more grid dimension), so small meshes fill the GPU
hipError_t gdmk_launch_mass3(int p, int dir_kind, const double *src, double *dst, int len, int64_t stride,
                             int64_t n_lines, int64_t A, int64_t B, const double *lrow, const double *urow,
                             const double *invd, const double *cst, int row_lo, int row_hi, int allow_segments,
                             hipStream_t st);
// the x pass (dir_kind 0, contiguous lines, no segments) with the RK update
// fused into its store; hipErrorNotSupported when the v3 x pass cannot run
// unsegmented for this shape (the caller then solves and updates separately)
hipError_t gdmk_launch_mass3_rk(int p, const double *src, int len, int64_t n_lines, const double *lrow,
                                const double *urow, const double *invd, const double *cst, int row_lo, int row_hi,
                                const gdmk::RkOut &rk, hipStream_t st);
hipError_t gdmk_launch_face(const gdmk::FaceArgs &f, hipStream_t st);
// step 1 alone of n inflow faces in one launch (cell form, each face its own T)
hipError_t gdmk_launch_faces_step1(const gdmk::FaceArgs *fa, int n, hipStream_t st);
// step 2 of n inflow faces from their T, fused with the ordered adds into dst
// (the sums of face-by-face step-2 launches); fg: the faces' node geometry
hipError_t gdmk_launch_faces_step2_add(const gdmk::FaceArgs *fa, const gdmk::FaceAddFace *fg, int n, int64_t N0,
                                       int64_t N1, int64_t own_off, double *dst, hipStream_t st);
hipError_t gdmk_launch_axpby(int64_t n, double a, const double *x, double b, double *y, hipStream_t st);
hipError_t gdmk_launch_dot(int64_t n, const double *x, const double *y, double *partial, int n_partial, double *out,
                           hipStream_t st);
hipError_t gdmk_launch_zero(int64_t n, double *y, hipStream_t st);
}
