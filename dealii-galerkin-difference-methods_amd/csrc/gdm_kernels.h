// gdm_kernels.h -- device-side argument blocks and launchers of gdm_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gdmk {

// Fused Kronecker stencil: out = B_x M_y M_z + M_x B_y M_z + M_x M_y B_z (or
// M_x M_y M_z for the mass operator) applied to the input box, written for
// the output box.  Arrays are [z - z0][y - y0][x] with full x extent.
struct StencilArgs {
  const double *__restrict__ src;
  double *__restrict__ dst;
  int Nx, Ny, Nz;
  int in_y0, in_y1, in_z0, in_z1;      // valid input box (global indices)
  int out_y0, out_y1, out_z0, out_z1;  // output box
  int zchunk;                          // output planes per workgroup
  const double *__restrict__ tMx;      // [2p+1] Toeplitz (interior) row of M_x
  const double *__restrict__ tBx;      // [2p+1] Toeplitz (interior) row of B_x
  const double *__restrict__ corrX;    // [2(p+1)][2 (2p+1)] (row_M(x) - tM, row_B(x) - tB) of the wall
                                       //   columns: slot x for x < x_corr_left, slot p+1+j for
                                       //   column Nx - x_corr_right + j
  int x_corr_left, x_corr_right;       // wall columns with corrections (<= p+1 each)
  const double *__restrict__ colMy;    // [Ny + 2p][2p+1] row s + p: M_y(s - p + k, s)
  const double *__restrict__ colBy;
  const double *__restrict__ colMz;    // [Nz][2p+1]      M_z(z - p + k, z)
  const double *__restrict__ colBz;
};

// Inflow boundary-data projection of one box face (two tangential directions
// t0, t1; trivial directions have one node, one point and weight 1).
struct FaceArgs {
  const double *U;  // [Q1][Q0] stage boundary values of the face
  int Q0, Q1;
  int i0_begin, i0_end, i1_begin, i1_end;  // owned output nodes
  const int *qs0, *qc0, *qs1, *qc1;
  const double *w0, *w1;
  int wmax0, wmax1;
  double *T;  // scratch Q1 x (i0_end - i0_begin)
  double *dst;
  int64_t base, stride0, stride1;  // dst offset of node (i0_begin, i1_begin)
  double scale;
};

}  // namespace gdmk

extern "C" {
hipError_t gdmk_launch_stencil(int p, bool mass, const gdmk::StencilArgs &a, hipStream_t st);
int gdmk_stencil_tile_rows(int p);
hipError_t gdmk_launch_chol_lines(int p, double *v, int len, int64_t stride, int64_t n_lines, int64_t A, int64_t B,
                                  int64_t C, const double *lrow, const double *inv_diag, hipStream_t st);
hipError_t gdmk_launch_face(const gdmk::FaceArgs &f, hipStream_t st);
hipError_t gdmk_launch_axpby(int64_t n, double a, const double *x, double b, double *y, hipStream_t st);
hipError_t gdmk_launch_dot(int64_t n, const double *x, const double *y, double *partial, int n_partial, double *out,
                           hipStream_t st);
hipError_t gdmk_launch_zero(int64_t n, double *y, hipStream_t st);
}
