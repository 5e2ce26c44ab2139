// gdm_faces.hip -- step 2 of the inflow boundary-data projection for all faces
// of an operator in ONE launch (advection/stiffness.h:473-532: the inflow term
// -<(a.n) g, v> on the box faces; step 1 (the t0 contraction into the per-face
// scratch T) runs on the side stream during the interior stencil launch, see
// gdm_capi.cpp gdm_apply).  Step 2 contracts t1 and adds into dst; it must
// follow the stencil's stores, so it sits on the critical path after the join:
// one launch over every face (grid.z = face) instead of one per face lets the
// faces' short, latency-bound grids overlap.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gdm_faces.h"

namespace gdmk {

__global__ void __launch_bounds__(256) face_step2_multi_kernel(Step2Set s, double *__restrict__ dst) {
  const Step2Face &F = s.f[blockIdx.z];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i1 = F.i1_begin + (int)blockIdx.y;
  if (t >= F.n0 || i1 >= F.i1_end) return;
  const double *w = F.w1 + (int64_t)i1 * F.wmax1;
  const int n = F.qc1[i1], q = F.qs1[i1];
  double acc = 0.0;
  for (int m = 0; m < n; ++m) acc = fma(w[m], F.T[(int64_t)(q + m) * F.n0 + t], acc);
  double *d = dst + F.base + (int64_t)t * F.stride0 + (int64_t)(i1 - F.i1_begin) * F.stride1;
  *d += F.scale * acc;
}

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_face_step2_multi(const gdmk::Step2Set &s, double *dst, hipStream_t st) {
  if (s.n <= 0) return hipSuccess;
  int gx = 1, gy = 1;
  for (int k = 0; k < s.n; ++k) {
    gx = gx > (s.f[k].n0 + 255) / 256 ? gx : (s.f[k].n0 + 255) / 256;
    gy = gy > s.f[k].i1_end - s.f[k].i1_begin ? gy : s.f[k].i1_end - s.f[k].i1_begin;
  }
  hipLaunchKernelGGL(gdmk::face_step2_multi_kernel, dim3(gx, gy, s.n), dim3(256), 0, st, s, dst);
  return hipGetLastError();
}
