// gdm_faces.h -- fused step 2 of the inflow boundary-data projection (gdm_faces.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gdmk {

// one face's step 2: dst[base + t stride0 + (i1 - i1_begin) stride1] +=
// scale sum_m w1[i1][m] T[qs1[i1] + m][t], t < n0, i1 in [i1_begin, i1_end)
struct Step2Face {
  const double *T;
  int n0, i1_begin, i1_end, wmax1;
  const int *qs1, *qc1;
  const double *w1;
  int64_t base, stride0, stride1;
  double scale;
};
struct Step2Set {
  Step2Face f[6];
  int n;
};

}  // namespace gdmk

extern "C" hipError_t gdmk_launch_face_step2_multi(const gdmk::Step2Set &s, double *dst, hipStream_t st);
