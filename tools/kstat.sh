#!/bin/bash
# Fast register/ISA check of one stencil instance (p, advection, 16-B DMA):
#   tools/kstat.sh [P] [extra hipcc flags]   -> /tmp/kstat.s + resource usage
P=${1:-5}; shift
SRC=/root/repo/dealii-galerkin-difference-methods_amd/csrc/gdm_kernels.hip
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-function --cuda-device-only -S \
  -DGDM_ONLY_P=$P "$@" $SRC -o /tmp/kstat.s -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "error|Function Name|VGPRs:|SGPRs:|Spill|Occupancy" | grep -A6 "stencil8" | sed 's/.*remark: //'
