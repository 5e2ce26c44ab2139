#!/bin/bash
# Experiment build for an on-box A/B of the stencil:
#   tools/build_variant.sh NAME [hipcc -D flags...]  -> dealii-galerkin-difference-methods_amd/lib/ab/NAME/libgdm_hip.so
# gdm_kernels.hip is rebuilt with the flags (ONLY_P=5 by default: that degree's
# stencil only; BUILD_CAPI=1: gdm_capi.cpp
# too; BUILD_MASS=1: gdm_mass.hip too; BUILD_KERNELS=0: the in-tree stencil object),
# every other object comes from the in-tree build (lib/obj).  Select it
# with GDM_HIP_LIB (tools/gpu_ab.sh, tools/time_apply.py) and delete
# lib/ab/NAME when the experiment is recorded.
NAME=$1; shift
C=/root/repo/dealii-galerkin-difference-methods_amd/csrc
B=/root/repo/dealii-galerkin-difference-methods_amd/lib/obj
O=/root/repo/dealii-galerkin-difference-methods_amd/lib/ab/$NAME
mkdir -p $O
X=""
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-function -DGDM_ONLY_P=${ONLY_P:-5} $X $*"
CAPI=$B/gdm_capi.o
if [ "${BUILD_CAPI:-0}" = 1 ]; then
  /opt/rocm/bin/hipcc $F -x hip -c $C/gdm_capi.cpp -o $O/capi.o || exit 1
  CAPI=$O/capi.o
fi
MASS=$B/gdm_mass.o
if [ "${BUILD_MASS:-0}" = 1 ]; then
  /opt/rocm/bin/hipcc $F -c $C/gdm_mass.hip -o $O/mass.o || exit 1
  MASS=$O/mass.o
fi
KERN=$B/gdm_kernels.o
if [ "${BUILD_KERNELS:-1}" = 1 ]; then
  /opt/rocm/bin/hipcc $F -c $C/gdm_kernels.hip -o $O/kernels.o || exit 1
  KERN=$O/kernels.o
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libgdm_hip.so $CAPI $KERN $B/gdm_setup.o \
  $B/gdm_csr.o $MASS $B/gdm_rk.o $B/gdm_post.o $B/gdm_cut.o $B/gdm_cut_advection.o $B/gdm_cut_wave.o \
  $B/gdm_band.o && rm -f $O/kernels.o $O/capi.o $O/mass.o && echo "built $O"
