#!/bin/bash
# Build a p=5-only (ONLY_P=7: p=7-only) experiment variant of libgdm_hip.so:
#   tools/build_variant.sh NAME [hipcc -D flags...]  -> .../lib/variants/NAME/libgdm_hip.so
# Select it with GDM_HIP_LIB=<path> (bench.py / tests load through gdm_amd._capi).
# The csr / mass / rk / post objects are taken from the in-tree build (lib/obj).
NAME=$1; shift
C=/root/repo/dealii-galerkin-difference-methods_amd/csrc
B=/root/repo/dealii-galerkin-difference-methods_amd/lib/obj
O=/root/repo/dealii-galerkin-difference-methods_amd/lib/variants/$NAME
mkdir -p $O
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-function -DGDM_ONLY_P=${ONLY_P:-5} $*"
/opt/rocm/bin/hipcc $F -x hip -c $C/gdm_capi.cpp -o $O/capi.o &&
/opt/rocm/bin/hipcc $F -c $C/gdm_kernels.hip -o $O/kernels.o &&
g++ -O3 -std=c++17 -fPIC -c $C/gdm_setup.cpp -o $O/setup.o &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libgdm_hip.so $O/capi.o $O/kernels.o $O/setup.o \
  $B/gdm_csr.o $B/gdm_mass.o $B/gdm_rk.o $B/gdm_post.o $B/gdm_cut.o $B/gdm_cut_advection.o $B/gdm_cut_wave.o $B/gdm_band.o && echo "built $O"
