#!/bin/bash
# Build an experiment variant of libgdm_hip.so that differs only in gdm_mass.hip:
#   tools/build_mass_variant.sh NAME [hipcc -D flags...] -> .../lib/variants/NAME/libgdm_hip.so
# (every other object from the in-tree build, lib/obj).  Select with GDM_HIP_LIB=<path>.
NAME=$1; shift
C=/root/repo/dealii-galerkin-difference-methods_amd/csrc
B=/root/repo/dealii-galerkin-difference-methods_amd/lib/obj
O=/root/repo/dealii-galerkin-difference-methods_amd/lib/variants/$NAME
mkdir -p $O
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-function "$@" -c $C/${GDM_MASS_SRC:-gdm_mass.hip} -o $O/mass.o &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libgdm_hip.so $B/gdm_capi.o $B/gdm_kernels.o $B/gdm_setup.o \
  $B/gdm_csr.o $O/mass.o $B/gdm_rk.o $B/gdm_post.o $B/gdm_cut.o $B/gdm_cut_advection.o $B/gdm_cut_wave.o $B/gdm_band.o && echo "built $O"
