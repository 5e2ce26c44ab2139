# like tools/build_capi_variant.sh but rebuilds only the mass kernels (gdm_mass.hip) with extra flags
NAME=$1; shift
C=/root/repo/dealii-galerkin-difference-methods_amd/csrc
B=/root/repo/dealii-galerkin-difference-methods_amd/lib/obj
O=/root/repo/dealii-galerkin-difference-methods_amd/lib/ab/$NAME
mkdir -p $O
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-function $*"
/opt/rocm/bin/hipcc $F -c $C/gdm_mass.hip -o $O/mass.o &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libgdm_hip.so $B/gdm_capi.o $B/gdm_kernels.o $B/gdm_setup.o \
  $B/gdm_csr.o $O/mass.o $B/gdm_rk.o $B/gdm_post.o $B/gdm_cut.o $B/gdm_cut_advection.o $B/gdm_cut_wave.o $B/gdm_band.o && echo "built $O"
