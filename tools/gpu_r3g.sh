# stencil tile variants (2 workgroups per CU: TY 16; p=7 tiles) and launch rounds: parity vs the oracle + compute_rhs timing
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3g; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
run() {  # name lib p kind config [env]
  local name=$1 lib=$2 p=$3 kind=$4 cfg=$5; shift 5
  if [ "$lib" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$lib/libgdm_hip.so; fi
  env "$@" timeout -k 10 240 python -u tools/variant_check.py --p $p --kind $kind --config $cfg > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; echo "== $name rc=$rc $(cat $OUT/$name.json)"; [ $rc -le 1 ] || exit $rc
}
run c3_main main 5 advection C3 X=1
run c4_main main 7 wave C4 X=1
run c3_r2 main 5 advection C3 GDM_ROUNDS=2
run c4_r2 main 7 wave C4 GDM_ROUNDS=2
run c3_wg2 p5wg2 5 advection C3 X=1
run c3_wg2b p5wg2b 5 advection C3 X=1
run c4_p7main p7main 7 wave C4 X=1
run c4_p7wg2 p7wg2 7 wave C4 X=1
run c4_p7main_r2 p7main 7 wave C4 GDM_ROUNDS=2
run c3_main2 main 5 advection C3 X=1
