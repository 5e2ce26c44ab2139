# consumer-wave priority A/B (s_setprio in the stencil consumer waves): C3 p=5 and C4 p=7, same-config builds
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r3p}; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
run() {  # name lib p kind config
  local name=$1 lib=$2 p=$3 kind=$4 cfg=$5
  if [ "$lib" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$lib/libgdm_hip.so; fi
  timeout -k 10 240 python -u tools/variant_check.py --p $p --kind $kind --config $cfg > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; echo "== $name rc=$rc $(cat $OUT/$name.json)"; [ $rc -le 1 ] || exit $rc
}
for i in 1 2 3; do
  run c3_base5_$i base5 5 advection C3
  run c3_prio3_$i prio3 5 advection C3
  run c3_prio1_$i prio1 5 advection C3
  run c4_base7_$i base7 7 wave C4
  run c4_prio3_$i prio3p7 7 wave C4
done
