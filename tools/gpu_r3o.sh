# 2D cut wave on the device (wave_1 / step85 goldens) + cut wave 1D regression; full-size C2 / C3 / C4 checks;
# consumer-wave priority A/B (s_setprio)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_cut_wave2d.py tests/test_gpu_cut_wave.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_cut.log 2>&1; rc=$?; echo cut rc=$rc; tail -n 12 $OUT/pytest_cut.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -m gpu -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/pytest_fullsize.log 2>&1; rc=$?; echo fullsize rc=$rc; tail -n 5 $OUT/pytest_fullsize.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
run() {  # name lib p kind config
  local name=$1 lib=$2 p=$3 kind=$4 cfg=$5
  if [ "$lib" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$lib/libgdm_hip.so; fi
  timeout -k 10 240 python -u tools/variant_check.py --p $p --kind $kind --config $cfg > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; echo "== $name rc=$rc $(cat $OUT/$name.json)"; [ $rc -le 1 ] || exit $rc
}
for i in 1 2; do
  run c3_main_$i main 5 advection C3
  run c3_prio3_$i prio3 5 advection C3
  run c3_prio1_$i prio1 5 advection C3
  run c4_main_$i main 7 wave C4
  run c4_prio3_$i prio3p7 7 wave C4
done
