# all-faces step-2 launch (atomic edges) + one-launch z-mixed stencil (GDM_ZMIX=1): parity + A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3j; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rk.py tests/test_gpu_periodic.py tests/test_gpu_cut_advection.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pt_default.log 2>&1; rc=$?; echo pytest default rc=$rc; tail -n 2 $OUT/pt_default.log; [ $rc -le 1 ] || exit $rc
GDM_ZMIX=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rk.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pt_zmix.log 2>&1; rc=$?; echo pytest zmix rc=$rc; tail -n 2 $OUT/pt_zmix.log; [ $rc -le 1 ] || exit $rc
for z in 0 1 0 1; do
  for c in "5 advection C3" "7 wave C4"; do
    set -- $c
    GDM_ZMIX=$z timeout -k 10 240 python -u tools/variant_check.py --p $1 --kind $2 --config $3 > $OUT/v.json 2> $OUT/v.err; rc=$?
    echo "zmix=$z $3 rc=$rc $(cat $OUT/v.json)"; [ $rc -le 1 ] || exit $rc
  done
done
