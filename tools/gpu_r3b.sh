# SPIKE refinement rounds on the device + C++ driver (incl. 3-round case); stencil phase breakdown (diag build)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_spike.py tests/test_host_driver.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pt_spike.log 2>&1; rc=$?; echo spike rc=$rc; tail -n 3 $OUT/pt_spike.log; [ $rc -eq 0 ] || exit $rc
GDM_DIAG_BITS=0,8,16,31,63,95,127,32,15,47,3,12,64 timeout -k 10 300 python -u tools/diag_stencil.py > $OUT/diag.txt 2>&1; rc=$?; echo diag rc=$rc; cat $OUT/diag.txt | grep dbg; [ $rc -eq 0 ] || exit $rc
