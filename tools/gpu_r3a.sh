# round 3, first box: the engine-first import order, then the full rehearsal
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_host_driver.py tests/test_gpu_sparse.py tests/test_runtime.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_order.log 2>&1; rc=$?; echo order rc=$rc; tail -n 2 $OUT/pytest_order.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT bash tools/gpu_final.sh
