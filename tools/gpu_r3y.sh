# locate the slow / hanging GPU test of r3x: verbose, per-test timeout below the silence limit
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread --durations=15 > $OUT/pytest_parity.log 2>&1; rc=$?; echo parity rc=$rc; tail -n 25 $OUT/pytest_parity.log
