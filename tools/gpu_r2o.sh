set -o pipefail
mkdir -p gpurun_out/r2o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_host_driver.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k multirank > gpurun_out/r2o/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/r2o/pytest.log; exit $rc
