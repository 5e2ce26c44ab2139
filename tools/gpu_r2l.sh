# device RK (python + C++ mirrors), separable boundary functions: parity, RK step timings, kernel stats
set -o pipefail
mkdir -p gpurun_out/r2l
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_host_driver.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu > gpurun_out/r2l/pytest_rk.log 2>&1; rc=$?; echo rk rc=$rc; tail -3 gpurun_out/r2l/pytest_rk.log; [ $rc -eq 0 ] || exit $rc
