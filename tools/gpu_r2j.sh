# device RK (python + C++ mirrors), separable boundary functions: parity, RK step timings, kernel stats
set -o pipefail
mkdir -p gpurun_out/r2j
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rk.py tests/test_host_driver.py tests/test_gpu_periodic.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu > gpurun_out/r2j/pytest_rk.log 2>&1; rc=$?; echo rk rc=$rc; tail -3 gpurun_out/r2j/pytest_rk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4,C2 --ops rk_step > gpurun_out/r2j/ops.jsonl 2>&1; echo ops rc=$?; grep config gpurun_out/r2j/ops.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2j/prof -o rk -- python3 tools/bench_ops.py --configs C3,C4 --iters 3 --ops rk_step > gpurun_out/r2j/prof.log 2>&1; echo prof rc=$?
