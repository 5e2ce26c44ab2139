# device RK (wave-rk / advection with device boundary functions): parity, timings, kernel stats
set -o pipefail
mkdir -p gpurun_out/r2i
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2i/pytest_rk.log 2>&1; rc=$?; echo rk rc=$rc; tail -3 gpurun_out/r2i/pytest_rk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4 --ops apply,mass_solve,rk_step > gpurun_out/r2i/ops.jsonl 2>&1; echo ops rc=$?; grep config gpurun_out/r2i/ops.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2i/prof -o rk -- python3 tools/bench_ops.py --configs C4 --iters 5 --ops rk_step > gpurun_out/r2i/prof.log 2>&1; echo prof rc=$?
