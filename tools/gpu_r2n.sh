# device postprocess + distributed mass inverse: parity tests, timing
set -o pipefail
mkdir -p gpurun_out/r2n
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_post.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2n/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/r2n/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_post.py 511 5 > gpurun_out/r2n/bench_post.log 2>&1; rc=$?; cat gpurun_out/r2n/bench_post.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/bench_post.py 255 7 >> gpurun_out/r2n/bench_post.log 2>&1; rc=$?; tail -1 gpurun_out/r2n/bench_post.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2n/prof -o post -- python3 $GRAFT_REPO_ROOT/tools/bench_post.py 511 5 > $GRAFT_REPO_ROOT/gpurun_out/r2n/prof.log 2>&1; echo prof rc=$?
