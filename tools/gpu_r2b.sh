set -o pipefail
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2b/pytest_sparse.log 2>&1; echo sparse rc=$?; tail -3 gpurun_out/r2b/pytest_sparse.log
timeout -k 10 200 python -u tools/bench_ops.py > gpurun_out/r2b/ops.jsonl 2> gpurun_out/r2b/ops.err || exit 1
cat gpurun_out/r2b/ops.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2b/prof -o ops -- python3 tools/bench_ops.py --iters 5 > gpurun_out/r2b/prof.log 2>&1; echo prof rc=$?
timeout -k 10 300 python -u tools/bench_csr.py > gpurun_out/r2b/csr.json 2> gpurun_out/r2b/csr.err; echo csr rc=$?; cat gpurun_out/r2b/csr.json
