# round-end rehearsal: smoke, the whole GPU suite, the default bench line
set -o pipefail
mkdir -p gpurun_out/full
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -2 gpurun_out/full/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1; rc=$?; echo gpu rc=$rc; tail -3 gpurun_out/full/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err; echo bench rc=$?; cat gpurun_out/full/bench.json | cut -c1-400
