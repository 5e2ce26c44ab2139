# GPU suite (after the cut-advection tolerance fix), then the r3g stencil variant experiments
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo gpu rc=$rc; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r3g.sh
