set -o pipefail
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mass_solve" > gpurun_out/r2d/pytest_mass.log 2>&1; rc=$?; echo mass tests rc=$rc; tail -3 gpurun_out/r2d/pytest_mass.log; [ $rc -le 1 ] || exit $rc
for v in 3 2; do
  GDM_MASS=$v timeout -k 10 120 python -u tools/bench_ops.py --ops mass_solve --configs C3,C4,C2 > gpurun_out/r2d/ops_v$v.jsonl 2>&1 || exit 1
  echo "v=$v"; grep config gpurun_out/r2d/ops_v$v.jsonl | cut -c1-150
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2d/prof -o ops -- python3 tools/bench_ops.py --ops mass_solve --iters 5 --configs C3,C4 > gpurun_out/r2d/prof.log 2>&1; echo prof rc=$?
