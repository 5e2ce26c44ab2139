set -o pipefail
mkdir -p gpurun_out/r2c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mass" > gpurun_out/r2c/pytest_mass.log 2>&1; rc=$?; echo mass tests rc=$rc; tail -3 gpurun_out/r2c/pytest_mass.log; [ $rc -le 1 ] || exit $rc
for w in 0 256 512 1024 2048; do
  GDM_MASS_WGS=$w timeout -k 10 120 python -u tools/bench_ops.py --ops mass_solve --configs C3,C4,C2 > gpurun_out/r2c/ops_w$w.jsonl 2>&1 || exit 1
  echo "wgs=$w"; cut -c1-150 gpurun_out/r2c/ops_w$w.jsonl
done
GDM_MASS=1 timeout -k 10 120 python -u tools/bench_ops.py --ops mass_solve --configs C3 > gpurun_out/r2c/ops_v1.jsonl 2>&1 || exit 1
cut -c1-150 gpurun_out/r2c/ops_v1.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2c/prof -o ops -- python3 tools/bench_ops.py --ops mass_solve --iters 5 > gpurun_out/r2c/prof.log 2>&1; echo prof rc=$?
