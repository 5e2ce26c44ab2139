# round 2, mass inverse v3: parity (mass tests first), v2/v3 timings, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out/r2f
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mass" > gpurun_out/r2f/pytest_mass.log 2>&1; rc=$?; echo mass rc=$rc; tail -3 gpurun_out/r2f/pytest_mass.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; env "$@" timeout -k 10 120 python -u tools/bench_ops.py --configs C3,C4,C2 --ops mass_solve > gpurun_out/r2f/ops_$tag.jsonl 2>&1 || exit 1; echo "== $tag"; grep config gpurun_out/r2f/ops_$tag.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print('  %s %-10s %.4f ms  frac %.3f'%(d['config'],d['op'],d['ms'],d['frac_8TBps']))"; }
run v3 GDM_MASS=3
run v2 GDM_MASS=2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2f/prof -o ops -- python3 tools/bench_ops.py --configs C3,C4 --iters 5 --ops mass_solve > gpurun_out/r2f/prof.log 2>&1; echo prof rc=$?
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2f/pytest_gpu.log 2>&1; rc=$?; echo gpu rc=$rc; tail -3 gpurun_out/r2f/pytest_gpu.log
