set -o pipefail
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2e/pytest_parity.log 2>&1; rc=$?; echo parity rc=$rc; tail -3 gpurun_out/r2e/pytest_parity.log; [ $rc -le 1 ] || exit $rc
run() { tag=$1; shift; env "$@" timeout -k 10 120 python -u tools/bench_ops.py --configs C3,C4 > gpurun_out/r2e/ops_$tag.jsonl 2>&1 || exit 1; echo "== $tag"; grep config gpurun_out/r2e/ops_$tag.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print('  %s %-10s %.4f ms  frac %.3f'%(d['config'],d['op'],d['ms'],d['frac_8TBps']))"; }
run default
run noxcd GDM_XCD=0
run rounds2 GDM_ROUNDS=2
run rounds3 GDM_ROUNDS=3
run nozint GDM_NO_ZINT=1
run xu16 GDM_MASS_XU=16
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2e/prof -o ops -- python3 tools/bench_ops.py --configs C3 --iters 5 > gpurun_out/r2e/prof.log 2>&1; echo prof rc=$?
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r2e/pmc -o pmc_$(echo $c|cut -d' ' -f1) -- python3 bench.py --pmc-child > /dev/null 2>&1; echo pmc $c rc=$?
done
