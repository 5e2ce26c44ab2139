# GPU suite (cut advection full-row formulation, mass rows v5), mass A/B v5 vs v4, fresh PMC of the shipped C3 stencil
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo gpu rc=$rc; tail -n 4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
for v in main massv4 main massv4; do
  if [ $v = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$v/libgdm_hip.so; fi
  timeout -k 10 300 python -u tools/bench_ops.py --configs C3,C4,C2 --ops mass_solve,rk_step --iters 20 > $OUT/ops_$v.jsonl 2> $OUT/ops_$v.err; rc=$?
  echo "== $v rc=$rc"; python3 -c "import json,sys
for l in open('$OUT/ops_$v.jsonl'):
  d=json.loads(l); print(d['config'], d['op'], '%.4f' % d.get('stage_ms', d['ms']))"; [ $rc -eq 0 ] || exit $rc
done
unset GDM_HIP_LIB
timeout -k 10 900 bash tools/pmc_stencil.sh r3i/pmc_c3 > $OUT/pmc_c3.txt 2>&1; rc=$?; echo pmc rc=$rc; grep -A30 "stencil8" $OUT/pmc_c3.txt | head -70
