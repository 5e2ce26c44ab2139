# stencil tile variants (2 workgroups per CU: TY 16, 4+4 waves): smoke parity + C3 compute_rhs timing, A/B with main
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3e; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3 --ops apply --iters 30 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print('%.4f ms' % d['ms'])"; }
for v in main wg2 wg2db main wg2; do
  if [ $v = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$v/libgdm_hip.so; fi
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$v.log 2>&1 || { echo "smoke $v failed"; tail -3 $OUT/smoke_$v.log; exit 1; }
  echo "== stencil $v $(ops) | $(tail -1 $OUT/smoke_$v.log | cut -c1-80)"
done
