# y-wall corrections in the consumer waves: parity of the stencil paths, A/B compute_rhs timing, cut-Poisson device CG
export TMPDIR=/tmp
OUT=gpurun_out/r2u; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
timeout -k 10 200 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 150 --timeout-method thread -k "cut_poisson" > $OUT/pt_cut.log 2>&1; echo "cut rc=$? $(tail -n 1 $OUT/pt_cut.log)"


ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3 --ops apply --iters 30 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print('%s %s %.4f ms frac %.3f' % (d['config'], d['op'], d['ms'], d['frac_8TBps']))"; }
for v in main yw0 yw1 main yw0 yw1; do
  if [ $v = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$v/libgdm_hip.so; fi
  echo "== $v $(ops)" || exit 1
done
