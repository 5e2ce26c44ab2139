# row-block SpMV: sparse parity suite, then SpMV / CG timing on the config-5 cut matrix and the synthetic C5 stencil
export TMPDIR=/tmp
OUT=gpurun_out/r2z2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 200 --timeout-method thread > $OUT/pt_sparse.log 2>&1; rc=$?; echo "sparse rc=$rc $(tail -n 1 $OUT/pt_sparse.log)"; [ $rc -eq 0 ] || { tail -30 $OUT/pt_sparse.log; exit $rc; }
GDM_CSR_MODE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 200 --timeout-method thread > $OUT/pt_sparse_m1.log 2>&1; rc=$?; echo "sparse mode1 rc=$rc $(tail -n 1 $OUT/pt_sparse_m1.log)"; [ $rc -eq 0 ] || { tail -30 $OUT/pt_sparse_m1.log; exit $rc; }
for m in 1 0; do
  GDM_CSR_MODE=$m timeout -k 10 200 python -u tools/bench_cut_c5.py --max-it 50 > $OUT/cut_m$m.json 2> $OUT/cut_m$m.err || { tail -3 $OUT/cut_m$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/cut_m$m.json')); print('cut mode $m spmv %.3f ms %.0f GB/s rel %.1e cg %.3f ms/it' % (d['spmv_ms'], d['spmv_GBps'], d['spmv_rel_vs_host'], d['cg_ms_per_it']))"
done
for m in 1 0; do
  GDM_CSR_MODE=$m timeout -k 10 200 python -u tools/bench_csr.py > $OUT/syn_m$m.json 2> $OUT/syn_m$m.err || { tail -3 $OUT/syn_m$m.err; exit 1; }
  echo "synthetic mode $m: $(cut -c1-300 $OUT/syn_m$m.json)"
done
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3 --ops apply --iters 30 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print('%.4f ms' % d['ms'])"; }
for v in main pf3 np6 np4 main; do
  if [ $v = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$v/libgdm_hip.so; fi
  echo "== stencil $v $(ops)" || exit 1
done
