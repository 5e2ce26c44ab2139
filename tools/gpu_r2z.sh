# CSR SpMV lanes-per-row on the config-5 cut matrix (rows of 49 and of 1 nonzero)
export TMPDIR=/tmp
OUT=gpurun_out/r2z; mkdir -p $OUT
for k in 4 8 16 32; do
  GDM_CSR_LANES=$k timeout -k 10 200 python -u tools/bench_cut_c5.py --max-it 50 > $OUT/lanes$k.json 2> $OUT/lanes$k.err || { tail -3 $OUT/lanes$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/lanes$k.json')); print('lanes $k spmv %.3f ms %.0f GB/s rel %.1e' % (d['spmv_ms'], d['spmv_GBps'], d['spmv_rel_vs_host']))"
done
