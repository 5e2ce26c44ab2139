# cut-cell product path on the GPU: sparse tests (incl. the library assembly end to end) + config 5 with cut values
export TMPDIR=/tmp
OUT=gpurun_out/r2x; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py -x -q --timeout 200 --timeout-method thread > $OUT/pt_sparse.log 2>&1; rc=$?; echo "sparse rc=$rc $(tail -n 1 $OUT/pt_sparse.log)"; [ $rc -eq 0 ] || { tail -30 $OUT/pt_sparse.log; exit $rc; }
timeout -k 10 400 python -u tools/bench_cut_c5.py --max-it 2000 > $OUT/c5_cut.json 2> $OUT/c5_cut.err; rc=$?; cat $OUT/c5_cut.json; [ $rc -eq 0 ] || { tail $OUT/c5_cut.err; exit $rc; }
