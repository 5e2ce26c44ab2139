# cut_poisson_app (the prototype over the C ABI) + the cut / sparse GPU tests
export TMPDIR=/tmp
OUT=gpurun_out/cutapp; mkdir -p $OUT
timeout -k 10 120 ./dealii-galerkin-difference-methods_amd/lib/host/cut_poisson_app > $OUT/app.out 2> $OUT/app.err; rc=$?; cat $OUT/app.out $OUT/app.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_host_driver.py tests/test_gpu_sparse.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pt.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -n 1 $OUT/pt.log)"; exit $rc
