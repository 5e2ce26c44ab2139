# HEAD check after removing the racy fused face step 2: smoke, parity suite, ops timing, bench line
export TMPDIR=/tmp
OUT=gpurun_out/r2r; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pt.log 2>&1; rc=$?; echo "parity rc=$rc $(tail -n 1 $OUT/pt.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4,C2 --ops apply,mass_solve --iters 20 > $OUT/ops.jsonl 2>&1; rc=$?; cut -c1-220 $OUT/ops.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; cut -c1-700 $OUT/bench.json; exit $rc
