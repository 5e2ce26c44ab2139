# x-wall precompute + fused face step 2: parity, ops timing, bench line
export TMPDIR=/tmp
OUT=gpurun_out/r2q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pt.log 2>&1; rc=$?; echo "parity rc=$rc $(tail -n 1 $OUT/pt.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4,C2 --ops apply --iters 20 > $OUT/ops.jsonl 2>&1; rc=$?; cat $OUT/ops.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit $rc
GDM_SERIAL=1 timeout -k 10 200 python -u tools/bench_ops.py --configs C3 --ops apply --iters 20 > $OUT/ops_serial.jsonl 2>&1; cat $OUT/ops_serial.jsonl | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; cut -c1-600 $OUT/bench.json; exit $rc
