# round-end rehearsal: smoke, the whole GPU suite, the default bench line, rocprof kernel stats of the bench, C5 cut solve
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/final}; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo gpu rc=$rc; tail -n 2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo bench rc=$rc; cut -c1-300 $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
# per-config kernel statistics: the metric's compute_rhs only (no mass / RK / PMC / CPU legs in the trace)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python -u bench.py --metric-only > $OUT/bench_prof.json 2> $OUT/bench_prof.err; rc=$?; echo prof rc=$rc; [ $rc -eq 0 ] || exit $rc
find $OUT/ks -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
timeout -k 10 300 python -u tools/bench_cut_c5.py --max-it 60000 > $OUT/c5_cut.json 2> $OUT/c5_cut.err; rc=$?; echo c5 rc=$rc; cut -c1-500 $OUT/c5_cut.json
