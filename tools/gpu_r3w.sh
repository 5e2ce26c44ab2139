# non-temporal mass accesses: mass / RK / parity GPU tests + bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3w; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo tests rc=$rc; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo bench rc=$rc; cut -c1-200 $OUT/bench.json
