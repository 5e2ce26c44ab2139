# short verification of the non-temporal mass / stencil stores: mass, stencil parity, full size, RK; bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mass_segments.py tests/test_gpu_fullsize.py tests/test_gpu_rk.py tests/test_gpu_spike.py -x -v -m gpu -p no:cacheprovider --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo tests rc=$rc; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo bench rc=$rc; cut -c1-200 $OUT/bench.json
