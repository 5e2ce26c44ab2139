# cut_wave_app (wave-app.cc over the C ABI) against every applications/wave golden
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3r; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_host_driver.py -x -v -m gpu -k cut_wave -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_cut_wave_app.log 2>&1; rc=$?; echo rc=$rc; tail -n 12 $OUT/pytest_cut_wave_app.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 dealii-galerkin-difference-methods_amd/lib/host/cut_wave_app 2 wave > $OUT/wave_1.out 2> $OUT/wave_1.err; echo app rc=$?
