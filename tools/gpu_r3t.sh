# RK stage kernels (vectorized non-temporal update, one boundary launch for all faces): stage profile at C3 + the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3t; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ps -o ps --output-format csv -- python -u tools/profile_stage.py > $OUT/stage.txt 2> $OUT/stage.err; rc=$?; echo prof rc=$rc; cat $OUT/stage.txt; [ $rc -eq 0 ] || exit $rc
find $OUT/ps -name "*kernel_stats.csv" -exec cp {} $OUT/stage_kernel_stats.csv \;
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo tests rc=$rc; tail -n 3 $OUT/pytest.log
