# cut_wave_app vs every applications/wave golden; RK-stage kernel breakdown at C3
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r3r.sh || exit $?
OUT=gpurun_out/r3s; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ps -o ps --output-format csv -- python -u tools/profile_stage.py > $OUT/stage.txt 2> $OUT/stage.err; rc=$?; echo prof rc=$rc; cat $OUT/stage.txt
find $OUT/ps -name "*kernel_stats.csv" -exec cp {} $OUT/stage_kernel_stats.csv \;
