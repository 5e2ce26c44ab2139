# cut wave on the device: 1D presets, composite presets, 2D wave_1 / step85; then the consumer-priority A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_cut_wave.py tests/test_gpu_cut_wave2d.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_cut.log 2>&1; rc=$?; echo cut rc=$rc; tail -n 14 $OUT/pytest_cut.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3p.sh
