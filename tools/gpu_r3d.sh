# cut-cell advection on the device vs the oracle / test_01 golden
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_cut_advection.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pt_cutadv.log 2>&1; rc=$?; echo cutadv rc=$rc; tail -n 12 $OUT/pt_cutadv.log; [ $rc -eq 0 ] || exit $rc
