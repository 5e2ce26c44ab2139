# face step 2 on the side stream (apply timing), strided-x mass pass A/B (timing + parity), focused tests
export TMPDIR=/tmp
OUT=gpurun_out/r4i; mkdir -p $OUT
V=dealii-galerkin-difference-methods_amd/lib/variants
timeout -k 10 200 python -u tools/bench_ops.py --configs C3 --ops apply --iters 30 > $OUT/ops_main.jsonl 2>&1; rc=$?; cat $OUT/ops_main.jsonl; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4,C2 --ops mass_solve --iters 20 >> $OUT/mass_main.jsonl 2>&1 || exit 3
  GDM_HIP_LIB=$V/mx/libgdm_hip.so timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4,C2 --ops mass_solve --iters 20 >> $OUT/mass_mx.jsonl 2>&1 || exit 3
done
cat $OUT/mass_main.jsonl $OUT/mass_mx.jsonl | cut -c1-160
GDM_HIP_LIB=$V/mx/libgdm_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mass_segments.py -k "mass" -q -p no:cacheprovider --timeout 300 > $OUT/mx_tests.log 2>&1; echo "mx tests rc=$?"; tail -n 2 $OUT/mx_tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mass_segments.py tests/test_gpu_cut_wave.py tests/test_gpu_spike.py tests/test_host_mpi.py tests/test_gpu_cut_advection.py tests/test_gpu_rk.py -q -s -p no:cacheprovider --timeout 300 > $OUT/tests.log 2>&1; echo "main tests rc=$?"
grep -E "segmented mass|passed|failed|^FAILED" $OUT/tests.log | tail -15
