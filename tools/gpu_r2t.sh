# mass inverse v4 (buffer addressing, streamed stores, per-part table rows): parity + A/B timing
export TMPDIR=/tmp
OUT=gpurun_out/r2t; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spike.py -x -q --timeout 200 --timeout-method thread -k "mass_solve" > $OUT/pt.log 2>&1; rc=$?; echo "mass tests rc=$rc $(tail -n 1 $OUT/pt.log)"; [ $rc -eq 0 ] || { tail -30 $OUT/pt.log; exit $rc; }
ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3,C4,C2 --ops mass_solve --iters 20 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print('%s %s %.3f ms frac %.3f' % (d['config'], d['op'], d['ms'], d['frac_8TBps']))"; }
echo "== main"; ops || exit 1
echo "== old"; GDM_HIP_LIB=$L/old/libgdm_hip.so ops || exit 1
echo "== e2"; GDM_HIP_LIB=$L/e2/libgdm_hip.so ops || exit 1
echo "== main again"; ops || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python tools/bench_ops.py --configs C3,C4 --ops mass_solve --iters 5 > $OUT/ks.log 2>&1 || exit 1
find $OUT/ks -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -6
