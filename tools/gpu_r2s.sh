# mass-inverse diagnosis: FIFO depth variants, interior-rows-everywhere timing, kernel stats, PMC passes
export TMPDIR=/tmp
OUT=gpurun_out/r2s; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3,C4 --ops mass_solve --iters 20 2>/dev/null | cut -c1-160; }
echo "== main"; ops || exit 1
echo "== notab"; GDM_MASS_NOTAB=1 ops || exit 1
echo "== q16"; GDM_HIP_LIB=$L/q16/libgdm_hip.so ops || exit 1
echo "== q24"; GDM_HIP_LIB=$L/q24/libgdm_hip.so ops || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python tools/bench_ops.py --configs C3 --ops mass_solve --iters 5 > $OUT/ks.log 2>&1 || exit 1
find $OUT/ks -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -6
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 100 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python tools/bench_ops.py --configs C3 --ops mass_solve --iters 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1; head -80 $OUT/pmc_summary.txt
