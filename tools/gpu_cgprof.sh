# per-kernel times of the device SolverCG on the config-5 cut system (200 iterations)
export TMPDIR=/tmp
OUT=gpurun_out/cgprof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python -u tools/bench_cut_c5.py --max-it 200 > $OUT/c5.json 2> $OUT/c5.err; rc=$?; echo rc=$rc; [ $rc -eq 0 ] || { tail -5 $OUT/c5.err; exit $rc; }
find $OUT/ks -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:10]:
    print(r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))"
