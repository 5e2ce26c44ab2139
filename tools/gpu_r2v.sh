# stencil phase breakdown (diagnostic build) + the default bench line under rocprof kernel stats
export TMPDIR=/tmp
OUT=gpurun_out/r2v; mkdir -p $OUT
timeout -k 10 200 python -u tools/diag_stencil.py 511 5 advection > $OUT/diag.txt 2>&1; rc=$?; cat $OUT/diag.txt | grep dbg; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/ks -o ks --output-format csv -- python -u bench.py --pmc 0 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; cut -c1-400 $OUT/bench.json; [ $rc -eq 0 ] || { tail $OUT/bench.err; exit $rc; }
find $OUT/ks -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:10]:
    print(r['Name'][:70], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))"
