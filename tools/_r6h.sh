export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o mt --output-format csv -- python -u bench.py --metric-only --steps 200 > $O/metric.json 2>> $O/err.log || exit 3
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/metric_trace.csv \;
