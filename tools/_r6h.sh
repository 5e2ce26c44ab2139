export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do timeout -k 10 200 python -u tools/rank_legs.py 20 > $O/legs_$rep.json 2>> $O/err.log || exit 2; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o rl --output-format csv -- python -u tools/rank_legs.py 20 > $O/prof_legs.json 2>> $O/err.log || exit 3
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/rank_kernel_stats.csv \;
