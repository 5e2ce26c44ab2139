#!/bin/bash
# The round-end run, exactly as the driver does it, on one GPU box:
#   smoke(), the WHOLE `pytest -x -q -m gpu` suite (never a hand-picked
#   subset), the default bench line, and rocprofv3 kernel stats of the bench
#   metric (compute_rhs only).  Extra perf steps go after it, per call:
#     gpurun -- 'bash tools/gpu_check.sh r4a && <extra steps>'
# Usage: tools/gpu_check.sh TAG   -> gpurun_out/TAG/{smoke.log,pytest_gpu.log,bench.json,kernel_stats.csv}
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-check}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -n 1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -n 2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "bench rc=$rc"; cut -c1-300 "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ks" -o ks --output-format csv -- \
  python -u bench.py --metric-only > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/ks" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/ks" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
# the stats average every launch (settle + warm-up + timed); the timed steps alone:
python3 tools/trace_avg.py "$OUT/kernel_trace.csv" 50 > "$OUT/kernel_timed_avg.txt"
exit 0
