#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.
# Usage (on the box, from the repo root): tools/gpu_suite.sh TAG [pytest-args...]
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
TAG=${1:-run}; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
stop_if_fatal() {  # rc: 0 ok, 1 test failures (continue); anything else -> stop
  if [ "$1" -gt 1 ]; then echo "fatal rc=$1 in $2; stopping"; exit "$1"; fi
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider "$@" > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"; stop_if_fatal $rc pytest
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-480} python bench.py ${BENCH_ARGS:---steps 30 --warmup 5} > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -2 "$OUT/bench.err"; stop_if_fatal $rc bench
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --steps 10 --warmup 2 --pmc 0 --no-cpu-baseline > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; stop_if_fatal $rc rocprof
  f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cat "$f" | cut -c1-220
fi
exit 0
