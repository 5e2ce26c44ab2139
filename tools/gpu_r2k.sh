# fork/join compute_rhs: parity, serial vs concurrent timings, bench line, rocprof
set -o pipefail
mkdir -p gpurun_out/r2k
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "advection or stencil or slab or planes" > gpurun_out/r2k/pytest.log 2>&1; rc=$?; echo parity rc=$rc; tail -2 gpurun_out/r2k/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do GDM_SERIAL=$v timeout -k 10 200 python -u tools/bench_ops.py --configs C3,C4 --ops apply > gpurun_out/r2k/ops_serial$v.jsonl 2>&1 || exit 1; echo "serial=$v"; grep config gpurun_out/r2k/ops_serial$v.jsonl | cut -c1-160; done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2k/bench.json 2> gpurun_out/r2k/bench.err; echo bench rc=$?; cat gpurun_out/r2k/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2k/prof -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc 0 > gpurun_out/r2k/prof.log 2>&1; echo prof rc=$?
