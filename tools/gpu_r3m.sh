# templated (whole-line / segmented) mass kernels, 1-chunk segments, deal.II adapter: tests + per-op times
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mass_segments.py tests/test_host_driver.py tests/test_gpu_parity.py tests/test_gpu_spike.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_ops.py --configs C3,C4,C2 --ops apply,mass_solve,rk_step --iters 20 > $OUT/ops.jsonl 2> $OUT/ops.err; rc=$?; echo ops rc=$rc; python3 -c "import json
for l in open('$OUT/ops.jsonl'):
  d=json.loads(l); print(d['config'], d['op'], '%.4f' % d.get('stage_ms', d['ms']))"; [ $rc -eq 0 ] || exit $rc
