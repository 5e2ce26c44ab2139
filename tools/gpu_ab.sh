#!/bin/bash
# GPU A/B session: parity tests (optional), then bench.py per stencil version.
#   tools/gpu_ab.sh TAG "7 8" [pytest -k expr]
TAG=${1:-ab}; VERS=${2:-"7 8"}; K=${3:-}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest.log 2>&1
  rc=$?; tail -4 $OUT/pytest.log; echo "pytest rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for v in $VERS; do
  # variant tokens: 7, 8, 8n (v8 without the interior-z split)
  unset GDM_NO_ZINT; [ "${v%n}" != "$v" ] && export GDM_NO_ZINT=1
  GDM_STENCIL=${v%n} timeout -k 10 200 python bench.py --steps 20 --warmup 3 --pmc 0 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_v$v.json 2> $OUT/bench_v$v.err || { echo "bench v$v failed"; tail -3 $OUT/bench_v$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/bench_v$v.json'));r=d['roofline'];print('v$v step %.3f ms kernel %.3f ms frac %.3f' % (d['ms_per_step'], r['kernel_ms'], r['frac']))"
done
