#!/bin/bash
# The multi-rank GPU tests (SPIKE, the 8 C3 ranks, the C++ drivers) and two
# runs of the per-rank bench legs: tools/rank_check.sh TAG -> gpurun_out/TAG/
export TMPDIR=/tmp
TAG=${1:-rank}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_spike.py tests/test_gpu_c3_ranks.py tests/test_host_driver.py -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u tools/rank_legs.py 20 >> "$OUT/rank_legs.jsonl" 2>> "$OUT/rank_legs.err" || exit 1
done
python3 - "$OUT/rank_legs.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print("c3 rhs %.4f spike %.4f | c4 stencil %.4f spike %.4f" % (r["c3"]["compute_rhs_ms"], r["c3"]["spike_solve_ms"],
                                                                  r["c4"]["stencil_ms"], r["c4"]["spike_solve_ms"]))
PY
