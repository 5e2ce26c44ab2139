#!/bin/bash
# PMC passes of the stencil (one rocprofv3 run per pass, counters within the
# per-block slot limits of MI355X_MICROARCH.md; no tracing domain beside --pmc).
#   tools/pmc_passes.sh TAG "PASS1 COUNTERS" "PASS2 COUNTERS" ...   (bench.py --pmc-child: 3 C3 compute_rhs)
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
i=0
for p in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o pmc -- python bench.py --pmc-child > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $p"
  if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT"
