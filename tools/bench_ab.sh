#!/bin/bash
# A/B of whole-library builds on the bench metric (compute_rhs with inflow data
# at C3, bench.py --metric-only), interleaved over two repetitions:
#   tools/bench_ab.sh TAG lib1 lib2 ...   (lib "main" = the in-tree build, else lib/ab/NAME)
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=dealii-galerkin-difference-methods_amd/lib/ab/$L/libgdm_hip.so; fi
    timeout -k 10 200 python -u bench.py --metric-only --steps 40 > "$OUT/$L.$rep.json" 2>> "$OUT/err.log"
    rc=$?
    python3 -c "import json,sys; d=json.load(open('$OUT/$L.$rep.json')); print('$L rep$rep', round(d['ms_per_step'],4), 'ms/step, kernel', round(d['roofline']['kernel_ms'],4), 'ms, frac', round(d['roofline']['frac'],3))" 2>/dev/null || echo "$L rep$rep rc=$rc"
    if [ $rc -gt 1 ]; then exit $rc; fi
  done
done
