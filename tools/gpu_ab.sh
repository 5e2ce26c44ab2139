#!/bin/bash
# A/B of stencil builds on one box: parity (tools/variant_check.py, wall-touching
# meshes vs the oracle's Kronecker form) + compute_rhs timing at a config.
#   tools/gpu_ab.sh TAG CONFIG KIND lib1 lib2 ...   (lib "main" = the in-tree build)
# Stops at the first crash / time-out (rc > 1); a parity failure (rc 1) is reported.
export TMPDIR=/tmp
TAG=$1; CFG=$2; KIND=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
V=dealii-galerkin-difference-methods_amd/lib/ab
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$V/$L/libgdm_hip.so; fi
    timeout -k 10 150 python -u tools/variant_check.py --p ${P:-5} --kind $KIND --config $CFG >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
    rc=$?
    echo "$L rep$rep rc=$rc: $(tail -n 1 $OUT/ab.jsonl)"
    if [ $rc -gt 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
  done
done
exit 0
