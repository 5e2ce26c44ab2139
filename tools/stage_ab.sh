#!/bin/bash
# A/B of whole-library builds on the C3 RK stage (tools/profile_stage.py:
# AdvectionProblem.step / 4), interleaved over two repetitions:
#   tools/stage_ab.sh TAG lib1 lib2 ...   (lib "main" = the in-tree build, else lib/ab/NAME)
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=dealii-galerkin-difference-methods_amd/lib/ab/$L/libgdm_hip.so; fi
    r=$(timeout -k 10 200 python -u tools/profile_stage.py 2>> "$OUT/err.log"); rc=$?
    echo "$L rep$rep $r" | tee -a "$OUT/stage.txt"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
