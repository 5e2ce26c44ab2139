#!/bin/bash
# bench variants x GDM_ROUNDS values (no tests): tools/gpu_rounds.sh TAG "ROUNDS..." NAME...
TAG=$1; RS=$2; shift 2
export TMPDIR=/tmp; OUT=gpurun_out/$TAG; mkdir -p $OUT
L=dealii-galerkin-difference-methods_amd/lib
for v in "$@"; do for r in $RS; do
  if [ "$v" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$PWD/$L/variants/$v/libgdm_hip.so; fi
  GDM_ROUNDS=$r timeout -k 10 200 python bench.py --steps 20 --warmup 3 --pmc 0 --no-cpu-baseline > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { echo "bench $v failed"; tail -3 $OUT/b_${v}_$r.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/b_${v}_$r.json'));r=d['roofline'];print('$v rounds $r: kernel %.3f ms frac %.3f' % (r['kernel_ms'], r['frac']))"
done; done
