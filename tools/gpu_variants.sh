#!/bin/bash
# Benchmark p=5 experiment variants (tools/build_variant.sh) on the GPU box:
#   tools/gpu_variants.sh TAG NAME...   (NAME "main" = the in-tree library)
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; mkdir -p $OUT
L=dealii-galerkin-difference-methods_amd/lib
for v in "$@"; do
  if [ "$v" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$PWD/$L/variants/$v/libgdm_hip.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "(ragged and 5) or (cell_loop and 3-5-7) or full_size" > $OUT/pt_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pt_$v.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --pmc 0 --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail -3 $OUT/bench_$v.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/bench_$v.json'));r=d['roofline'];print('$v step %.3f ms kernel %.3f ms frac %.3f' % (d['ms_per_step'], r['kernel_ms'], r['frac']))"
done
