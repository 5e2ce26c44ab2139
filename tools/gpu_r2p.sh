# stencil tile / wall variants (p=5 advection-only builds, tools/build_variant.sh): parity + C3 apply timing
export TMPDIR=/tmp
OUT=gpurun_out/r2p; mkdir -p $OUT
L=dealii-galerkin-difference-methods_amd/lib
run() {  # name zchunk
  v=$1; zc=$2
  if [ "$v" = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$PWD/$L/variants/$v/libgdm_hip.so; fi
  if [ "$zc" = "-" ]; then unset GDM_ZCHUNK; else export GDM_ZCHUNK=$zc; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "advection and 5" > $OUT/pt_${v}_$zc.log 2>&1
  rc=$?; echo "$v zc=$zc pytest rc=$rc $(tail -n 1 $OUT/pt_${v}_$zc.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 120 python -u tools/bench_ops.py --configs C3 --ops apply --iters 20 > $OUT/ops_${v}_$zc.json 2>&1 || { echo "ops $v failed"; tail -n 3 $OUT/ops_${v}_$zc.json; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/ops_${v}_$zc.json').read().strip().splitlines()[-1]);print('$v zc=$zc apply %.3f ms frac %.3f' % (d['ms'], d['frac_8TBps']))"
}
run main -
run base -
run noy -
run nox -
run t444 256
run t486 -
run t484 -
run pf3 -
run base 128
