# cost of the wall tiles: x / y wall corrections disabled (wrong near the walls, timing only), z-chunk and serial variants
export TMPDIR=/tmp
OUT=gpurun_out/r2w; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3 --ops apply --iters 30 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print('%.4f ms' % d['ms'])"; }
for v in main nox noy noxy main; do
  if [ $v = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$v/libgdm_hip.so; fi
  echo "== $v $(ops)" || exit 1
done
unset GDM_HIP_LIB
echo "== serial $(GDM_SERIAL=1 ops)"
for zc in 128 171 256 512; do echo "== zchunk $zc $(GDM_ZCHUNK=$zc ops)"; done
echo "== noxy serial $(GDM_HIP_LIB=$L/noxy/libgdm_hip.so GDM_SERIAL=1 ops)"
echo "== store pattern"; timeout -k 10 60 ./tools/microbench/store_pattern
