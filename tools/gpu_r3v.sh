# mass inverse cache-policy A/B (non-temporal loads / stores of the v3 line solves): C3, C4, C2 mass_solve + C3 RK step
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3v; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
for i in 1 2; do
  for v in base ntst ntld ntall; do
    GDM_HIP_LIB=$L/$v/libgdm_hip.so timeout -k 10 240 python -u tools/bench_ops.py --configs C3,C4,C2 --ops mass_solve,rk_step > $OUT/${v}_$i.jsonl 2> $OUT/${v}_$i.err; rc=$?
    echo "== $v $i rc=$rc"; cut -c1-200 $OUT/${v}_$i.jsonl; [ $rc -eq 0 ] || exit $rc
  done
done
