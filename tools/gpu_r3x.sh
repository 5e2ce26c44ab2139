# stencil cache-policy A/B (non-temporal output stores / plane DMA), then the whole GPU suite + bench (NT mass default)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3x; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
for i in 1 2 3; do
  for v in sbase sntst sntall; do
    GDM_HIP_LIB=$L/$v/libgdm_hip.so timeout -k 10 240 python -u tools/variant_check.py --p 5 --kind advection --config C3 > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err; rc=$?
    echo "== $v $i rc=$rc $(cut -c1-60 $OUT/${v}_$i.json | head -c 0)$(python3 -c "import json,sys; d=json.load(open('$OUT/${v}_$i.json')); print('%.4f %.3f %s' % (d['ms'], d['frac'], d['parity_ok']))" 2>/dev/null)"; [ $rc -le 1 ] || exit $rc
  done
done
bash tools/gpu_r3w.sh
