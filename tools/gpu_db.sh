# double-buffered (A, B) handoff (variant build, p = 5): parity of the p = 5 stencil paths, then A/B timing
export TMPDIR=/tmp
OUT=gpurun_out/db; mkdir -p $OUT
L=$PWD/dealii-galerkin-difference-methods_amd/lib/variants
export GDM_HIP_LIB=$L/${VAR:-db}/libgdm_hip.so
timeout -k 10 150 python -u -c "
import sys, numpy as np, torch
sys.path[:0] = ['dealii-galerkin-difference-methods_amd', 'oracle']
import gdm_amd, oracle as O
a = (1.0, 0.15, -0.05)
n3 = (90, 50, 40)
op = gdm_amd.GdmOperator(3, 5, n3, 0.0, 1.0, 'advection', params=a, device=0)
m = O.Mesh(3, 5, list(n3))
u = np.random.default_rng(0).uniform(-1, 1, m.n_dofs)
M = [m.matrices_1d(d)[0] for d in range(3)]
B = [m.advection_outflow_B(d, a[d]) for d in range(3)]
ref = m.kron_apply([(B[0], M[1], M[2]), (M[0], B[1], M[2]), (M[0], M[1], B[2])], u)
y = op.new_vector(local=False)
op.apply(torch.from_numpy(u).cuda(), y)
torch.cuda.synchronize()
print('quick check rel err %.3e' % (np.linalg.norm(y.cpu().numpy() - ref) / np.linalg.norm(ref)))
" > $OUT/quick.log 2>&1; rc=$?; cat $OUT/quick.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "advection_apply_vs_cell_loop and a0-3-5 or v8" > $OUT/pt.log 2>&1; rc=$?; echo "db parity rc=$rc $(tail -n 1 $OUT/pt.log)"; [ $rc -le 1 ] || exit $rc
ops() { timeout -k 10 120 python -u tools/bench_ops.py --configs C3 --ops apply --iters 30 2>/dev/null | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print('%.4f ms' % d['ms'])"; }
for v in ${VAR:-db} main ${VAR:-db} main; do
  if [ $v = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=$L/$v/libgdm_hip.so; fi
  echo "== stencil $v $(ops)" || exit 1
done
