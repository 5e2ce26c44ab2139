#!/bin/bash
# A/B of mass-solve builds on one box: rocprof kernel stats of bench_ops mass_solve (C3, C4), twice each.
#   tools/gpu_mass_ab.sh TAG lib1 lib2 ...   (lib "main" = the in-tree build)
export TMPDIR=/tmp; TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for L in "$@"; do
    if [ $L = main ]; then unset GDM_HIP_LIB; else export GDM_HIP_LIB=dealii-galerkin-difference-methods_amd/lib/ab/$L/libgdm_hip.so; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$L$rep -o ks --output-format csv -- python -u tools/bench_ops.py --configs C3,C4 --ops mass_solve --iters 10 > $O/$L$rep.log 2>&1 || exit 1
    find $O/$L$rep -name "*kernel_stats.csv" -exec cp {} $O/ks_$L$rep.csv \;
    python3 -c "
import csv,json
for r in csv.DictReader(open('$O/ks_$L$rep.csv')):
    if 'mass3' in r['Name']: print('$L$rep', r['Name'][13:40], r['Calls'], round(float(r['AverageNs'])/1e3,1))
for l in open('$O/$L$rep.log'):
    if l.startswith('{'): d=json.loads(l); print('$L$rep', d['config'], d['op'], round(d['ms'],4))
"
  done
done
