# stencil phase breakdown (diag build), C4 (p=7 wave 256^3) PMC passes, bench incl. the C4 leg
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3c; mkdir -p $OUT
GDM_DIAG_BITS=0,8,16,31,63,95,127,32,15,47,3,12,64 timeout -k 10 300 python -u tools/diag_stencil.py > $OUT/diag.txt 2>&1; rc=$?; echo diag rc=$rc; grep dbg $OUT/diag.txt; [ $rc -eq 0 ] || { tail -5 $OUT/diag.txt; exit $rc; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --pmc 0 --steps 20 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo bench rc=$rc; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], d['rk4_stage_ms']); print(json.dumps(d['c4_wave']))"
timeout -k 10 900 bash tools/pmc_stencil.sh r3c/pmc_c4 --n 255 --p 7 --kind wave > $OUT/pmc_c4.txt 2>&1; rc=$?; echo pmc rc=$rc; grep -A30 "stencil8" $OUT/pmc_c4.txt | head -70
