# per-operator and RK4-step timings at C3 / C4 / C2 (current code)
export TMPDIR=/tmp
OUT=gpurun_out/rk; mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_ops.py --configs C3,C4,C2 --ops apply,mass_solve,rk_step --iters 10 > $OUT/ops.jsonl 2> $OUT/ops.err; rc=$?; cut -c1-220 $OUT/ops.jsonl; exit $rc
