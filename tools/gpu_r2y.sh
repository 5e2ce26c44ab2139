# config 5 with the reference's cut values solved to the reference's tolerance (identity CG, rel 1e-6)
export TMPDIR=/tmp
OUT=gpurun_out/r2y; mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_cut_c5.py --max-it 60000 > $OUT/c5_cut_full.json 2> $OUT/c5_cut_full.err; rc=$?; cat $OUT/c5_cut_full.json; [ $rc -eq 0 ] || { tail $OUT/c5_cut_full.err; exit $rc; }
