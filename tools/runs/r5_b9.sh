# round 5, call b9: the in-wave decision path reloads only the output layer
# of the lane records afterwards (load_rec_out: 13 of 41 16-B pieces; the
# input layer stays in registers without new spills) and the certificate's
# bound counts the packed chain's P = U / 2 roundings instead of U
# (out_roundings: a tighter e, fewer certificate failures): the whole -m gpu
# suite, same-box A/Bs against the previous product (a095280e as
# ab/lib_a095.so), the SQ counters of the product
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b9}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_a095.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2 3; do
  for L in $P ab/lib_a095.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
bash tools/pmc_sq.sh ${RUN:-r5_b9}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
echo done > $OUT/ok
