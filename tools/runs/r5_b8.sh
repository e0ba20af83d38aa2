# round 5, call b8: the product with certificate failures decided inside the
# game wave (eight game waves per block), the lone-saturated certificate rule,
# scalar wave flags, actions as paddle moves and the mailbox slots recomputed
# in the rare blocks (common frame 190 VALU, no scratch on it): the whole
# -m gpu suite, same-box A/Bs against the previous product (commit fa5cc2f,
# the service-wave form: ab/lib_fa5.so), the SQ counters of the product
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b8}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_fa5.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2 3; do
  for L in $P ab/lib_fa5.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
bash tools/pmc_sq.sh ${RUN:-r5_b8}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
echo done > $OUT/ok
