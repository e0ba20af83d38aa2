# round 5, call b15: k_prep_records storing each unit pair as it is made
# (prep_rec: 67 VGPRs instead of 372, the same records): the whole -m gpu
# suite, same-box A/Bs against e71743e9 (ab/lib_e717.so) -- the sweep's
# counters must be identical (same records, same games) --, a rocprof kernel
# trace of each library's bench run, then the final measurement of this
# library (tools/runs/r5_final.sh as RUN=r5_final6).  Outcome: prep 150 vs 98 us,
# the bench -2 %: rejected and reverted (the r5_final6 set was not kept)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b15}; mkdir -p $OUT; ROOT=$(pwd)
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
  for L in $P ab/lib_e717.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2 3; do
  for L in $P ab/lib_e717.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$ROOT/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
for L in new old; do
  LIB=$P; [ $L = old ] && LIB=ab/lib_e717.so
  PONG_GA_LIB=$ROOT/$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_$L -o kt -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_prof_$L.json 2> $OUT/prof_$L.err || exit 1
done
RUN=r5_final6 bash tools/runs/r5_final.sh || exit 1
echo done > $OUT/ok
