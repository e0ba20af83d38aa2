# round 5, call b5: call b4 again without the test suite (its A/B baseline lacked an ABI-10 symbol),
# plus the service wave at issue priority 3 (ab/lib_svcprio3.so, -DPG_SVC_PRIO=3):
# table), the half exchange as one DPP move, and the sliced self-play
# schedule (pg_schedule_args.hof_slices: a rank plays its block's slice of the
# hall); the whole -m gpu suite (config 4 over 8 gloo ranks vs one process with
# the sliced schedule included), same-box A/Bs against the round-4 kernel
# headers, the SQ counters of the product, the N = 8 scale model under rocprof;
# f64-stored wide nets on k_wide<4, double> (spill-free)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b5}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
# (the -m gpu suite passed on this library in call b4: profiles/r05/gpu_tests_b4.log)
for i in 1 2 3; do
  for L in $P ab/lib_r4base.so ab/lib_svcprio3.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for L in $P ab/lib_r4base.so ab/lib_svcprio3.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
bash tools/pmc_sq.sh ${RUN:-r5_b5}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/$OUT/scale_prof -o kt -- python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done > $OUT/ok
