# round 5, call b3: k_service's frame bookkeeping against a wave-scalar frame
# counter (no per-frame timeout/total/frames updates, the score-based end and
# total_frames only at points, the top block behind one scalar flag, forwards
# counted per game), the service wave back to one request at a time, the
# horizon fields out of SlowSlot: the whole -m gpu suite, then same-box A/Bs
# against the round-4 kernel headers (ab/lib_r4base.so) -- one launch on the
# sweep workload and the driver's bench command, alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b3}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_r4base.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for L in $P ab/lib_r4base.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/$OUT/scale_prof -o kt -- python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done > $OUT/ok
