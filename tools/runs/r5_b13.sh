# round 5, call b13: the frame bound computed by the whole wave inside serve_inline
# (frame_bound_wave, from the lane records; b12 computed it in the requesting
# lanes and spilled: 1.08 vs 1.20 ·10^10), ahead of the f64 genome fetch:
# the whole -m gpu suite,
# then same-box A/Bs against the library before it (0a51d667 as ab/lib_0a51.so)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b13}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_0a51.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2 3; do
  for L in $P ab/lib_0a51.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
echo done > $OUT/ok
