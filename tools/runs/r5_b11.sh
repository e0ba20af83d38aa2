# round 5, call b11: the f64 gap test's plateau widths computed one per lane
# (one exp per lane instead of one per output pair: k_service's VGPR spills
# 69 -> 43, scratch instructions 135 -> 79, all on the f64 decision path):
# the whole -m gpu suite, same-box A/Bs against the previous product
# (ac53a5e8 as ab/lib_ac53.so), then the final measurement of this library
# (tools/runs/r5_final.sh as RUN=r5_final3)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b11}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_ac53.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2 3; do
  for L in $P ab/lib_ac53.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
RUN=r5_final3 bash tools/runs/r5_final.sh || exit 1
echo done > $OUT/ok
