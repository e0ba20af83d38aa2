# round 5, call b7: the product's source plus (ab/lib_inline.so) certificate
# failures decided inside the game wave (eight game waves per block, no
# service wave; the weights reloaded from their lane records after a
# decision), the certificate's saturated rule only for a lone maybe-saturated
# output (lane masks, no branches), the wave-uniform flags as scalars, and
# actions kept as the paddles' moves in centroid units (common frame 198 -> 190
# VALU); ab/lib_inline_p3.so: the same with the deciding wave at issue
# priority 3.  The whole -m gpu suite on the inline library, then same-box
# A/Bs against the product
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b7}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
PONG_GA_LIB=$(pwd)/ab/lib_inline.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_inline.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_inline.so ab/lib_inline_p3.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for L in $P ab/lib_inline.so ab/lib_inline_p3.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
echo done > $OUT/ok
