# round 5, call b6: k_service's common frame 222 -> 198 VALU -- the game kept
# in the features' doubled units (PongK: no feature arithmetic; paddles inside
# the clamp band, so no row clamp or centroid clip; one range test for a face;
# the moved ball stored unconditionally), the output bias folded into the
# first lane's partial chains, the certificate returning the action code, the
# rally bounce reported by the step (one compare gating the rare block),
# forwards from the frame counter, the network block run in every lane, the
# loop left at a game end: the whole -m gpu suite (incl. the forward-count
# test), same-box A/Bs against the same source before these trims
# (ab/lib_pretrim.so), the round-4 kernel headers (ab/lib_r4base.so) and the
# trimmed source with the service wave at issue priority 3
# (ab/lib_svcprio3.so); the SQ counters of the product; the N = 8 scale model
# under rocprof
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b6}; mkdir -p $OUT
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
sha256sum $P ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for L in $P ab/lib_pretrim.so ab/lib_r4base.so ab/lib_svcprio3.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_ab.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for L in $P ab/lib_pretrim.so ab/lib_r4base.so ab/lib_svcprio3.so; do
    echo "$L" >> $OUT/bench_ab.log
    PONG_GA_LIB=$(pwd)/$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> $OUT/bench_ab.log 2>> $OUT/bench_ab.err || exit 1
  done
done
bash tools/pmc_sq.sh ${RUN:-r5_b6}/sq 8 || exit 1
python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/$OUT/scale_prof -o kt -- python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done > $OUT/ok
