# round 5, call b2: the in-situ issue cost of each instruction class in
# k_service (PG_PROBE_EXTRA variants: N extra independent instructions of one
# class per visible frame, the games unchanged) and the service wave's share
# (PG_ABLATE_SLOW: certificate failures decided by the f32 guess, no round
# trip), alternating with the product on the bench workload; plus the parity
# suite on the round's library (horizon slots past the serve table)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5_b2}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_parity.log 2>&1 || exit 1
P=neuro-genetic-pong-self-play_amd/libpong_ga.so
for i in 1 2; do
  for L in $P ab/lib_probe1.so ab/lib_probe2.so ab/lib_probe3.so ab/lib_probe4.so $P ab/lib_probe5.so ab/lib_probe7.so ab/lib_probe9.so ab/lib_noslow.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_probe.log 2>&1 || exit 1
  done
done
echo done > $OUT/ok
