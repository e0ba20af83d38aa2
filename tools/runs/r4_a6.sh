# round 4, call a6: the service wave taking up to 4 posted requests at once
# (fast_f64_decide_batch; PG_SVC_BATCH, product 4) -- the parity suites, then a
# same-box A/B of the product against batch 1 (the previous service loop) and
# batch 2 on the bench workload (N(0,3) genes) and on U[0,1) genes (--dist init)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a6}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_parity.log 2>&1 || exit 1
for i in 1 2; do
  for L in neuro-genetic-pong-self-play_amd/libpong_ga.so variants/svc_b1.so variants/svc_b2.so; do
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 3 >> $OUT/sweep_svc_batch.log 2>&1 || exit 1
    timeout -k 10 300 python -u tools/sweep.py --libs $L --lanes 0 --reps 2 --dist uniform >> $OUT/sweep_svc_batch.log 2>&1 || exit 1
  done
done
echo done > $OUT/ok
