# round 4, call a7: the service-wave batch A/B on the workload that loads the
# service wave (bench.py --dist init: an evolved U[0,1) population, ~16 % of
# forwards fail the f32 certificate): product (batch 4) vs batch 1, alternating;
# then the whole -m gpu suite on the product
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a7}; mkdir -p $OUT; ROOT=$(pwd)
for i in 1 2; do
  for L in neuro-genetic-pong-self-play_amd/libpong_ga.so variants/svc_b1.so; do
    echo "$L" >> $OUT/bench_init_ab.log
    PONG_GA_LIB=$ROOT/$L timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --dist init --no-cpu-baseline >> $OUT/bench_init_ab.log 2> $OUT/err.log || exit 1
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
echo done > $OUT/ok
