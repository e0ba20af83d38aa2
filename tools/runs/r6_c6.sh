# round 6: f64 constants of the decision code materialized at their use
# (PG_K, pg_f64math.h: k_service's scratch instructions 96 -> 24) and k_decide
# in its own translation unit: the parity suites on the product; A/B against
# ab/nok (-DPG_NO_K) on --dist init, the headline and the wide config.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c6}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_limits.py tests/test_gpu_wide.py tests/test_gpu_blas_order.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in product nok; do
    if [ $v = product ]; then L=""; else L=ab/$v.so; fi
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --dist init --steps 5 --warmup 2 --no-cpu-baseline > $OUT/init_${v}_$rep.json 2>> $OUT/err.log || exit 1
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/head_${v}_$rep.json 2>> $OUT/err.log || exit 1
  done
done
for v in product nok; do
  if [ $v = product ]; then L=""; else L=ab/$v.so; fi
  PONG_GA_LIB=$L timeout -k 10 600 python3 -u bench.py --config wide --steps 2 --warmup 1 --no-cpu-baseline > $OUT/wide_${v}.json 2>> $OUT/err.log || exit 1
done
echo done > $OUT/ok
