# round 6: serve_inline without the static-bound plateau rule before the frame
# bound, the f64 stage's bound sums in f32, the horizon instance deciding in
# its game waves: parity + hard cases + horizon on the product; A/B against
# ab/prev (the last commit: PG_K only) on --dist init, the headline, --horizon;
# the per-stage cycles of the new serve path.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c11}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_limits.py tests/test_gpu_blas_order.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in product prev; do
    if [ $v = product ]; then L=""; else L=ab/$v.so; fi
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --dist init --steps 5 --warmup 2 --no-cpu-baseline > $OUT/init_${v}_$rep.json 2>> $OUT/err.log || exit 1
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/head_${v}_$rep.json 2>> $OUT/err.log || exit 1
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --horizon 1000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/horizon_${v}_$rep.json 2>> $OUT/err.log || exit 1
  done
done
PONG_GA_LIB=ab/stages.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 uniform > $OUT/stages_init.log 2>&1 || exit 1
PONG_GA_LIB=ab/stages.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 normal > $OUT/stages_normal.log 2>&1 || exit 1
echo done > $OUT/ok
