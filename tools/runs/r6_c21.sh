# round 6: each inline-deciding wave's LDS cache of the last network it served
# (ServeCache, PG_SERVE_CACHE: the frame bound's record inputs and the f64
# stage's genes): parity and hard cases on it; A/B against ab/c820.so (the
# shipped library without it) on --dist init, the headline and --horizon.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c21}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_limits.py tests/test_gpu_blas_order.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in product c820; do
    if [ $v = product ]; then L=""; else L=ab/$v.so; fi
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --dist init --steps 5 --warmup 2 --no-cpu-baseline > $OUT/init_${v}_$rep.json 2>> $OUT/err.log || exit 1
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/head_${v}_$rep.json 2>> $OUT/err.log || exit 1
  done
done
for v in product c820; do
  if [ $v = product ]; then L=""; else L=ab/$v.so; fi
  PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --horizon 1000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/horizon_${v}_1.json 2>> $OUT/err.log || exit 1
done
echo done > $OUT/ok
