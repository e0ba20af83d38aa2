# round 6: where --dist init's extra k_service time goes: the product with
# the frame bound restored (parity), PG_DECIDE_PROBE (shader cycles inside
# serve_inline until the reload lands vs the waves' total), timing-only
# ablations PG_ABLATE_SERVE (no serve_inline) and PG_ABLATE_SLOW (no rare
# decision path at all), on --dist init and the headline.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c5}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_limits.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for v in product probe noserve noslow; do
  if [ $v = product ]; then L=""; else L=ab/$v.so; fi
  PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --dist init --steps 5 --warmup 2 --no-cpu-baseline > $OUT/init_${v}_1.json 2>> $OUT/err.log || exit 1
  PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/head_${v}_1.json 2>> $OUT/err.log || exit 1
done
echo done > $OUT/ok
