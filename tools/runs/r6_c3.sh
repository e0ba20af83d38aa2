# round 6: the saturated rule before plateau_f32 in k_service's rare block
# (sat_move): parity tests on it; A/B against -DPG_NO_SAT_MOVE on --dist init
# and the headline; the PG_INLINE_LOG classification of the requests that
# reach serve_inline on --dist init (tools/init_probe.py).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so ab/*.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_cases.py tests/test_gpu_limits.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in product nosat; do
    if [ $v = product ]; then L=""; else L=ab/$v.so; fi
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --dist init --steps 5 --warmup 2 --no-cpu-baseline > $OUT/init_${v}_$rep.json 2>> $OUT/err.log || exit 1
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/head_${v}_$rep.json 2>> $OUT/err.log || exit 1
  done
done
PONG_GA_LIB=ab/log.so timeout -k 10 300 python3 -u tools/init_probe.py $OUT/init_probe.npz 3 > $OUT/init_probe.log 2>&1 || exit 1
echo done > $OUT/ok
