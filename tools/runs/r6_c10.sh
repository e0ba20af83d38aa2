# round 6: serve_inline's cycles per stage, accumulated per wave (PG_SERVE_STAGES;
# the first probe's per-mark atomics were contending), and served twice.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c10}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum ab/*.so > $OUT/lib_sha.txt
for v in stages twice; do
PONG_GA_LIB=ab/$v.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 uniform > $OUT/${v}_init.log 2>&1 || exit 1
PONG_GA_LIB=ab/$v.so timeout -k 10 300 python3 -u tools/init_probe.py stages 3 normal > $OUT/${v}_normal.log 2>&1 || exit 1
done
echo done > $OUT/ok
# the fixed-horizon instance deciding in its game waves (PG_HORIZON_INLINE):
# its parity tests, then A/B against ab/hsvc (round 5's service wave)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_limits.py -m gpu -x -q -k "horizon" --timeout 300 --timeout-method thread > $OUT/gpu_tests_horizon.log 2>&1 || exit 1
for rep in 1 2; do
  for v in product hsvc; do
    if [ $v = product ]; then L=""; else L=ab/$v.so; fi
    PONG_GA_LIB=$L timeout -k 10 300 python3 -u bench.py --horizon 1000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/horizon_${v}_$rep.json 2>> $OUT/err.log || exit 1
  done
done
echo done2 > $OUT/ok2
