# round 2, session 4, call d7: longest-lineage-first evaluation order -- GA
# tests, then bench with and without it, alternating
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_d7; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_evolve.py tests/test_gpu_ga.py -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/bench_order_$i.json 2> $OUT/bench_order_$i.err || exit 1
  PG_NO_LENGTH_ORDER=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/bench_noorder_$i.json 2> $OUT/bench_noorder_$i.err || exit 1
done
echo done > $OUT/ok
