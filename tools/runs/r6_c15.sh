# round 6: the hall-of-fame prepare enqueued before the side stream's work
# (evolve.DeviceGA.prepare_first) and the slots uploaded straight into
# hof_slot: the GA / generation / distributed tests on it; A/B of the driver's
# bench command against PG_NO_PREPARE_FIRST=1, alternating, three each.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c15}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_generation.py tests/test_gpu_evolve.py tests/test_gpu_dist.py tests/test_gpu_hof_native.py tests/test_gpu_configs.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_product_$rep.json 2>> $OUT/err.log || exit 1
  PG_NO_PREPARE_FIRST=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_sidefirst_$rep.json 2>> $OUT/err.log || exit 1
done
echo done > $OUT/ok
