# round 2, session 4, call d1: bench's N > 1 path over RCCL at world size 1,
# the sharded DeviceGA tests, the default bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2_d1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dist.py -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
