# round 4, call a5: sharded variation (pg_ga_args.pair_mask, DeviceGA.shard_vary;
# the game ring reverted) -- the GA tests incl. the sharded ones (2, 3 and 8
# gloo ranks on cuda:0, config 4 at P = 524 288), the parity suite, the
# headline bench and the N = 8 weak-scaling model (tools/scale_model.py)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4_a5}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_generation.py tests/test_gpu_evolve.py -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests_ga.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 700 --timeout-method thread > $OUT/gpu_tests_dist.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 600 python3 -u tools/scale_model.py 8 4 > $OUT/scale_model.log 2>&1 || exit 1
echo done > $OUT/ok
