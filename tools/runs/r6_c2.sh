# round 6: the new distributed tests alone first (wide split, sliced hall), then
# the whole -m gpu suite, smoke(), the driver's bench command.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_limits.py tests/test_gpu_replay.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests_new.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
