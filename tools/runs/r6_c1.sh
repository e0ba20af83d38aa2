# round 6, first call: ABI 11 (episode limits), the timeout-after-point fix,
# the config-5 split tests (wide DeviceGA over 1/2/8 gloo ranks, balanced
# shards), the sliced-hall fix: the whole -m gpu suite, smoke(), the driver's
# bench command.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c1}
OUT=gpurun_out/$TAG; mkdir -p $OUT
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
