# round 6: the pipelined step() (evolve.DeviceGA.pipeline: the next
# generation's evaluation launched once the hall-of-fame update is enqueued,
# before step() returns): the whole -m gpu suite (incl.
# test_pipelined_step_equals_unpipelined); A/B of the driver's bench command
# against PG_NO_PIPELINE=1, alternating, three each; a kernel trace of the product.
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c29}
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd)
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_pipe_$rep.json 2>> $OUT/err.log || exit 1
  PG_NO_PIPELINE=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_nopipe_$rep.json 2>> $OUT/err.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
