# round 6: the host's two waits per generation poll their events
# (evolve.DeviceGA.spin_wait) and the scan's pinned buffers persist: the
# generation-path GPU tests; A/B of the driver's bench command against
# PG_NO_SPIN=1, alternating, three each; a kernel + HIP runtime trace of the
# product (the host's launch times against the device's gaps).
set -o pipefail
export TMPDIR=/tmp
TAG=${RUN:-r6_c27}
OUT=gpurun_out/$TAG; mkdir -p $OUT; ROOT=$(pwd)
sha256sum neuro-genetic-pong-self-play_amd/libpong_ga.so > $OUT/lib_sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_generation.py tests/test_hof.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_spin_$rep.json 2>> $OUT/err.log || exit 1
  PG_NO_SPIN=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/head_nospin_$rep.json 2>> $OUT/err.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
