# round 3, call b1: the fused generation path (csrc/pg_gen.hip) -- its parity
# tests and the GA suites that now run through it, then the driver's bench
# command and a kernel trace of a short bench for the per-generation gaps
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_b1}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_generation.py tests/test_gpu_evolve.py tests/test_gpu_hof_native.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/$OUT/prof -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
