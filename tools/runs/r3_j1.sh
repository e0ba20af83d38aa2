# round 3, call j1: re-entry check of the rebuilt library (ABI 7) -- the
# whole -m gpu suite, smoke, the driver's bench command, rocprof stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r3_j1}; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
echo done > $OUT/ok
