set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/$OUT/prof -o bench -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
