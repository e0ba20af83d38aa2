set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r2/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err || exit 2
timeout -k 10 400 python bench.py --config wide --no-cpu-baseline > gpurun_out/r2/bench_wide.json 2> gpurun_out/r2/bench_wide.err || exit 3
