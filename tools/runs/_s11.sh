set -o pipefail
mkdir -p gpurun_out/s11
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_evolve.py tests/test_gpu_dist.py tests/test_gpu_ga.py > gpurun_out/s11/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s11/bench.json 2> gpurun_out/s11/bench.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s11/bench2.json 2> gpurun_out/s11/bench2.err || exit 1
