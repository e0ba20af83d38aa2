set -o pipefail
mkdir -p gpurun_out/e1
timeout -k 10 600 python -u -m pytest tests/test_gpu_evolve.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/e1/evolve.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/e1/tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/e1/bench.json 2> gpurun_out/e1/bench.err || exit 3
