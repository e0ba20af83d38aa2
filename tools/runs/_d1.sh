set -o pipefail
mkdir -p gpurun_out/d1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_replay.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/d1/tests.log 2>&1 || exit 1
