set -o pipefail
mkdir -p gpurun_out/x1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pixels.py tests/test_gpu_evolve.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/x1/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/pixel_probe.py > gpurun_out/x1/probe.log 2>&1 || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/x1/prof -o kt --output-format csv -- python3 tools/pixel_probe.py > gpurun_out/x1/prof.log 2>&1 || exit 3
