set -o pipefail
mkdir -p gpurun_out/px
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pixels.py > gpurun_out/px/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/pixel_probe.py > gpurun_out/px/pixel_probe.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/gpurun_out/px/prof -o px -- python3 tools/pixel_probe.py > gpurun_out/px/prof.log 2>&1 || exit 1
