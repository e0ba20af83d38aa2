set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ga.py tests/test_gpu_evolve.py > gpurun_out/s8/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $(pwd)/gpurun_out/s8/prof -o ga -- python3 tools/ga_profile.py 524288 3 > gpurun_out/s8/ga.log 2>&1 || exit 1
