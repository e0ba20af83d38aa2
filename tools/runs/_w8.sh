set -o pipefail
mkdir -p gpurun_out/w8
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wide.py > gpurun_out/w8/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wide_probe.py 4096 > gpurun_out/w8/probe_new.log 2>&1 || exit 1
PONG_GA_LIB=$PWD/variants/lib_wideold.so timeout -k 10 300 python -u tools/wide_probe.py 4096 > gpurun_out/w8/probe_old.log 2>&1 || exit 1
