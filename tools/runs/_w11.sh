set -o pipefail
mkdir -p gpurun_out/w11
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wide.py > gpurun_out/w11/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wide_probe.py 4096 > gpurun_out/w11/probe_main.log 2>&1 || exit 1
PONG_GA_LIB=$PWD/variants/lib_wideilp.so timeout -k 10 300 python -u tools/wide_probe.py 4096 > gpurun_out/w11/probe_ilp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/w11/bench.json 2> gpurun_out/w11/bench.err || exit 1
