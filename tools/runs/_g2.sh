set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g2/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/g2/smoke.log 2>&1 || exit 1
