set -o pipefail
mkdir -p gpurun_out/w2
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/w2/tests.log 2>&1 || exit 1
for v in d2 d3; do PONG_GA_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python -u tools/wide_probe.py 8192 >> gpurun_out/w2/probe.log 2>&1 || exit 2; echo "^^ $v" >> gpurun_out/w2/probe.log; done
