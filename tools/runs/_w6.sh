set -o pipefail
mkdir -p gpurun_out/w7
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/w7/tests.log 2>&1 || exit 1
for v in D2 D3; do
  PONG_GA_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python -u tools/wide_probe.py 4096 >> gpurun_out/w7/probe.log 2>&1 || exit 2
  echo "^^ $v" >> gpurun_out/w7/probe.log
done
