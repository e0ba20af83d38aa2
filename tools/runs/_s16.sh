set -o pipefail
mkdir -p gpurun_out/s16
PONG_GA_LIB=$PWD/variants/lib_s_iterative-ilp.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_ga.py > gpurun_out/s16/parity.log 2>&1 || exit 1
for v in default itilp default itilp; do
  if [ $v = default ]; then L=$PWD/neuro-genetic-pong-self-play_amd/libpong_ga.so; else L=$PWD/variants/lib_s_iterative-ilp.so; fi
  PONG_GA_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline >> gpurun_out/s16/bench_$v.json 2>> gpurun_out/s16/bench_$v.err || exit 1
done
