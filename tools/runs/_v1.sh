set -o pipefail
mkdir -p gpurun_out/v1
for v in noskip s128 s256x4 s512x8; do
  PONG_GA_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/v1/bench_$v.json 2> gpurun_out/v1/bench_$v.err || exit 1
done
