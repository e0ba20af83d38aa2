set -o pipefail
mkdir -p gpurun_out/r4
for v in default r64s4 r128s4 r128s8 r192s4; do
  if [ $v = default ]; then L=$PWD/neuro-genetic-pong-self-play_amd/libpong_ga.so; else L=$PWD/variants/lib_$v.so; fi
  PONG_GA_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4/bench_$v.json 2> gpurun_out/r4/bench_$v.err || exit 1
done
