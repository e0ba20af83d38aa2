set -o pipefail
PMC=1 bash tools/gpu_check.sh r3 || exit 1
timeout -k 10 400 python bench.py --config wide > gpurun_out/r3/bench_wide.json 2> gpurun_out/r3/bench_wide.err || exit 2
