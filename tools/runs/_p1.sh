set -o pipefail
mkdir -p gpurun_out/p1
timeout -k 10 300 python -u tools/ga_profile.py > gpurun_out/p1/profile.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/p1/bench.json 2> gpurun_out/p1/bench.err || exit 2
