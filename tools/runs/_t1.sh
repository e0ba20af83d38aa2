set -o pipefail
mkdir -p gpurun_out/t1
PONG_GA_LIB=$PWD/variants/lib_timeline.so timeout -k 10 300 python -u tools/timeline.py --out gpurun_out/t1/timeline.npz > gpurun_out/t1/timeline.log 2>&1 || exit 1
