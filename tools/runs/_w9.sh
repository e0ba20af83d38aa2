set -o pipefail
mkdir -p gpurun_out/w9
PONG_GA_LIB=$PWD/variants/lib_stamps.so timeout -k 10 300 python -u tools/wide_probe.py 4096 > gpurun_out/w9/probe_stamps.log 2>&1 || exit 1
