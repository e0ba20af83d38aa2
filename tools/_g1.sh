set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/sweep.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 && \
timeout -k 10 600 python tools/sweep.py --lanes 8,16 --reps 3 > gpurun_out/sweep.log 2>&1 && \
PONG_GA_LIB=$PWD/variants/timeline.so timeout -k 10 300 python tools/timeline.py --pop 65536 > gpurun_out/timeline.log 2>&1
