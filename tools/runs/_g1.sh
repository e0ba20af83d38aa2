set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 && \
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err
