set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/s2/parity.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_w2reg.so --lanes 8 --reps 5 > gpurun_out/s2/sweep.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_w2reg.so --lanes 8 --reps 5 --sigma 1 >> gpurun_out/s2/sweep.log 2>&1 || exit 1
