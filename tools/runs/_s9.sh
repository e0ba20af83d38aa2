set -o pipefail
mkdir -p gpurun_out/s9
timeout -k 10 400 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_sl8.so,variants/lib_sl32.so,variants/lib_sl127.so,neuro-genetic-pong-self-play_amd/libpong_ga.so --lanes 8 --reps 5 > gpurun_out/s9/sweep.log 2>&1 || exit 1
