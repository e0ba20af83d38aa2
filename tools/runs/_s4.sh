set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 400 python -u tools/sweep.py --libs neuro-genetic-pong-self-play_amd/libpong_ga.so,variants/lib_lb1.so,variants/lib_lb4.so,variants/lib_lb8.so --lanes 8 --reps 3 > gpurun_out/s4/sweep.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/sweep.py --lanes 8 --reps 3 --dtype f32 >> gpurun_out/s4/sweep.log 2>&1 || exit 1
